#!/usr/bin/env python3
"""Dev diagnostic: where does a closed-loop tick's solve launch spend its time?

  python tools/cl_wstamps.py build          # here (CPU): devlib/libalipmpc_wstamp.so, one TU, -DALIP_WSTAMP
  python tools/cl_wstamps.py run [--out D]  # GPU box: cold cfg2 solve + one closed-loop walking step (f_cyc = 40)

The diagnostic build records, per solved instance, the start / end of its wave on the constant 100 MHz clock, its
HW_ID / XCC_ID (which SIMD), iterations, line-search trials and restorations (alipmpc.hip WSTAMP_*).  Per launch it
prints the span, the dispatch spread (how late the last wave started), duration quantiles and the per-SIMD load, so
late dispatch and long instances piling onto a few SIMDs can be told apart.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd")
sys.path.insert(0, PKG)
LIB = os.path.join(ROOT, "devlib", "libalipmpc_wstamp.so")


def build():
    os.environ["ALIPMPC_SINGLE_TU"] = "1"
    from alipmpc import build as b
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    b.build(force=True, out=LIB, extra=["-DALIP_WSTAMP"])


def simd_key(hw, xcc):
    # gfx9 HW_ID: wave [3:0], simd [5:4], cu [11:8], sh [12], se [15:13]; XCC_ID [3:0]
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    return ((((xcc & 15) * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd


def summarize(rec, active=None, tag=""):
    """rec: (B, 8) records of one launch."""
    ok = rec[:, 1] > 0
    if active is not None:
        ok &= active
    r = rec[ok]
    t0, t1 = r[:, 0].astype(np.int64), r[:, 1].astype(np.int64)
    base = t0.min()
    st, en = (t0 - base) / 100.0, (t1 - base) / 100.0      # microseconds
    dur = en - st
    its, trials, rest = r[:, 5].astype(np.int64), r[:, 6].astype(np.int64), r[:, 7].astype(np.int64)
    hw = (r[:, 4] & 0xFFFFFFFF).astype(np.int64)
    xcc = (r[:, 4] >> 32).astype(np.int64)
    keys = np.array([simd_key(h, x) for h, x in zip(hw, xcc)])
    uk, inv = np.unique(keys, return_inverse=True)
    per_simd_n = np.bincount(inv)
    per_simd_end = np.zeros(len(uk))
    np.maximum.at(per_simd_end, inv, en)
    per_simd_its = np.bincount(inv, weights=its)
    per_simd_tr = np.bincount(inv, weights=trials)
    long_ = its >= 20
    per_simd_long = np.bincount(inv, weights=long_.astype(float))
    q = lambda a: [round(float(x), 1) for x in np.quantile(a, [0, 0.5, 0.9, 0.99, 1.0])]  # noqa: E731
    crit = int(np.argmax(en))
    out = {
        "tag": tag, "instances": int(ok.sum()), "span_us": round(float(en.max()), 1),
        "start_q_us": q(st), "end_q_us": q(en), "dur_q_us": q(dur),
        "iters_sum": int(its.sum()), "iters_q": q(its), "trials_sum": int(trials.sum()), "trials_q": q(trials),
        "rest_sum": int(rest.sum()),
        "us_per_iter_q": q(dur / np.maximum(its, 1)),
        "simds_used": int(len(uk)), "per_simd_n_q": q(per_simd_n), "per_simd_long_max": int(per_simd_long.max()),
        "per_simd_iters_q": q(per_simd_its), "per_simd_trials_q": q(per_simd_tr),
        "critical": {"start_us": round(float(st[crit]), 1), "dur_us": round(float(dur[crit]), 1),
                     "iters": int(its[crit]), "trials": int(trials[crit]), "rest": int(rest[crit]),
                     "simd_n": int(per_simd_n[inv[crit]]), "simd_iters": int(per_simd_its[inv[crit]]),
                     "simd_trials": int(per_simd_tr[inv[crit]])},
        "started_after_100us": int((st > 100).sum()),
    }
    return out


def run(args):
    os.environ["ALIPMPC_LIB"] = LIB
    import torch
    import alipmpc
    from alipmpc import scenes
    L = alipmpc.load()
    L.alipmpc_dbg_wstamps.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    L.alipmpc_dbg_wstamps.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    B, N = 4096, 3
    bt = scenes.make_batch(B, seed=0, n_cir=5, N=N)
    cfg = alipmpc.default_cfg(alipmpc.VARIANT_MODI, N, nc_max=5, ne_max=0, restoration=args.restoration)
    s = alipmpc.Solver(cfg, device=0)
    buf = np.zeros((48 * 4096, 8), np.uint64)
    os.makedirs(args.out, exist_ok=True)

    def grab(slots):
        rc = L.alipmpc_dbg_wstamps(buf.ctypes.data_as(ctypes.c_void_p), slots)
        assert rc == slots, rc
        return buf[:slots].copy()

    res = {"build_id": alipmpc.build_id(), "cold": [], "closed_loop": {}, "split": {}}
    for _ in range(3):
        out = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
        rec = grab(B)
        res["cold"].append(summarize(rec, tag=f"cold {s.last_kernel_ms():.3f} ms"))
        buf[:2 * B] = 0
    print(json.dumps(res["cold"][-1]))
    np.save(os.path.join(args.out, "cold_records.npy"), rec) if os.path.isdir(args.out) else None
    # split launches: phase-1 records in slots [0, B), phase-2 records in [B, 2B)
    for cut in args.cuts:
        os.environ["ALIPMPC_SPLIT_IT"] = str(cut)
        ss = alipmpc.Solver(cfg, device=0)
        for _ in range(3):
            buf[:2 * B] = 0
            ss.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
            rec = grab(2 * B)
        ms = ss.last_kernel_ms()
        p1, p2 = rec[:B], rec[B:]
        n2 = int((p2[:, 1] > 0).sum())
        base = int(p1[p1[:, 1] > 0, 0].min())
        e1 = (int(p1[p1[:, 1] > 0, 1].max()) - base) / 100.0
        s2 = (int(p2[p2[:, 1] > 0, 0].min()) - base) / 100.0 if n2 else None
        e2 = (int(p2[p2[:, 1] > 0, 1].max()) - base) / 100.0 if n2 else None
        r = {"cut": cut, "launch_ms": ms, "phase1_end_us": e1, "phase2_start_us": s2, "phase2_end_us": e2,
             "phase2_instances": n2, "phase1": summarize(p1, tag=f"split {cut} phase 1"),
             "phase2": summarize(p2, tag=f"split {cut} phase 2") if n2 else None}
        res["split"][str(cut)] = r
        os.makedirs(args.out, exist_ok=True)
        np.save(os.path.join(args.out, f"split{cut}_records.npy"), rec)
        print(json.dumps({k: v for k, v in r.items() if k not in ("phase1", "phase2")}))
        print(json.dumps(r["phase1"]))
        print(json.dumps(r["phase2"]))
    os.environ["ALIPMPC_SPLIT_IT"] = "0"
    foot0 = out["foot"][:, 0:2].copy()
    for order in (() if args.no_closed_loop else ("0", "1")):
        os.environ["ALIPMPC_CL_ORDER"] = order
        sc = alipmpc.Solver(cfg, device=0)
        F = 40
        for rep in range(2):
            buf[:] = 0
            o = sc.closed_loop(bt["x0"], foot0, bt["goal"], bt["leg"].astype(np.int8), bt["cir"], bt["nc"],
                               steps=1, f_cyc=F)
            ms = sc.last_kernel_ms()
            rec = grab(F * B).reshape(F, B, 8)
        # per tick and instance: duration (us), iterations, line-search trials (which episodes set each tick's time)
        dur = (rec[:, :, 1].astype(np.int64) - rec[:, :, 0].astype(np.int64)) / 100.0
        np.savez_compressed(os.path.join(args.out, f"cl_order{order}_per_instance.npz"), dur=dur,
                            iters=rec[:, :, 5].astype(np.int32), trials=rec[:, :, 6].astype(np.int32))
        ticks = []
        for i in range(F):
            act = o["status"][:, 0, i] != alipmpc.ROLLOUT_DONE
            sm = summarize(rec[i], act, tag=f"order={order} tick {i}")
            ticks.append(sm)
            if i in (0, 1, 5, 10, 20, 30, 39):
                print(json.dumps(sm))
        res["closed_loop"][order] = {"loop_ms": ms, "ticks": ticks}
        print(f"order={order}: loop {ms:.2f} ms, spans (us):", [t["span_us"] for t in ticks])
    os.makedirs(args.out, exist_ok=True)
    with open(os.path.join(args.out, "wstamps.json"), "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["build", "run"])
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "wst"))
    ap.add_argument("--cuts", type=int, nargs="*", default=[16])
    ap.add_argument("--no-closed-loop", action="store_true")
    ap.add_argument("--restoration", type=int, default=0, help="cfg.restoration (0 IPOPT, 1 substitute)")
    a = ap.parse_args()
    build() if a.what == "build" else run(a)
