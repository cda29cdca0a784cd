#!/usr/bin/env python3
"""Dev check: the closed loop of tests/test_gpu.py::test_closed_loop_matches_oracle driven from the host
(oracle.closed_loop_batch's driver), every tick's solve sent to BOTH the GPU program and the C oracle on the same
inputs — so kernel / oracle differences are told apart from the drift of two loops.  Saves the inputs of every tick
whose status or iteration count differs (npz, for a CPU replay through the numpy oracle).

  python tools/cl_same_inputs.py [--variant 0] [--kick 0.0] [--program 0] [--prec 0] [--out gpurun_out/same]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--kick", type=float, default=0.0)
    ap.add_argument("--program", type=int, default=0)
    ap.add_argument("--prec", type=int, default=0)
    ap.add_argument("--out", default="gpurun_out/same")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    import alipmpc
    import oracle as C
    from alipmpc import scenes
    B, S, F = 48, 4, 40
    v = a.variant
    bt = scenes.make_batch(B, seed=520 + v + int(a.kick * 100), n_cir=5)
    x0 = bt["x0"].copy()
    x0[:12, 0:2] = bt["goal"][:12] - (np.array([1.0, 0.8]) if v == 1 else np.array([0.6, 0.5]))
    leg = bt["leg"].astype(np.int8)
    co = C.default_cfg(v, 3, nc_max=5, ne_max=0)
    foot0 = C.solve_batch(co, x0, bt["goal"], leg, bt["cir"], bt["nc"], None, None, np.tile(x0, (1, 3)))["foot"][:, :2]
    kw = dict(precision=alipmpc.PREC_FP32) if a.prec else {}
    s = alipmpc.Solver(alipmpc.default_cfg(v, 3, nc_max=5, ne_max=0, program=a.program, **kw))
    c = s.cfg
    cc = C.default_cfg(v, 3, nc_max=5, ne_max=0, tol=c.tol, acceptable_tol=c.acceptable_tol)
    orig = C.solve_batch
    rec = {k: [] for k in ("x0", "goal", "leg", "cir", "nc", "u0", "gst", "git", "ost", "oit", "ferr")}
    n_tot = [0]

    def solve(cfg, x0_, goal, leg_, cir, nc, elp, ne, u0, nthreads=1):
        r = s.solve(x0_, goal, leg_, cir, nc, u0=u0)
        r["restorations"] = np.zeros(len(x0_), np.int32)
        ro = orig(cc, x0_, goal, leg_, cir, nc, None, None, u0, nthreads=8)
        n_tot[0] += len(x0_)
        m = (r["status"] != ro["status"]) | (r["iters"] != ro["iters"])
        if m.any():
            for k, val in (("x0", x0_), ("goal", goal), ("leg", leg_), ("cir", cir), ("nc", nc), ("u0", u0),
                           ("gst", r["status"]), ("git", r["iters"]), ("ost", ro["status"]), ("oit", ro["iters"]),
                           ("ferr", np.abs(r["foot"] - ro["foot"]).max(-1))):
                rec[k].append(np.asarray(val)[m])
        return ro   # the loop follows the oracle's path: every tick's inputs are the oracle loop's
    C.solve_batch = solve
    C.closed_loop_batch(co, x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=S, f_cyc=F, kick=a.kick, seed=7)
    C.solve_batch = orig
    R = {k: np.concatenate(v_) for k, v_ in rec.items() if v_}
    nd = len(R["gst"]) if R else 0
    rep = {"solves": n_tot[0], "differ": nd}
    if nd:
        st_diff = R["gst"] != R["ost"]
        rep.update(status_differ=int(st_diff.sum()), iters_differ_by_1=int((np.abs(R["git"] - R["oit"]) == 1).sum()),
                   pairs={f"{g}/{o}": int(((R["gst"] == g) & (R["ost"] == o)).sum())
                          for g, o in sorted(set(zip(R["gst"].tolist(), R["ost"].tolist())))})
        np.savez(os.path.join(a.out, f"differ_{v}_{a.kick}_{a.program}_{a.prec}.npz"), **R)
    print(json.dumps(rep))


if __name__ == "__main__":
    main()
