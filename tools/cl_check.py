#!/usr/bin/env python3
"""Dev check of alipmpc_closed_loop_batch against oracle.closed_loop_batch: where the first episodes part ways
(tick, statuses, iterates), and the closed-loop rate (episodes x steps x f_cyc solves per second).

  python tools/cl_check.py [--variant 0] [--kick 0.0] [--program 0] [--out gpurun_out/cl.npz] [--rate-batch 65536]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def episodes(C, variant, kick, B=48):
    from alipmpc import scenes
    bt = scenes.make_batch(B, seed=520 + variant + int(kick * 100), n_cir=5)
    x0 = bt["x0"].copy()
    x0[:12, 0:2] = bt["goal"][:12] - (np.array([1.0, 0.8]) if variant == 1 else np.array([0.6, 0.5]))
    leg = bt["leg"].astype(np.int8)
    co = C.default_cfg(variant, 3, nc_max=5, ne_max=0)
    foot0 = C.solve_batch(co, x0, bt["goal"], leg, bt["cir"], bt["nc"], None, None, np.tile(x0, (1, 3)))["foot"][:, :2]
    return bt, x0, foot0, leg, co


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--kick", type=float, default=0.0)
    ap.add_argument("--program", type=int, default=0)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--out", default="")
    ap.add_argument("--rate-batch", type=int, default=0)
    a = ap.parse_args()
    import alipmpc
    import oracle as C
    bt, x0, foot0, leg, co = episodes(C, a.variant, a.kick)
    s = alipmpc.Solver(alipmpc.default_cfg(a.variant, 3, nc_max=5, ne_max=0, program=a.program))
    o = s.closed_loop(x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=a.steps, f_cyc=40, kick=a.kick, seed=7)
    r = C.closed_loop_batch(co, x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=a.steps, f_cyc=40,
                            kick=a.kick, seed=7)
    B = len(x0)
    for b in range(B):
        so, sr = o["status"][b].ravel(), r["status"][b].ravel()
        io, ir = o["iters"][b].ravel(), r["iters"][b].ravel()
        d = np.nonzero((so != sr) | (io != ir))[0]
        ferr = np.nanmax(np.abs(o["foot"][b] - r["foot"][b])) if np.isfinite(r["foot"][b]).any() else 0.0
        if len(d) or ferr > 1e-6:
            t = d[0] if len(d) else -1
            print(f"ep {b:2d}: first differing tick {t} (step {t // 40}, tick {t % 40})"
                  f" dev st/it {so[t]}/{io[t]} oracle {sr[t]}/{ir[t]}  foot err {ferr:.2e}"
                  f"  stg {o['steps_to_goal'][b]} vs {r['steps_to_goal'][b]}")
            print("     dev   ", so[max(t - 3, 0):t + 6], io[max(t - 3, 0):t + 6])
            print("     oracle", sr[max(t - 3, 0):t + 6], ir[max(t - 3, 0):t + 6])
    if a.out:
        np.savez(a.out, **{"dev_" + k: v for k, v in o.items()}, **{"ref_" + k: v for k, v in r.items()})
    if a.rate_batch:
        from alipmpc import scenes
        Bn = a.rate_batch
        bb = scenes.make_batch_vec(Bn, seed=3, n_cir=5, N=3)
        s.closed_loop(bb["x0"][:256], bb["x0"][:256, :2], bb["goal"][:256], bb["leg"][:256], bb["cir"][:256],
                      bb["nc"][:256], steps=1, f_cyc=40)
        t0 = time.time()
        oo = s.closed_loop(bb["x0"], bb["x0"][:, :2], bb["goal"], bb["leg"], bb["cir"], bb["nc"], steps=1, f_cyc=40)
        dt = time.time() - t0
        n = int((oo["status"] > -10).sum())
        print(f"closed loop B={Bn}: {n} solves in {dt:.3f} s = {n / dt / 1e6:.2f} M solves/s (host wall, incl. H2D/D2H)")


if __name__ == "__main__":
    main()
