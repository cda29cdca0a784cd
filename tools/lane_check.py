#!/usr/bin/env python3
"""Dev check of the lane solver (csrc/lane_solve.inc) against the per-wave solve_kernel and the C oracle:
statuses / footholds on a seeded batch, and launch times at a few batch sizes.

  python tools/lane_check.py [--prec 32|64] [--batch B] [--sizes 4096,262144,1048576]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def solver(alipmpc, lane, prec, variant=0, nc=5, **kw):
    extra = {"precision": alipmpc.PREC_FP32} if prec == 32 else {}
    prog = alipmpc.PROGRAM_LANE if lane else alipmpc.PROGRAM_WAVE
    return alipmpc.Solver(alipmpc.default_cfg(variant, 3, nc_max=nc, ne_max=0, program=prog, **extra, **kw))


def timed(s, inp, out, reps=5):
    import torch
    st = torch.cuda.current_stream()
    s.solve_device(inp, out, stream=st)
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        s.solve_device(inp, out, stream=st)
        ms.append(s.last_kernel_ms())
    return float(np.median(ms))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", type=int, default=32)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--sizes", default="4096,65536,262144,1048576")
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--nc", type=int, default=5)
    a = ap.parse_args()
    import torch
    import alipmpc
    from alipmpc import scenes
    import oracle as C
    sl = solver(alipmpc, True, a.prec, a.variant, a.nc)
    sw = solver(alipmpc, False, a.prec, a.variant, a.nc)
    print("programs:", sl.solve_program(), "|", sw.solve_program(), "| lane slots", sl.solve_slots(), flush=True)
    bt = scenes.make_batch_vec(a.batch, seed=5, n_cir=a.nc, N=3)
    t0 = time.time()
    ol = sl.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    print(f"lane solve {time.time() - t0:.2f}s", flush=True)
    ow = sw.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    co = C.default_cfg(a.variant, 3, nc_max=a.nc, ne_max=0)
    m = min(a.batch, 1024)
    ref = C.solve_batch(co, bt["x0"][:m], bt["goal"][:m], bt["leg"][:m], bt["cir"][:m], bt["nc"][:m], None, None,
                        bt["u0"][:m], nthreads=8)
    cnt = lambda st: dict(zip(*np.unique(st, return_counts=True)))  # noqa: E731
    print("status lane", cnt(ol["status"]), "wave", cnt(ow["status"]), "oracle[:m]", cnt(ref["status"]))
    print("iters lane mean %.2f max %d | wave mean %.2f" % (ol["iters"].mean(), ol["iters"].max(), ow["iters"].mean()))
    tol = 1e-3 if a.prec == 32 else 1e-4
    for name, o in (("lane", ol), ("wave", ow)):
        both = (o["status"][:m] == 0) & (ref["status"] == 0)
        err = np.abs(o["foot"][:m] - ref["foot"]).max(1)
        print(f"{name} vs oracle: both-converged {both.mean():.3f}  foot within {tol:g}: {np.mean(err[both] <= tol):.4f}"
              f"  same status {np.mean(o['status'][:m] == ref['status']):.3f}  finite {np.isfinite(o['u']).all()}")
    both = (ol["status"] == 0) & (ow["status"] == 0)
    err = np.abs(ol["foot"] - ow["foot"]).max(1)
    print(f"lane vs wave: both {both.mean():.3f} within {tol:g}: {np.mean(err[both] <= tol):.4f}")
    dev = torch.device("cuda", 0)
    for B in [int(x) for x in a.sizes.split(",") if x]:
        bb = scenes.make_batch_vec(B, seed=0, n_cir=a.nc, N=3)
        inp = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in bb.items() if v is not None}
        inp["leg"] = inp["leg"].to(torch.int8)
        inp["nc"] = inp["nc"].to(torch.int32)
        out = {"u": torch.empty((B, 15), dtype=torch.float64, device=dev),
               "foot": torch.empty((B, 3), dtype=torch.float64, device=dev),
               "x_pred": torch.empty((B, 3, 5), dtype=torch.float64, device=dev),
               "status": torch.empty(B, dtype=torch.int32, device=dev),
               "iters": torch.empty(B, dtype=torch.int32, device=dev)}
        tl = timed(sl, inp, out)
        it_l = out["iters"].float().mean().item()
        tw = timed(sw, inp, out)
        print(f"B={B:8d}  lane {tl:8.3f} ms ({B / tl / 1e3:8.2f} M/s, iters {it_l:.2f})   wave {tw:8.3f} ms "
              f"({B / tw / 1e3:8.2f} M/s)   x{tw / tl:.2f}", flush=True)


if __name__ == "__main__":
    main()
