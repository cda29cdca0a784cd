"""Dev (GPU box): fp32 solve kernel vs fp64 on the cfg2 workload.

For each fp32 tolerance: status counts, mean/max iterations, kernel time, foothold agreement with the fp64
solve, and the "feasible fraction" of SURVEY 8d cfg5 — the share of instances whose solution u, evaluated by
the fp64 eval kernel (the reference callbacks), violates no active row by more than 1e-4.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import torch  # noqa: E402

import alipmpc  # noqa: E402
from alipmpc import scenes  # noqa: E402


def violation(ev):
    c, cl, cu, act = ev["c"], ev["cl"], ev["cu"], ev["row_active"].astype(bool)
    v = np.maximum(np.maximum(cl - c, c - cu), 0.0)
    v[~act] = 0.0
    return v.max(axis=1)


def timed_solve(s, bt, B, N, reps=5):
    dev = torch.device("cuda", 0)
    inp = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in bt.items() if v is not None}
    inp["leg"] = inp["leg"].to(torch.int8)
    inp["nc"] = inp["nc"].to(torch.int32)
    if "ne" in inp:
        inp["ne"] = inp["ne"].to(torch.int32)
    out = {"u": torch.empty((B, 5 * N), dtype=torch.float64, device=dev),
           "foot": torch.empty((B, 3), dtype=torch.float64, device=dev),
           "status": torch.empty(B, dtype=torch.int32, device=dev),
           "iters": torch.empty(B, dtype=torch.int32, device=dev)}
    ts = []
    for r in range(reps + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        s.solve_device(inp, out)
        b.record()
        torch.cuda.synchronize()
        if r:
            ts.append(a.elapsed_time(b))
    return {k: v.cpu().numpy() for k, v in out.items()}, float(np.median(ts))


def main(B=4096, N=3, n_elp=0, max_iter=30, tols=((1e-4, 1e-3), (3e-5, 1e-3), (1e-5, 1e-4), (1e-6, 1e-4))):
    bt = scenes.make_batch_vec(B, seed=0, n_cir=5, n_elp=n_elp, N=N, fields=min(B, 1024))
    kw = dict(nc_max=5, ne_max=n_elp, max_iter=max_iter)
    base = alipmpc.default_cfg(0, N, **kw)
    s64 = alipmpc.Solver(base)
    o64, ms64 = timed_solve(s64, bt, B, N)
    ev = s64.eval(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], bt["elp"], bt["ne"], u=o64["u"],
                  want_J=False)
    v64 = violation(ev)
    print(json.dumps(dict(prec="fp64", N=N, n_elp=n_elp, max_iter=max_iter, tol=base.tol, ms=ms64, iters_mean=float(o64["iters"].mean()),
                          status={int(k): int(c) for k, c in zip(*np.unique(o64["status"], return_counts=True))},
                          feasible=float(np.mean(v64 <= 1e-4)))))
    ok64 = o64["status"] == 0
    for tol, acc in tols:
        cfg = alipmpc.default_cfg(0, N, precision=alipmpc.PREC_FP32, tol=tol, acceptable_tol=acc, **kw)
        s32 = alipmpc.Solver(cfg)
        o32, ms32 = timed_solve(s32, bt, B, N)
        ev = s64.eval(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], bt["elp"], bt["ne"], u=o32["u"],
                      want_J=False)
        v32 = violation(ev)
        both = ok64 & (o32["status"] == 0)
        err = np.abs(o32["foot"] - o64["foot"]).max(axis=1)
        print(json.dumps(dict(
            prec="fp32", tol=tol, ms=ms32, speedup=ms64 / ms32, iters_mean=float(o32["iters"].mean()),
            iters_max=int(o32["iters"].max()),
            status={int(k): int(c) for k, c in zip(*np.unique(o32["status"], return_counts=True))},
            feasible=float(np.mean(v32 <= 1e-4)), both_ok=int(both.sum()),
            foot_err_p50=float(np.median(err[both])) if both.any() else None,
            foot_err_p99=float(np.quantile(err[both], 0.99)) if both.any() else None,
            within_1e3=float(np.mean(err[both] <= 1e-3)) if both.any() else None,
            within_1e4=float(np.mean(err[both] <= 1e-4)) if both.any() else None)))


if __name__ == "__main__":
    main()
    main(B=4096, N=5, n_elp=5, max_iter=100, tols=((1e-3, 1e-2), (3e-4, 3e-3), (1e-4, 1e-3)))
