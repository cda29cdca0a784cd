#!/usr/bin/env python3
"""One device-pointer solve launch at a given batch (profiling target for rocprofv3 --pmc / --kernel-trace).
  python tools/lane_prof.py [--prec 32|64] [--batch B] [--reps R] [--wave]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", type=int, default=64)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--nc", type=int, default=5)
    ap.add_argument("--wave", action="store_true", help="the per-wave solve_kernel (cfg.program = PROGRAM_WAVE)")
    a = ap.parse_args()
    import torch
    import alipmpc
    from alipmpc import scenes
    extra = {"precision": alipmpc.PREC_FP32} if a.prec == 32 else {}
    prog = alipmpc.PROGRAM_WAVE if a.wave else alipmpc.PROGRAM_LANE
    s = alipmpc.Solver(alipmpc.default_cfg(0, 3, nc_max=a.nc, ne_max=0, program=prog, **extra))
    B = a.batch
    bb = scenes.make_batch_vec(B, seed=0, n_cir=a.nc, N=3)
    dev = torch.device("cuda", 0)
    inp = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in bb.items() if v is not None}
    inp["leg"] = inp["leg"].to(torch.int8)
    inp["nc"] = inp["nc"].to(torch.int32)
    out = {"u": torch.empty((B, 15), dtype=torch.float64, device=dev),
           "foot": torch.empty((B, 3), dtype=torch.float64, device=dev),
           "x_pred": torch.empty((B, 3, 5), dtype=torch.float64, device=dev),
           "status": torch.empty(B, dtype=torch.int32, device=dev),
           "iters": torch.empty(B, dtype=torch.int32, device=dev)}
    for _ in range(a.reps):
        s.solve_device(inp, out)
        print(s.solve_program(), "B", B, "ms", round(s.last_kernel_ms(), 3), "iters", out["iters"].sum().item(), flush=True)


if __name__ == "__main__":
    main()
