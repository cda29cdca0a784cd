#!/usr/bin/env python3
"""Dev: the bench's closed loop (cfg2 episodes, f_cyc = 40, one walking step; bench.closed_loop_rate) under several
closed-loop launch settings, each on a fresh Solver in this process.  A setting is IT,TR,G = ALIPMPC_CL_SPLIT_IT,
ALIPMPC_CL_SPLIT_TR, ALIPMPC_CL_GROUPS.  Prints ms per loop (HIP events, the second of two loops) and status counts.

  python tools/cl_params.py 16,40,2 12,40,2 16,30,2 16,40,3
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import alipmpc  # noqa: E402


def main(settings, reps=2):
    dev = torch.device("cuda", 0)
    cfg = alipmpc.default_cfg(alipmpc.VARIANT_MODI, 3, nc_max=5, ne_max=0)
    B = 4096
    bt = bench.global_inputs("cfg2", 0, B, B, 0, 5, 0, 3)
    inp = {"x0": torch.from_numpy(bt["x0"]).to(dev), "goal": torch.from_numpy(bt["goal"]).to(dev),
           "leg": torch.from_numpy(bt["leg"].astype(np.int8)).to(dev), "cir": torch.from_numpy(bt["cir"]).to(dev),
           "nc": torch.from_numpy(bt["nc"].astype(np.int32)).to(dev), "u0": torch.from_numpy(bt["u0"]).to(dev)}
    out = {"u": torch.empty((B, 15), dtype=torch.float64, device=dev),
           "foot": torch.empty((B, 3), dtype=torch.float64, device=dev),
           "x_pred": torch.empty((B, 3, 5), dtype=torch.float64, device=dev),
           "status": torch.empty((B,), dtype=torch.int32, device=dev),
           "iters": torch.empty((B,), dtype=torch.int32, device=dev)}
    alipmpc.Solver(cfg, device=0).solve_device(inp, out)
    torch.cuda.synchronize(dev)
    for s in settings:
        it, tr, g = s.split(",")
        os.environ["ALIPMPC_CL_SPLIT_IT"], os.environ["ALIPMPC_CL_SPLIT_TR"], os.environ["ALIPMPC_CL_GROUPS"] = it, tr, g
        solver = alipmpc.Solver(cfg, device=0)
        ms = []
        for _ in range(reps):
            r = bench.closed_loop_rate(solver, inp, out, 1, dev)
            ms.append(r["ms"])
        print(s, "ms", " ".join("%.2f" % x for x in ms), "M tick-solves/s %.2f" % (r["ticks"] / min(ms) / 1e3),
              r["status_counts"], flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or ["16,40,2"])
