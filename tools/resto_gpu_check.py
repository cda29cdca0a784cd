#!/usr/bin/env python3
"""Dev check on the GPU box (r6): the wave program with IPOPT's restoration phase against the C oracle (same
cfg.restoration), for one or more library builds, and the cfg2-shaped launch time of each with both restoration modes.

  python tools/resto_gpu_check.py [lib.so ...]     (default: the in-tree library)
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(lib):
    if lib != "default":
        os.environ["ALIPMPC_LIB"] = os.path.join(ROOT, lib)
    sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import alipmpc
    from alipmpc import scenes
    import oracle as C
    for name, N, nc, ne, B, prec in (("cfg2", 3, 5, 0, 4096, 0), ("n5e", 5, 5, 5, 512, 0), ("cfg2f32", 3, 5, 0, 1024, 1),
                                     ("sig", 3, 4, 0, 512, 0)):
        for rest in (0, 1):
            variant = 1 if name == "sig" else 0
            cfg = alipmpc.default_cfg(variant, N, nc_max=nc, ne_max=ne, restoration=rest, precision=prec)
            s = alipmpc.Solver(cfg)
            bt = scenes.make_batch(B, seed=0 if name == "cfg2" else 3, n_cir=nc, n_elp=ne, N=N)
            elp = bt.get("elp")
            out = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], elp, bt.get("ne"), u0=bt["u0"])
            co = C.default_cfg(variant, N, nc_max=nc, ne_max=ne)
            co.restoration = rest
            if prec:
                co.tol, co.acceptable_tol = cfg.tol if cfg.tol != 1e-8 else 1e-4, 1e-3
            ref = C.solve_batch(co, bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"],
                                elp if elp is not None else np.zeros((B, 0, 5)),
                                bt["ne"] if elp is not None else np.zeros(B), bt["u0"], nthreads=16)
            d = np.max(np.abs(out["foot"] - ref["foot"]), axis=1)
            both = (out["status"] == 0) & (ref["status"] == 0)
            ms = []
            if name == "cfg2":
                dev = torch.device("cuda", 0)
                inp = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in bt.items() if v is not None}
                inp["leg"] = inp["leg"].to(torch.int8)
                inp["nc"] = inp["nc"].to(torch.int32)
                o = {"u": torch.empty((B, 15), dtype=torch.float64, device=dev),
                     "foot": torch.empty((B, 3), dtype=torch.float64, device=dev),
                     "x_pred": torch.empty((B, 3, 5), dtype=torch.float64, device=dev),
                     "status": torch.empty(B, dtype=torch.int32, device=dev),
                     "iters": torch.empty(B, dtype=torch.int32, device=dev)}
                for r in range(23):
                    s.solve_device(inp, o, stream=torch.cuda.current_stream())
                    ms.append(s.last_kernel_ms())
            st_g = {int(k): int(v) for k, v in zip(*np.unique(out["status"], return_counts=True))}
            st_o = {int(k): int(v) for k, v in zip(*np.unique(ref["status"], return_counts=True))}
            print(f"{lib} {name} rest={rest}: status eq {np.mean(out['status'] == ref['status']):.4f} "
                  f"iters eq {np.mean(out['iters'] == ref['iters']):.4f} "
                  f"feet<=1e-4 {np.mean(d <= 1e-4):.4f} (both conv {np.mean(d[both] <= 1e-4) if both.any() else 0:.4f}) "
                  f"gpu {st_g} oracle {st_o} mean it {out['iters'].mean():.2f}/{ref['iters'].mean():.2f}"
                  + (f" ms median {np.median(ms[3:]):.4f}" if ms else ""), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--one":
        one(sys.argv[2])
    else:
        for lib in (sys.argv[1:] or ["default"]):
            subprocess.check_call([sys.executable, __file__, "--one", lib])
