"""Dev: kernel-time sweep over batch size / iteration cap (run on the GPU box)."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import torch
import alipmpc
from alipmpc import scenes

def run(B, max_iter=100, N=3, n_cir=5, n_elp=0, reps=5, variant=0):
    bt = scenes.make_batch(B, seed=0, n_cir=n_cir, n_elp=n_elp, N=N, scenes_per_batch=min(B, 4096))
    cfg = alipmpc.default_cfg(variant, N, nc_max=n_cir, ne_max=n_elp, max_iter=max_iter)
    s = alipmpc.Solver(cfg)
    dev = torch.device("cuda", 0)
    inp = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in bt.items() if v is not None}
    inp["leg"] = inp["leg"].to(torch.int8); inp["nc"] = inp["nc"].to(torch.int32)
    if "ne" in inp: inp["ne"] = inp["ne"].to(torch.int32)
    out = {"u": torch.empty((B, 5 * N), dtype=torch.float64, device=dev),
           "foot": torch.empty((B, 3), dtype=torch.float64, device=dev),
           "status": torch.empty(B, dtype=torch.int32, device=dev),
           "iters": torch.empty(B, dtype=torch.int32, device=dev)}
    ts = []
    for r in range(reps + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); s.solve_device(inp, out); b.record(); torch.cuda.synchronize()
        if r: ts.append(a.elapsed_time(b))
    it = out["iters"].cpu().numpy()
    return dict(B=B, N=N, max_iter=max_iter, ms=float(np.median(ts)), solves_per_s=B / np.median(ts) * 1e3,
                iters_mean=float(it.mean()), iters_max=int(it.max()))

if __name__ == "__main__":
    res = []
    for B in [64, 1024, 4096, 16384, 65536]:
        res.append(run(B))
    for mi in [30, 50, 70]:
        res.append(run(4096, max_iter=mi))
    res.append(run(65536, N=5, n_cir=5, n_elp=5))
    for r in res:
        print(json.dumps(r))
