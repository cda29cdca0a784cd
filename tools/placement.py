"""Dev: launch time of the cfg2 batch vs the placement of its long instances (instance b runs on wave b: workgroup
b // 4, whose 4 waves sit on the 4 SIMDs of one CU).  The long instances (>= 25 iterations, from a first solve)
are put one per workgroup (spread), packed into the first workgroups (packed), or left where they are."""
import os, sys, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import alipmpc
from alipmpc import scenes
dev = torch.device("cuda", 0)
B = 4096
bt = scenes.make_batch(B, seed=0, n_cir=5, N=3)
s = alipmpc.Solver(alipmpc.default_cfg(0, 3, nc_max=5, ne_max=0))
keys = ("x0", "goal", "leg", "cir", "nc", "u0")
def tens(perm):
    d = {k: np.ascontiguousarray(bt[k][perm]) for k in keys}
    d["leg"] = d["leg"].astype(np.int8); d["nc"] = d["nc"].astype(np.int32)
    return {k: torch.from_numpy(v).to(dev) for k, v in d.items()}
out = {"u": torch.empty((B, 15), dtype=torch.float64, device=dev), "foot": torch.empty((B, 3), dtype=torch.float64, device=dev),
       "x_pred": torch.empty((B, 3, 5), dtype=torch.float64, device=dev), "status": torch.empty(B, dtype=torch.int32, device=dev),
       "iters": torch.empty(B, dtype=torch.int32, device=dev)}
st = torch.cuda.current_stream()
def timeit(inp, K=20):
    for _ in range(3): s.solve_device(inp, out, stream=st)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(K): s.solve_device(inp, out, stream=st)
    b.record(st); torch.cuda.synchronize()
    return a.elapsed_time(b) / K
ident = np.arange(B)
base = timeit(tens(ident))
its = out["iters"].cpu().numpy().copy()
for thr in (25, 20, 16):
    longi = np.where(its >= thr)[0]; short = np.where(its < thr)[0]
    # spread: long instance k at wave 4 * (k * (B // 4) // len(longi)) (one per workgroup, evenly over the grid)
    perm = np.empty(B, np.int64); slots = np.zeros(B, bool)
    wg = (np.arange(len(longi)) * (B // 4)) // max(1, len(longi))
    pos = 4 * wg + (np.arange(len(longi)) % 4)   # rotate the SIMD too
    perm[pos] = longi; slots[pos] = True
    perm[~slots] = short
    sp = timeit(tens(perm))
    assert int(out["iters"].sum()) == int(its.sum())
    packed = np.concatenate([longi, short])
    pk = timeit(tens(packed))
    print(f"long >= {thr}: {len(longi)} instances; as generated {base:.3f} ms, spread {sp:.3f} ms, packed {pk:.3f} ms")
