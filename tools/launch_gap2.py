"""Dev probe 2: host-side blocking of device-pointer launches (default vs side stream)."""
import os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import alipmpc
from alipmpc import scenes
dev = torch.device("cuda", 0)
cfg = alipmpc.default_cfg(0, 3, nc_max=5, ne_max=0)
s = alipmpc.Solver(cfg, 0)
Bs = 65536
bt = scenes.make_batch(Bs, seed=7, n_cir=5, N=3, scenes_per_batch=4096)
n, m = 15, 3 * s.rps
inp = {"x0": torch.from_numpy(bt["x0"]).to(dev), "goal": torch.from_numpy(bt["goal"]).to(dev),
       "leg": torch.from_numpy(bt["leg"].astype(np.int8)).to(dev), "cir": torch.from_numpy(bt["cir"]).to(dev),
       "nc": torch.from_numpy(bt["nc"].astype(np.int32)).to(dev), "u": torch.from_numpy(bt["u0"]).to(dev)}
out = {"f": torch.empty(Bs, dtype=torch.float64, device=dev), "grad": torch.empty((Bs, n), dtype=torch.float64, device=dev),
       "c": torch.empty((Bs, m), dtype=torch.float64, device=dev), "J": torch.empty((Bs, m, n), dtype=torch.float64, device=dev)}
for name, st in (("default", torch.cuda.current_stream(dev)), ("side", torch.cuda.Stream(dev))):
    for _ in range(3):
        s.eval_device(inp, out, stream=st)
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        s.eval_device(inp, out, stream=st)
        ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    print(name, "per-call host ms:", " ".join(f"{1e3*t:.3f}" for t in ts))
# raw torch kernel launches for comparison
x = torch.zeros(1 << 24, device=dev)
torch.cuda.synchronize()
ts = []
for _ in range(10):
    t0 = time.perf_counter(); x.add_(1.0); ts.append(time.perf_counter() - t0)
torch.cuda.synchronize()
print("torch add_ host ms:", " ".join(f"{1e3*t:.3f}" for t in ts))
