"""Dev probe: where does the gap between HIP-event launch time and rocprof kernel time come from?"""
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
for Bs, what in ((65536, "eval"), (4096, "solve")):
    bt = scenes.make_batch(Bs, seed=7, n_cir=5, N=3, scenes_per_batch=4096)
    n, m = 15, 3 * s.rps
    inp = {"x0": torch.from_numpy(bt["x0"]).to(dev), "goal": torch.from_numpy(bt["goal"]).to(dev),
           "leg": torch.from_numpy(bt["leg"].astype(np.int8)).to(dev), "cir": torch.from_numpy(bt["cir"]).to(dev),
           "nc": torch.from_numpy(bt["nc"].astype(np.int32)).to(dev), "u": torch.from_numpy(bt["u0"]).to(dev),
           "u0": torch.from_numpy(bt["u0"]).to(dev)}
    if what == "eval":
        out = {"f": torch.empty(Bs, dtype=torch.float64, device=dev), "grad": torch.empty((Bs, n), dtype=torch.float64, device=dev),
               "c": torch.empty((Bs, m), dtype=torch.float64, device=dev), "J": torch.empty((Bs, m, n), dtype=torch.float64, device=dev)}
        call = lambda st: s.eval_device(inp, out, stream=st)
    else:
        out = {"u": torch.empty((Bs, 15), dtype=torch.float64, device=dev), "foot": torch.empty((Bs, 3), dtype=torch.float64, device=dev),
               "x_pred": torch.empty((Bs, 3, 5), dtype=torch.float64, device=dev), "status": torch.empty(Bs, dtype=torch.int32, device=dev),
               "iters": torch.empty(Bs, dtype=torch.int32, device=dev)}
        call = lambda st: s.solve_device(inp, out, stream=st)
    st = torch.cuda.current_stream(dev)
    for _ in range(3):
        call(st)
    torch.cuda.synchronize()
    K = 20
    t0 = time.perf_counter()
    for _ in range(K):
        call(st)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(K):
        call(st)
    b.record(st)
    torch.cuda.synchronize()
    print(f"{what}: host enqueue {1e3*(t1-t0)/K:.3f} ms/launch, wall {1e3*(t2-t0)/K:.3f} ms/launch, "
          f"one event pair {a.elapsed_time(b)/K:.3f} ms/launch, lib events last {s.last_kernel_ms():.3f} ms")
