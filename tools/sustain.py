"""Dev: cfg2 solve launches back to back for a sustained period (per-launch HIP events): does the launch time
drift (clocks / power), and how does a warm start from the previous solution change the launch time at an
unchanged iteration sum?"""
import os, sys, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import alipmpc
from alipmpc import scenes
dev = torch.device("cuda", 0)
B = 4096
bt = scenes.make_batch(B, seed=0, n_cir=5, N=3)
s = alipmpc.Solver(alipmpc.default_cfg(0, 3, nc_max=5, ne_max=0))
inp = {k: torch.from_numpy(np.ascontiguousarray(bt[k] if k != "leg" else bt[k].astype(np.int8))).to(dev)
       for k in ("x0", "goal", "leg", "cir", "u0")}
inp["nc"] = torch.from_numpy(bt["nc"].astype(np.int32)).to(dev)
mk = lambda: {"u": torch.empty((B, 15), dtype=torch.float64, device=dev), "foot": torch.empty((B, 3), dtype=torch.float64, device=dev),  # noqa: E731
              "x_pred": torch.empty((B, 3, 5), dtype=torch.float64, device=dev), "status": torch.empty(B, dtype=torch.int32, device=dev),
              "iters": torch.empty(B, dtype=torch.int32, device=dev)}
out = mk()
st = torch.cuda.current_stream()


def run(inp, out, K):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for a, b in ev:
        a.record(st); s.solve_device(inp, out, stream=st); b.record(st)
    torch.cuda.synchronize()
    return np.array([a.elapsed_time(b) for a, b in ev])


d = run(inp, out, 400)
print("cold x400: first10", np.round(d[:10], 3), "mean by 50:", np.round(d.reshape(8, 50).mean(1), 3))
it0 = out["iters"].sum().item()
warm = dict(inp)
warm["u0"] = out["u"].clone()
out2 = mk()
d2 = run(warm, out2, 100)
print("warm (u0 = the solution) x100: mean by 25:", np.round(d2.reshape(4, 25).mean(1), 3), "iters", out2["iters"].sum().item(), "cold iters", it0)
d3 = run(inp, out, 50)
print("cold again x50:", np.round(d3.reshape(2, 25).mean(1), 3))
# chained warm starts (the closed loop's rule: each solve starts from the previous plan), same x0
chain = dict(inp)
chain["u0"] = inp["u0"].clone()
ds, its = [], []
for t in range(40):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st); s.solve_device(chain, out, stream=st); b.record(st)
    torch.cuda.synchronize()
    ds.append(a.elapsed_time(b)); its.append(out["iters"].sum().item())
    chain["u0"].copy_(out["u"])
print("chained warm x40 ms:", np.round(ds, 3))
print("chained warm x40 iters:", its)
# enqueued without host syncs (as alipmpc_closed_loop_batch does): solves alone, then solves interleaved with a
# tiny kernel that uses no scratch (the closed loop's project / update kernels stand in)
tiny = torch.zeros(4096, dtype=torch.float64, device=dev)
for inter in (False, True, False):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(40)]
    for a, b in ev:
        if inter:
            tiny.add_(1.0)
        a.record(st); s.solve_device(inp, out, stream=st); b.record(st)
        if inter:
            tiny.mul_(0.5)
    torch.cuda.synchronize()
    print("interleaved" if inter else "alone      ", np.round([a.elapsed_time(b) for a, b in ev], 2))
