"""Dev: the sweep kernel's output hash and time per launch shape (ALIPMPC_SWEEP_SHAPE: 641 = 64 instances per wave,
1 wave per workgroup; 322; 164).  Run once per shape (the shape is read once per process); the hashes must agree."""
import hashlib, os, sys, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import alipmpc
from alipmpc import scenes
dev = torch.device("cuda", 0)
Bs = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
cfg = alipmpc.default_cfg(0, 3, nc_max=5, ne_max=0)
s = alipmpc.Solver(cfg)
bt = scenes.make_batch_vec(Bs, seed=7, n_cir=5, N=3, fields=4096)
n, m = 15, 3 * s.rps
inp = {"x0": torch.from_numpy(bt["x0"]).to(dev), "goal": torch.from_numpy(bt["goal"]).to(dev),
       "leg": torch.from_numpy(bt["leg"].astype(np.int8)).to(dev), "cir": torch.from_numpy(bt["cir"]).to(dev),
       "nc": torch.from_numpy(bt["nc"].astype(np.int32)).to(dev), "u": torch.from_numpy(bt["u0"]).to(dev)}
full = {"f": torch.empty(Bs, dtype=torch.float64, device=dev), "grad": torch.empty((Bs, n), dtype=torch.float64, device=dev),
        "c": torch.empty((Bs, m), dtype=torch.float64, device=dev), "J": torch.empty((Bs, m, n), dtype=torch.float64, device=dev)}
st = torch.cuda.current_stream()
for _ in range(3):
    s.eval_device(inp, full, stream=st)
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
for a, b in ev:
    a.record(st); s.eval_device(inp, full, stream=st); b.record(st)
torch.cuda.synchronize()
ms = float(np.mean([a.elapsed_time(b) for a, b in ev[1:]]))
h = hashlib.sha1()
for k in ("f", "grad", "c", "J"):
    h.update(full[k].cpu().numpy().tobytes())
print(f"shape {os.environ.get('ALIPMPC_SWEEP_SHAPE', 'default')} B {Bs} {ms:.4f} ms {Bs * 4272 / (ms * 1e-3) / 1e9:.0f} GB/s "
      f"hash {h.hexdigest()[:16]}")
