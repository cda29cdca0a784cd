"""Dev: per-tick iteration / status profile of the closed loop on the cfg2 episodes (what makes late ticks slow)."""
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
out = {"u": torch.empty((B, 15), dtype=torch.float64, device=dev), "foot": torch.empty((B, 3), dtype=torch.float64, device=dev),
       "x_pred": torch.empty((B, 3, 5), dtype=torch.float64, device=dev), "status": torch.empty(B, dtype=torch.int32, device=dev),
       "iters": torch.empty(B, dtype=torch.int32, device=dev)}
s.solve_device(inp, out)
torch.cuda.synchronize()
F = 40
cin = {"x0": inp["x0"], "foot0": out["foot"][:, 0:2].contiguous(), "goal": inp["goal"], "leg": inp["leg"],
       "cir": inp["cir"], "nc": inp["nc"]}
co = {"status": torch.empty((B, 1, F), dtype=torch.int32, device=dev), "iters": torch.empty((B, 1, F), dtype=torch.int32, device=dev),
      "steps_to_goal": torch.empty((B,), dtype=torch.int32, device=dev)}
s.closed_loop_device(cin, co, 1, f_cyc=F)
torch.cuda.synchronize()
st = co["status"].cpu().numpy()[:, 0, :]
it = co["iters"].cpu().numpy()[:, 0, :]
for i in range(F):
    r = st[:, i] != -10
    print(f"tick {i:2d} ran {r.sum():5d} mean_it {it[r, i].mean():5.2f} n>=25 {(it[r, i] >= 25).sum():4d} "
          f"st2 {(st[r, i] == 2).sum():4d} st-1 {(st[r, i] == -1).sum():4d} sum_it {it[r, i].sum():6d}")
