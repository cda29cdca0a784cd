"""Dev: closed-loop time per tick for several (steps, f_cyc) on the cfg2 episodes (last_kernel_ms / ticks)."""
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
cin = {"x0": inp["x0"], "foot0": out["foot"][:, 0:2].contiguous(), "goal": inp["goal"], "leg": inp["leg"],
       "cir": inp["cir"], "nc": inp["nc"]}
for S, F in [(1, 40), (40, 1), (1, 2), (2, 1), (1, 10), (10, 1), (1, 40)]:
    co = {"status": torch.empty((B, S, F), dtype=torch.int32, device=dev), "iters": torch.empty((B, S, F), dtype=torch.int32, device=dev),
          "steps_to_goal": torch.empty((B,), dtype=torch.int32, device=dev)}
    s.closed_loop_device(cin, co, S, f_cyc=F)
    torch.cuda.synchronize()
    ms = s.last_kernel_ms()
    it = co["iters"].cpu().numpy()
    st = co["status"].cpu().numpy()
    ran = st != -10
    per_tick_it = [int(it[:, a, b][ran[:, a, b]].sum()) for a in range(S) for b in range(F)]
    print(f"S={S:2d} F={F:2d} ticks={S*F:3d} ms={ms:8.2f} ms/tick={ms/(S*F):6.3f} it/tick(first,last)={per_tick_it[0]},{per_tick_it[-1]} "
          f"ran(last)={int(ran[:, -1, -1].sum())}")
