"""Dev: DD (unicycle) solve-kernel timing.   python tools/dd_bench.py [B] [N] [n_cir] [n_elp]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import alipmpc  # noqa: E402
from alipmpc import scenes  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
N = int(sys.argv[2]) if len(sys.argv) > 2 else 3
nc = int(sys.argv[3]) if len(sys.argv) > 3 else 5
ne = int(sys.argv[4]) if len(sys.argv) > 4 else 0
bt = scenes.make_batch_vec(B, seed=5, n_cir=nc, n_elp=ne, N=N)
rng = np.random.default_rng(6)
x0 = np.ascontiguousarray(np.stack([bt["x0"][:, 0], bt["x0"][:, 1], bt["x0"][:, 4]], 1))
lu = np.ascontiguousarray(np.stack([rng.uniform(0.45, 0.75, B), rng.uniform(-0.15, 0.15, B)], 1))
s = alipmpc.Solver(alipmpc.default_cfg(2, N, nc_max=nc, ne_max=ne))
ms = []
for r in range(6):
    o = s.solve(x0, bt["goal"], None, bt["cir"], bt["nc"], bt.get("elp") if ne else None, bt.get("ne") if ne else None,
                u0=np.tile(lu, (1, N)), last_u=lu)
    ms.append(s.last_kernel_ms())
k = float(np.mean(ms[1:]))
print(json.dumps({"B": B, "N": N, "nc": nc, "ne": ne, "kernel_ms": k, "solves_per_s": B / k * 1e3,
                  "mean_iters": float(o["iters"].mean()), "status0": float((o["status"] == 0).mean())}))
