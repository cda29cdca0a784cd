#!/usr/bin/env python3
"""Dev (r6, GPU box): where a restoration phase spends its cycles — the -DALIP_STAMPS build's per-section timers of
solve_one (slots 0-9, 24) and resto_wave (10-21; 22 / 23 = calls / iterations), on the cfg2 bench batch with IPOPT's
restoration phase and with the substitute.

  python tools/cl_wstamps.py-like build: ALIPMPC_SINGLE_TU=1, extra -DALIP_STAMPS -DALIP_DEV_ONLY_KSM=10
  python tools/resto_stamps.py [devlib/libalipmpc_stamps.so]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["ALIPMPC_LIB"] = os.path.join(ROOT, sys.argv[1] if len(sys.argv) > 1 else "devlib/libalipmpc_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import alipmpc  # noqa: E402
from alipmpc import scenes  # noqa: E402

L = alipmpc.load()
L.alipmpc_dbg_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
MAIN = ["eval", "grad+J^Ty", "err+mu", "sigma/w", "hess+MFMA+K", "chol+solve", "dV+steps+ftb", "linesearch", "exit",
        "update"]
RES = ["entry", "orig check", "coef+J^Ty", "err+mu", "weights", "hess blocks", "MFMA K+rhs", "GJ", "dV+steps+amin",
       "linesearch", "accept", "hand back"]
bt = scenes.make_batch(4096, seed=0, n_cir=5)
for rest in (alipmpc.RESTORATION_IPOPT, alipmpc.RESTORATION_SUBSTITUTE):
    s = alipmpc.Solver(alipmpc.default_cfg(0, nc_max=5, ne_max=0, restoration=rest))
    buf = np.zeros(26, np.uint64)
    s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    L.alipmpc_dbg_stamps(buf.ctypes.data_as(ctypes.c_void_p), 1)
    o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    L.alipmpc_dbg_stamps(buf.ctypes.data_as(ctypes.c_void_p), 1)
    its = int(o["iters"].sum())
    calls, rits = int(buf[22]), int(buf[23])
    main = buf[:10].astype(float)
    print(f"restoration={rest}: kernel {s.last_kernel_ms():.3f} ms, iterations {its}, restoration calls {calls}, "
          f"restoration iterations {rits}; wave cycles per regular iteration {main.sum() / max(1, its - rits):.0f}")
    for n, v in zip(MAIN, main):
        print(f"   {n:14s} {v / max(1, its - rits):10.0f} cyc/iter")
    print(f"   {'resto call':14s} {float(buf[25]) / max(1, calls):10.0f} cyc/call (solve_one's view)")
    print(f"   {'post-resto':14s} {float(buf[24]) / max(1, calls):10.0f} cyc/call")
    if calls:
        r = buf[10:22].astype(float)
        print(f"   restoration: {r.sum() / calls:.0f} cyc/call, {r.sum() / max(1, rits):.0f} cyc per restoration iteration")
        for n, v in zip(RES, r):
            print(f"     {n:14s} {v / calls:10.0f} cyc/call {v / max(1, rits):10.0f} cyc/iter")
