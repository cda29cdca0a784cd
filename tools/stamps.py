"""Dev: per-phase cycle breakdown of solve_kernel from the -DALIP_STAMPS build (GPU box)."""
import os, sys, ctypes
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["ALIPMPC_LIB"] = os.path.join(ROOT, sys.argv[1] if len(sys.argv) > 1 else "devlib/libalipmpc_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import alipmpc
from alipmpc import scenes
L = alipmpc.load()
L.alipmpc_dbg_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
names = ["eval", "grad+J^Ty", "err+mu", "sigma/w", "hess+MFMA+K", "chol+solve", "dV+steps+ftb", "linesearch", "exit", "update"]
for B in [64, 4096]:
    bt = scenes.make_batch(B, seed=0, n_cir=5)
    s = alipmpc.Solver(alipmpc.default_cfg(0, nc_max=5, ne_max=0))
    buf = np.zeros(10, np.uint64)
    s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    L.alipmpc_dbg_stamps(buf.ctypes.data_as(ctypes.c_void_p), 1)
    o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    L.alipmpc_dbg_stamps(buf.ctypes.data_as(ctypes.c_void_p), 1)
    its = o["iters"].sum()
    tot = buf.sum()
    print(f"B={B} kernel {s.last_kernel_ms():.3f} ms, iterations {its}, cycles/iter (wave) {tot/its:.0f}")
    for n, v in zip(names, buf):
        print(f"   {n:14s} {v/its:10.0f} cyc/iter  {100*v/tot:5.1f}%")
