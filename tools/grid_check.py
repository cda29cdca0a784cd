"""Dev: cfg2 solve time vs persistent-grid size (ALIP_GRID workgroups, -DALIP_DEV_GRID build)."""
import os, sys, subprocess, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 2:
    os.environ["ALIPMPC_LIB"] = os.path.join(ROOT, sys.argv[1])
    sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
    import alipmpc
    from alipmpc import scenes
    s = alipmpc.Solver(alipmpc.default_cfg(0, nc_max=5, ne_max=0))
    bt = scenes.make_batch(4096, seed=0, n_cir=5)
    ms = []
    for r in range(6):
        o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"]); ms.append(s.last_kernel_ms())
    print(f"grid {os.environ.get('ALIP_GRID')}: {np.median(ms[1:]):.3f} ms  (min {min(ms[1:]):.3f})  iters {o['iters'].mean():.2f}", flush=True)
else:
    for g in ["0", "1024", "896", "768", "640", "512"]:
        subprocess.check_call([sys.executable, __file__, sys.argv[1], "x"], env=dict(os.environ, ALIP_GRID=g))
