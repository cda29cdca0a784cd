import os, sys, time
import numpy as np
sys.path.insert(0, "mujoco-lip-mpc-simulation_amd")
import alipmpc
from alipmpc import scenes
variant, kick, B, prec = 0, 0.0, 4096, 1
S, F = 2, 40
bt = scenes.make_batch(B, seed=710 + variant + 3 * prec, n_cir=5)
x0 = bt["x0"].copy()
x0[:300, 0:2] = bt["goal"][:300] - np.array([0.6, 0.5])
leg = bt["leg"].astype(np.int8)
cfg = alipmpc.default_cfg(variant, 3, nc_max=5, ne_max=0, precision=alipmpc.PREC_FP32)
s0 = alipmpc.Solver(cfg)
foot0 = s0.solve(x0, bt["goal"], leg, bt["cir"], bt["nc"], u0=np.tile(x0, (1, 3)))["foot"][:, 0:2]
for cut, tr, grp in (("0", "0", "1"), ("16", "40", "4"), ("3", "0", "3"), ("8", "5", "1"), ("0", "0", "4")):
    os.environ["ALIPMPC_CL_SPLIT_IT"] = cut; os.environ["ALIPMPC_CL_SPLIT_TR"] = tr; os.environ["ALIPMPC_CL_GROUPS"] = grp
    t0 = time.time()
    o = alipmpc.Solver(cfg).closed_loop(x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=S, f_cyc=F, kick=kick, seed=3)
    print(cut, tr, grp, "%.2f s" % (time.time() - t0), flush=True)
