import sys, os, numpy as np
R=os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, R+"/mujoco-lip-mpc-simulation_amd"); sys.path.insert(0, R+"/oracle")
import alipmpc, oracle as C
g=np.load(R+"/tests/golden/g2_setup_modi.npz")
B=len(g["m"])
s=alipmpc.Solver(alipmpc.default_cfg(0))
o=s.eval(g["x0"], g["goal"], g["leg"], g["cir"], g["nc"], g["elp"], g["ne"], np.tile(g["x0"], (1, 3)))
for t in range(B):
    if not np.allclose(o["goal_eff"][t], g["goal_eff"][t], atol=1e-12):
        print(t, "gpu", o["goal_eff"][t], "ref", g["goal_eff"][t], "goal", g["goal"][t], "x0", g["x0"][t][:2], "nc", g["nc"][t], "sel", g["sel_cir"][t])
        print("   cir", g["cir"][t][:g["nc"][t]].tolist())
