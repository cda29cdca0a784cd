"""Dev: closed-loop outputs with the episodes in groups on streams of their own (ALIPMPC_CL_GROUPS) vs one group, on a
batch with stops, kicks and infeasible scenes (bit identity), under ALIPMPC_LIB.  python tools/groups_check.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import alipmpc
from alipmpc import scenes

for variant, kick in ((0, 0.0), (1, 0.05)):
    B, S, F = 3000, 2, 40
    bt = scenes.make_batch(B, seed=610 + variant, n_cir=5)
    x0 = bt["x0"].copy()
    x0[:300, 0:2] = bt["goal"][:300] - np.array([0.6, 0.5])
    leg = bt["leg"].astype(np.int8)
    cfg = alipmpc.default_cfg(variant, 3, nc_max=5, ne_max=0)
    foot0 = alipmpc.Solver(cfg).solve(x0, bt["goal"], leg, bt["cir"], bt["nc"], u0=np.tile(x0, (1, 3)))["foot"][:, 0:2]
    ref = None
    for grp in ("1", "2", "4", "8", "3"):
        os.environ["ALIPMPC_CL_GROUPS"] = grp
        o = alipmpc.Solver(cfg).closed_loop(x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=S, f_cyc=F, kick=kick,
                                            seed=3)
        ref = o if ref is None else ref
        bad = {k: int((o[k] != ref[k]).reshape(B, -1).any(axis=1).sum()) if o[k].dtype.kind != "f" else
               int((~np.isclose(o[k], ref[k], rtol=0, atol=0, equal_nan=True)).reshape(B, -1).any(axis=1).sum())
               for k in ref}
        print(f"variant {variant} kick {kick} groups {grp}: episodes differing {bad}", flush=True)
