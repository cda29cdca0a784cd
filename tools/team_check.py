"""Dev: closed-loop outputs under several split / team settings vs the one-phase loop (bit identity), to localise a
mismatch.  python tools/team_check.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import alipmpc
from alipmpc import scenes

B, S, F = 3000, 2, 40
bt = scenes.make_batch(B, seed=610, n_cir=5)
x0 = bt["x0"].copy()
x0[:300, 0:2] = bt["goal"][:300] - np.array([0.6, 0.5])
leg = bt["leg"].astype(np.int8)
cfg = alipmpc.default_cfg(0, 3, nc_max=5, ne_max=0)
foot0 = alipmpc.Solver(cfg).solve(x0, bt["goal"], leg, bt["cir"], bt["nc"], u0=np.tile(x0, (1, 3)))["foot"][:, 0:2]
ref = None
for cut, tr, grp in (("0", "0", "1"), ("16", "40", "1"), ("0", "0", "4"), ("16", "40", "4"), ("16", "40", "2"), ("0", "12", "8")):
    os.environ["ALIPMPC_CL_SPLIT_IT"], os.environ["ALIPMPC_CL_SPLIT_TR"], os.environ["ALIPMPC_CL_GROUPS"] = cut, tr, grp
    o = alipmpc.Solver(cfg).closed_loop(x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=S, f_cyc=F, seed=3)
    if ref is None:
        ref = o
    bad = {k: int((~np.isclose(o[k], ref[k], rtol=0, atol=0, equal_nan=True)).reshape(B, -1).any(axis=1).sum())
           for k in ref}
    first = None
    if bad["foot"]:
        d = (o["foot"] != ref["foot"]).reshape(B, -1).any(axis=1)
        first = int(np.argmax(d))
    print(f"cut {cut} tr {tr} groups {grp}: episodes differing per output {bad} first {first}", flush=True)
