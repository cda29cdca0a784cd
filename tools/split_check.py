"""Dev: split-launch bit identity per cut (ALIPMPC_SPLIT_IT) — which instances differ from the one-phase launch."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import alipmpc
from alipmpc import scenes
prec = int(sys.argv[1]) if len(sys.argv) > 1 else 1
B = 4000
bt = scenes.make_batch_vec(B, seed=900 + 3 + 0 + 7 * prec, n_cir=5, n_elp=0, N=3)
kw = dict(nc_max=5, ne_max=0)
if prec:
    kw["precision"] = alipmpc.PREC_FP32
cfg = alipmpc.default_cfg(0, 3, **kw)
def run(k):
    os.environ["ALIPMPC_SPLIT_IT"] = str(k)
    s = alipmpc.Solver(cfg)
    return s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
ref = run(0)
again = run(0)
print("one-phase repeat identical:", all(np.array_equal(ref[k], again[k]) for k in ref))
for k in (1, 2, 3, 5, 7, 10, 16, 25, 29):
    o = run(k)
    d = np.nonzero(np.any(o["u"] != ref["u"], axis=1) | (o["iters"] != ref["iters"]) | (o["status"] != ref["status"]))[0]
    print(f"cut {k}: {len(d)} differ; ran past the cut {(ref['iters'] > k).sum()}; differing iters "
          f"{np.unique(ref['iters'][d])[:10]}; max |du| {np.abs(o['u'] - ref['u']).max():.3e}")
