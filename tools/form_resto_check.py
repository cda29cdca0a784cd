#!/usr/bin/env python3
"""Dev (r6, GPU box): the cfg2 batch with IPOPT's restoration phase through each launch form of the wave program —
split (lean phase 1 + restoration-capable phase 2), one-phase one-wave-per-instance (ALIPMPC_SPLIT_IT=0), and the
work queue (the batch twice: B > the resident slots) — bits compared between forms and statuses against the C oracle."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(form):
    env = dict(os.environ)
    if form == "onephase":
        env["ALIPMPC_SPLIT_IT"] = "0"
    out = os.path.join(ROOT, "gpurun_out", f"form_{form}.npz")
    subprocess.check_call([sys.executable, __file__, "--one", form, out], env=env)
    return dict(np.load(out))


def one(form, out):
    sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
    import alipmpc
    from alipmpc import scenes
    bt = scenes.make_batch(4096, seed=0, n_cir=5)
    s = alipmpc.Solver(alipmpc.default_cfg(0, nc_max=5, ne_max=0))
    if form == "queue":
        idx = np.concatenate([np.arange(4096), np.arange(4096)])
        bt = {k: (v[idx] if v is not None else None) for k, v in bt.items()}
    o = s.solve(bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], u0=bt["u0"])
    np.savez(out, **{k: v[:4096] for k, v in o.items()})


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        one(sys.argv[2], sys.argv[3])
        sys.exit(0)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
    import oracle as C
    from alipmpc import scenes
    bt = scenes.make_batch(4096, seed=0, n_cir=5)
    ref = C.solve_batch(C.default_cfg(0, 3, nc_max=5, ne_max=0), bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"],
                        None, None, bt["u0"], nthreads=16)
    res = {f: run(f) for f in ("split", "onephase", "queue")}
    for f, o in res.items():
        d = np.abs(o["foot"] - ref["foot"]).max(1)
        print(f, "status eq oracle %.4f" % np.mean(o["status"] == ref["status"]), "feet<=1e-6 %.4f" % np.mean(d <= 1e-6),
              "bit-equal to split: u %.4f" % np.mean(np.all(o["u"] == res["split"]["u"], axis=1)), flush=True)
