#!/usr/bin/env python3
"""Dev: where the sweep kernel and eval_kernel (ALIPMPC_EVAL_KERNEL=group) differ on one case of
tests/test_gpu.py::test_sweep_kernel_bit_identical_to_group_eval (variant, circles, B)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))


def main(variant=1, nc=6, B=2048):
    import alipmpc
    from alipmpc import scenes
    bt = scenes.make_batch_vec(B, seed=23 + nc, n_cir=max(nc, 1), N=3)
    cir = np.ascontiguousarray(bt["cir"][:, :nc]) if nc else np.zeros((B, 0, 3))
    rng = np.random.default_rng(5)
    ncnt = np.where(rng.random(B) < 0.3, rng.integers(0, nc + 1, B), np.clip(bt["nc"], 0, nc)).astype(np.int32)
    u = bt["u0"] + 0.05 * rng.standard_normal(bt["u0"].shape)
    cfg = alipmpc.default_cfg(variant, 3, nc_max=nc, ne_max=0)
    outs = []
    for kern in ("sweep", "group"):
        if kern == "group":
            os.environ["ALIPMPC_EVAL_KERNEL"] = "group"
        s = alipmpc.Solver(cfg)
        outs.append(s.eval(bt["x0"], bt["goal"], bt["leg"], cir, ncnt, None, None, u))
    a, g = outs
    for k in a:
        if a[k] is None:
            continue
        d = a[k] != g[k]
        if d.any():
            rows = np.nonzero(d.reshape(B, -1).any(1))[0]
            print(k, "differs in", len(rows), "instances, e.g.", rows[:8], "max abs", np.abs(a[k] - g[k]).max())
            for b in rows[:3]:
                print("  b", b, "goal sweep", a["goal_eff"][b], "group", g["goal_eff"][b], "goal in", bt["goal"][b],
                      "detour", not np.array_equal(a["goal_eff"][b], bt["goal"][b]))
                print("   ", k, a[k][b].ravel()[:6], g[k][b].ravel()[:6])
        else:
            print(k, "equal")


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
