#!/usr/bin/env python3
"""Study (CPU): the cfg2 bench batch (4096 instances, seed 0, bench.scene_block) solved by the numpy
oracle with the build's restoration substitute and with IPOPT's restoration phase (np_oracle._resto): status mix,
iterations, line-search trials (the work a wave spends; the slowest instances set the split launch's phase 2) and how
the restorations ended.

  python tools/resto_batch.py [--B 4096] [--modes substitute,ipopt] [--prox u,p] [--out profiles/r6/resto/cfg2_batch.json]
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import np_oracle as O  # noqa: E402
from alipmpc import scenes  # noqa: E402

BT = None


def _init(B):
    global BT
    BT = scenes.make_batch(B, seed=0, n_cir=5, N=3)


def one(args):
    i, mode, prox = args
    O.RESTO["proximity"] = prox
    cfg = O.default_cfg(0, 3, nc_max=5, ne_max=0)
    pr = O.Problem(cfg, BT["x0"][i], BT["goal"][i], BT["leg"][i], BT["cir"][i][:BT["nc"][i]], np.zeros((0, 5)))
    st = {}
    u, s, it = O.solve_footholds(pr, BT["u0"][i], stats=st, restoration=mode)
    _, p0 = O.plan(pr, u)
    return p0, int(s), int(it), int(st.get("trials", 0)), int(st.get("restorations", 0)), st.get("resto", []), \
        int(st.get("resto_iters", 0))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--modes", default="substitute,ipopt")
    ap.add_argument("--prox", default="u")
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r6", "resto", "cfg2_batch.json"))
    a = ap.parse_args()
    rep = {"B": a.B}
    feet = {}
    with ProcessPoolExecutor(a.jobs, initializer=_init, initargs=(a.B,)) as ex:
        for mode in a.modes.split(","):
            for prox in (a.prox.split(",") if mode == "ipopt" else ["u"]):
                t0 = time.time()
                res = list(ex.map(one, [(i, mode, prox) for i in range(a.B)], chunksize=16))
                key = mode if mode != "ipopt" else f"ipopt_prox_{prox}"
                feet[key] = np.array([r[0] for r in res])
                st = np.array([r[1] for r in res])
                its = np.array([r[2] for r in res])
                tr = np.array([r[3] for r in res])
                rest = {}
                for r in res:
                    for e in r[5]:
                        rest[e] = rest.get(e, 0) + 1
                s2 = st == 2
                rep[key] = {"status": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
                            "mean_iters": float(its.mean()), "max_iters": int(its.max()),
                            "mean_trials": float(tr.mean()), "max_trials": int(tr.max()),
                            "trials_p99": float(np.percentile(tr, 99)),
                            "status2_mean_iters": float(its[s2].mean()) if s2.any() else 0.0,
                            "status2_mean_trials": float(tr[s2].mean()) if s2.any() else 0.0,
                            "line_search_failures": int(sum(r[4] for r in res)), "resto_outcomes": rest,
                            "resto_iters": int(sum(r[6] for r in res)), "s": round(time.time() - t0, 1)}
                print(key, json.dumps(rep[key]), flush=True)
    keys = list(feet)
    for k in keys[1:]:
        d = np.max(np.abs(feet[k] - feet[keys[0]]), axis=1)
        rep[f"{k}_vs_{keys[0]}_feet_within_1e-4"] = float(np.mean(d <= 1e-4))
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(rep, fh, indent=1)


if __name__ == "__main__":
    main()
