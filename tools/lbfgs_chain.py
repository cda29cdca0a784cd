#!/usr/bin/env python3
"""Study (CPU): does IPOPT's limited-memory Hessian — the mode cyipopt ran, since LIP_Prob has no
`hessian` (MPC_LIP_modi.py:394-655) — reproduce more of the 640 recorded cyipopt calls of sup_learn than the exact
Hessian the build uses?

The calls are replayed as the chain the reference ran (logger_iml.py:333-342: each call warm-started from the previous
call's plan x_mpc_tar, [x_nex] x 3 on the first) through the numpy oracle (oracle/np_oracle.py) in the reference's own
decision space u (n = 15, where a quasi-Newton method is not invariant to the parametrisation), with:
  exact_p      the build's algorithm (exact Hessian, foothold space, split f_en) — the reference count of the test suite
  lbfgs_u      L-BFGS (history 6) in u, the reference's kinked f_en row (IPOPT as cyipopt ran it)
  lbfgs_u_split  L-BFGS in u with the smooth split f_en rows
and the cold-start ([x_nex] x 3) form of each.  Counts footholds within 1e-4 / 1e-6 of the recorded ones.

  python tools/lbfgs_chain.py [--out profiles/r4/sup_learn/lbfgs_chain.json] [--max-iter 30] [--rows 640]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import np_oracle as O  # noqa: E402


def run(mode, d, max_iter, rows, chain):
    cfg = O.default_cfg(0, 3, nc_max=6, ne_max=0, max_iter=max_iter)
    goal = np.array([10.0, 10.0])
    K = O.Consts(cfg)
    feet = np.zeros((rows, 3))
    st = np.zeros(rows, np.int32)
    its = np.zeros(rows, np.int32)
    u_prev = None
    for i in range(rows):
        x0 = d["x_nex"][i]
        pr = O.Problem(cfg, x0, goal, d["leg"][i], d["cir_safe"], np.zeros((0, 5)), K=K)
        u0 = d["u0"][i] if (not chain or u_prev is None) else u_prev
        if mode == "exact_p":
            u, s, it = O.solve_footholds(pr, u0, max_iter=max_iter)
        elif mode == "lbfgs_u":
            u, s, it = O.solve(pr, u0, max_iter=max_iter, lbfgs=6)
        else:
            u, s, it = O.solve(pr.split_copy(), u0, max_iter=max_iter, lbfgs=6)
        X, p0 = O.plan(pr, u)
        feet[i], st[i], its[i] = p0, s, it
        u_prev = X.ravel()
    err = np.max(np.abs(feet[:, :2] - d["foot_logged"][:rows]), axis=1)
    return {"reproduced_1e-4": int((err <= 1e-4).sum()), "reproduced_1e-6": int((err <= 1e-6).sum()),
            "status": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
            "mean_iters": float(its.mean()), "err": err}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r4", "sup_learn", "lbfgs_chain.json"))
    ap.add_argument("--max-iter", type=int, default=30)
    ap.add_argument("--rows", type=int, default=640)
    ap.add_argument("--modes", default="exact_p,lbfgs_u,lbfgs_u_split")
    a = ap.parse_args()
    d = dict(np.load(os.path.join(ROOT, "tests", "golden", "g3_sup_learn.npz")))
    rep = {"rows": a.rows, "max_iter": a.max_iter, "history": 6}
    errs = {}
    for mode in a.modes.split(","):
        for chain in (True, False):
            t0 = time.time()
            r = run(mode, d, a.max_iter, a.rows, chain)
            key = f"{mode}_{'chain' if chain else 'cold'}"
            errs[key] = r.pop("err")
            r["s"] = round(time.time() - t0, 1)
            rep[key] = r
            print(key, r, flush=True)
    # rows the exact-Hessian chain misses that an L-BFGS chain reproduces, and the reverse
    if "exact_p_chain" in errs:
        base = errs["exact_p_chain"] <= 1e-4
        for k, e in errs.items():
            if k != "exact_p_chain":
                rep[f"{k}_vs_exact_chain"] = {"gained": int(((e <= 1e-4) & ~base).sum()),
                                              "lost": int((~(e <= 1e-4) & base).sum())}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(rep, fh, indent=1)
    print(json.dumps(rep))


if __name__ == "__main__":
    main()
