#!/usr/bin/env python3
"""Study (CPU): does IPOPT's feasibility restoration phase (np_oracle._resto, restoration="ipopt")
reproduce more of the 640 recorded cyipopt calls of sup_learn than the build's restoration substitute?

The calls are replayed as the chain the reference ran (logger_iml.py:333-342: each call warm-started from the previous
call's plan x_mpc_tar, [x_nex] x 3 on the first) and cold ([x_nex] x 3), through the numpy oracle in foothold space
(the build's algorithm, exact Hessian) with either restoration mode, at the reference cap max_iter 30.  Per row it
records the foothold error against the recorded one, the status, the number of line-search failures and how the
restorations ended; the misses of the substitute chain are classified by status and restoration count, and the 81
status-2 rows get the objective and violation of both modes' returned points.

  python tools/resto_chain.py [--out profiles/r6/resto/resto_chain.json] [--rows 640] [--jobs 8]
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
import np_oracle as O  # noqa: E402

D = dict(np.load(os.path.join(ROOT, "tests", "golden", "g3_sup_learn.npz")))
GOAL = np.array([10.0, 10.0])


def one(i, u0, mode, max_iter):
    cfg = O.default_cfg(0, 3, nc_max=6, ne_max=0, max_iter=max_iter)
    pr = O.Problem(cfg, D["x_nex"][i], GOAL, D["leg"][i], D["cir_safe"], np.zeros((0, 5)))
    st = {}
    u, s, it = O.solve_footholds(pr, u0, max_iter=max_iter, stats=st, restoration=mode)
    X, p0 = O.plan(pr, u)
    c = pr.constraints(u)
    hl, hu = np.isfinite(pr.cl), np.isfinite(pr.cu)
    viol = float(np.max(np.concatenate([[0.0], (pr.cl - c)[hl], (c - pr.cu)[hu]])))
    return dict(foot=p0, u_next=X.ravel(), status=int(s), iters=int(it), rest=int(st.get("restorations", 0)),
                resto=st.get("resto", []), resto_iters=int(st.get("resto_iters", 0)), f=float(pr.objective(u)), viol=viol)


def run_chain(mode, rows, max_iter):
    out, u_prev = [], None
    for i in range(rows):
        u0 = D["u0"][i] if u_prev is None else u_prev
        r = one(i, u0, mode, max_iter)
        out.append(r)
        u_prev = r["u_next"]
    return out


def run_cold(mode, rows, max_iter, jobs):
    with ProcessPoolExecutor(jobs) as ex:
        return list(ex.map(one, range(rows), [D["u0"][i] for i in range(rows)], [mode] * rows, [max_iter] * rows))


def summary(res, rows):
    feet = np.array([r["foot"] for r in res])
    err = np.max(np.abs(feet[:, :2] - D["foot_logged"][:rows]), axis=1)
    st = np.array([r["status"] for r in res])
    resto = {}
    for r in res:
        for e in r["resto"]:
            resto[e] = resto.get(e, 0) + 1
    return err, {"reproduced_1e-4": int((err <= 1e-4).sum()), "reproduced_1e-6": int((err <= 1e-6).sum()),
                 "status": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
                 "mean_iters": float(np.mean([r["iters"] for r in res])),
                 "line_search_failures": int(sum(r["rest"] for r in res)), "resto_outcomes": resto,
                 "resto_iters": int(sum(r["resto_iters"] for r in res))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r6", "resto", "resto_chain.json"))
    ap.add_argument("--rows", type=int, default=640)
    ap.add_argument("--max-iter", type=int, default=30)
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--modes", default="substitute,ipopt")
    a = ap.parse_args()
    rep = {"rows": a.rows, "max_iter": a.max_iter, "resto": O.RESTO}
    res = {}
    for mode in a.modes.split(","):
        for form in ("chain", "cold"):
            t0 = time.time()
            r = run_chain(mode, a.rows, a.max_iter) if form == "chain" else run_cold(mode, a.rows, a.max_iter, a.jobs)
            key = f"{mode}_{form}"
            res[key] = r
            err, sm = summary(r, a.rows)
            res[key + "_err"] = err
            sm["s"] = round(time.time() - t0, 1)
            rep[key] = sm
            print(key, json.dumps(sm), flush=True)
    if "substitute_chain" in res and "ipopt_chain" in res:
        for form in ("chain", "cold"):
            e0, e1 = res[f"substitute_{form}_err"], res[f"ipopt_{form}_err"]
            rep[f"ipopt_vs_substitute_{form}"] = {"gained": int(((e1 <= 1e-4) & ~(e0 <= 1e-4)).sum()),
                                                  "lost": int((~(e1 <= 1e-4) & (e0 <= 1e-4)).sum())}
        # the substitute chain's misses by status and line-search failure count
        sub = res["substitute_chain"]
        miss = np.where(res["substitute_chain_err"] > 1e-4)[0]
        cls = {}
        for i in miss:
            k = f"status {sub[i]['status']}, {min(sub[i]['rest'], 6)} failures" if sub[i]['rest'] else \
                f"status {sub[i]['status']}, no failure"
            d = cls.setdefault(k, {"rows": 0, "ipopt_reproduces": 0})
            d["rows"] += 1
            d["ipopt_reproduces"] += int(res["ipopt_chain_err"][i] <= 1e-4)
        rep["substitute_chain_misses"] = cls
        # the rows either chain ends with status 2: objective and violation of both modes' points
        ip = res["ipopt_chain"]
        s2 = [i for i in range(a.rows) if sub[i]["status"] == 2 or ip[i]["status"] == 2]
        rep["status2_rows"] = [{"row": int(i), "sub": [sub[i]["status"], round(sub[i]["f"], 6), sub[i]["viol"],
                                                       float(res["substitute_chain_err"][i])],
                                "ipopt": [ip[i]["status"], round(ip[i]["f"], 6), ip[i]["viol"],
                                          float(res["ipopt_chain_err"][i])]} for i in s2]
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(rep, fh, indent=1)
    print(json.dumps({k: v for k, v in rep.items() if k != "status2_rows"}, indent=1))


if __name__ == "__main__":
    main()
