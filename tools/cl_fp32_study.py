#!/usr/bin/env python3
"""Dev study: the fp32 lane closed loop's extra iteration-cap / acceptable stops.

  python tools/cl_fp32_study.py [--out gpurun_out/fp32cl] [--tag base] [--no-oracle]

The episodes of tests/test_gpu.py::test_closed_loop_step_failures_vs_oracle (4096 x one walking step of 40 ticks,
a quarter started within a metre of the goal).
1. alipmpc_closed_loop_batch on the lane program fp32 and fp64: status counts.
2. The C oracle's closed loop at the fp64 tolerances (tol 1e-8) AND at the fp32 program's (tol 1e-4, acceptable 1e-3):
   the same-tolerance comparator separates tolerance effects from precision effects.
3. A host-driven loop (oracle.closed_loop_batch's driver, every tick's solve on the GPU fp32 lane program) that also
   solves every tick's exact inputs with the C oracle at the fp32 tolerances: per-solve status / iterations on the same
   inputs (no path drift), with the tick's distance to the goal, saved as npz for classification on the CPU.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def counts(st):
    ran = st != -10
    u, c = np.unique(st[ran], return_counts=True)
    return {str(int(k)): int(v) for k, v in zip(u, c)}


def episodes(B=4096):
    from alipmpc import scenes
    bt = scenes.make_batch_vec(B, seed=4242, n_cir=5, N=3)
    rng = np.random.default_rng(4243)
    near = np.arange(B) % 4 == 0
    ang = rng.uniform(np.pi, 1.5 * np.pi, near.sum())
    rad = rng.uniform(0.2, 1.0, near.sum())
    bt["x0"] = bt["x0"].copy()
    bt["x0"][near, 0:2] = bt["goal"][near] + np.stack([rad * np.cos(ang), rad * np.sin(ang)], 1)
    bt["near"] = near
    return bt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/fp32cl")
    ap.add_argument("--tag", default="base")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--no-oracle", action="store_true")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    import alipmpc
    import oracle as C

    bt = episodes()
    B = len(bt["x0"])
    leg = bt["leg"].astype(np.int8)
    rep = {"episodes": B, "tag": a.tag, "build_id": alipmpc.build_id()}
    progs = {"lane_fp32": dict(program=1, precision=1), "lane_fp64": dict(program=1)}
    solvers = {k: alipmpc.Solver(alipmpc.default_cfg(0, 3, nc_max=5, ne_max=0, **kw)) for k, kw in progs.items()}
    s32 = solvers["lane_fp32"]
    foot0 = s32.solve(bt["x0"], bt["goal"], leg, bt["cir"], bt["nc"], u0=np.tile(bt["x0"], (1, 3)))["foot"][:, :2].copy()
    save = {"near": bt["near"], "x0": bt["x0"], "goal": bt["goal"], "foot0": foot0}
    for k, s in solvers.items():
        r = s.closed_loop(bt["x0"], foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=1, f_cyc=40)
        rep[f"device_{k}"] = {"status": counts(r["status"]), "near": counts(r["status"][bt["near"]]),
                              "far": counts(r["status"][~bt["near"]])}
        for f in ("status", "iters", "foot", "steps_to_goal"):
            save[f"{k}_{f}"] = r[f]
        print(k, rep[f"device_{k}"], flush=True)

    tol32 = dict(tol=alipmpc.FP32_TOL, acceptable_tol=alipmpc.FP32_ACCEPTABLE_TOL)
    co64 = C.default_cfg(0, 3, nc_max=5, ne_max=0)
    co32 = C.default_cfg(0, 3, nc_max=5, ne_max=0, **tol32)
    if not a.no_oracle:
        for name, co in (("oracle_tol64", co64), ("oracle_tol32", co32)):
            t0 = time.time()
            r = C.closed_loop_batch(co, bt["x0"], foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=1, f_cyc=40,
                                    nthreads=a.threads)
            rep[name] = {"status": counts(r["status"]), "near": counts(r["status"][bt["near"]]),
                         "far": counts(r["status"][~bt["near"]]), "s": time.time() - t0}
            for f in ("status", "iters", "foot", "steps_to_goal"):
                save[f"{name}_{f}"] = r[f]
            print(name, rep[name], flush=True)

    # host-driven loop: GPU fp32 solves; every tick's inputs also solved by the oracle at the fp32 tolerances
    orig = C.solve_batch
    rows = {k: [] for k in ("ep", "tick", "gst", "git", "ost", "oit", "dgoal", "dplan", "ferr", "o64st", "dbg")}
    dbg = "dbg" in os.environ.get("ALIPMPC_LIB", "")   # the -DALIP_LANE_DBG build: x_pred[:8] = convergence terms
    tick = [0]

    def gpu_solve(cfg, x0, goal, leg_, cir, nc, elp, ne, u0, nthreads=1):
        r = s32.solve(x0, goal, leg_, cir, nc, u0=u0)
        r["restorations"] = np.zeros(len(x0), np.int32)
        ro = orig(co32, x0, goal, leg_, cir, nc, None, None, u0, nthreads=a.threads)
        r64 = orig(co64, x0, goal, leg_, cir, nc, None, None, u0, nthreads=a.threads)
        rows["ep"].append(np.arange(len(x0), dtype=np.int32))   # (one walking step: every episode runs every tick)
        rows["tick"].append(np.full(len(x0), tick[0], np.int32))
        rows["gst"].append(r["status"]); rows["git"].append(r["iters"])
        rows["ost"].append(ro["status"]); rows["oit"].append(ro["iters"]); rows["o64st"].append(r64["status"])
        rows["dgoal"].append(np.hypot(*(x0[:, 0:2] - goal).T))
        rows["dplan"].append(np.hypot(*(ro["x_pred"][:, -1, 0:2] - goal).T))
        rows["ferr"].append(np.abs(r["foot"] - ro["foot"]).max(-1))
        if dbg:
            rows["dbg"].append(r["x_pred"].reshape(len(x0), -1)[:, :8].copy())
            r["x_pred"] = ro["x_pred"]   # (the driver's heading bookkeeping reads x_pred: take the oracle's)
        tick[0] += 1
        return r
    C.solve_batch = gpu_solve
    t0 = time.time()
    rh = C.closed_loop_batch(co32, bt["x0"], foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=1, f_cyc=40)
    C.solve_batch = orig
    for k in rows:
        if rows[k]:
            save[f"host_{k}"] = np.concatenate(rows[k])
    rep["host_driven"] = {"status": counts(rh["status"]), "s": time.time() - t0,
                          "gpu": counts(save["host_gst"]), "oracle32_same_inputs": counts(save["host_ost"]),
                          "oracle64_same_inputs": counts(save["host_o64st"])}
    print("host-driven", rep["host_driven"], flush=True)
    np.savez_compressed(os.path.join(a.out, f"study_{a.tag}.npz"), **save)
    with open(os.path.join(a.out, f"study_{a.tag}.json"), "w") as fh:
        json.dump(rep, fh, indent=1)


if __name__ == "__main__":
    main()
