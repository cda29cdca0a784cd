#!/usr/bin/env python3
"""Dev study: the status -3 (Error_In_Step_Computation) ticks of the closed loop.

  python tools/cl_m3.py [--episodes 65536] [--oracle-episodes 16384] [--out gpurun_out/m3]

1. cfg5's episodes (bench.global_inputs, seed 0), started as bench.closed_loop_rate starts them, through
   alipmpc_closed_loop_batch on the lane program fp32 / fp64 and the wave program fp64: -3 counts per tick.
2. The C oracle's closed loop on the first --oracle-episodes of them: its -3 count.
3. The same loop driven from the host (oracle.closed_loop_batch with every tick's solve sent to the GPU lane
   fp32 solver), which records the solve inputs of every -3 tick; those inputs are replayed through every
   program / precision and the C oracle (fp64), and saved (npz) for replay on the CPU.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=65536)
    ap.add_argument("--oracle-episodes", type=int, default=16384)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default="gpurun_out/m3")
    ap.add_argument("--record", default="lane_fp32", help="program whose -3 tick inputs the host-driven loop records")
    ap.add_argument("--test-episodes", action="store_true",
                    help="the episodes of tests/test_gpu.py::test_closed_loop_step_failures_vs_oracle instead of cfg5's")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    import alipmpc
    import oracle as C
    import bench

    B = a.episodes
    if a.test_episodes:
        from alipmpc import scenes
        B = 4096
        bt = scenes.make_batch_vec(B, seed=4242, n_cir=5, N=3)
        rng = np.random.default_rng(4243)
        near = np.arange(B) % 4 == 0
        ang = rng.uniform(np.pi, 1.5 * np.pi, near.sum())
        rad = rng.uniform(0.2, 1.0, near.sum())
        bt["x0"][near, 0:2] = bt["goal"][near] + np.stack([rad * np.cos(ang), rad * np.sin(ang)], 1)
    else:
        bt = bench.global_inputs("cfg5", 0, B, 32768, 0, 5, 0, 3)
    leg = bt["leg"].astype(np.int8)
    rep = {"episodes": B}
    progs = {"lane_fp32": dict(program=1, precision=1), "lane_fp64": dict(program=1), "wave_fp64": dict(program=0)}
    solvers = {k: alipmpc.Solver(alipmpc.default_cfg(0, 3, nc_max=5, ne_max=0, **kw)) for k, kw in progs.items()}
    # bench.closed_loop_rate's start: stance on the first foothold of the config's own solve from x0
    s32 = solvers[a.record]
    o = s32.solve(bt["x0"], bt["goal"], leg, bt["cir"], bt["nc"], u0=np.tile(bt["x0"], (1, 3)))
    foot0 = o["foot"][:, :2].copy()
    rep["cold_fp32_status"] = counts(o["status"])
    dev = {}
    for k, s in solvers.items():
        t0 = time.time()
        r = s.closed_loop(bt["x0"], foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=1, f_cyc=40)
        dev[k] = r
        st = r["status"]
        rep[f"device_{k}"] = {"status": counts(st), "s": time.time() - t0,
                              "m3_per_tick": [int(v) for v in (st[:, 0, :] == -3).sum(0)],
                              "m3_episodes": int((st == -3).any(axis=(1, 2)).sum()),
                              "m3_iters": counts(r["iters"][st == -3]) if (st == -3).any() else {}}
        print(k, rep[f"device_{k}"]["status"], flush=True)

    # the oracle's own closed loop (fp64) on a subset
    Bo = min(a.oracle_episodes, B)
    co = C.default_cfg(0, 3, nc_max=5, ne_max=0)
    t0 = time.time()
    ro = C.closed_loop_batch(co, bt["x0"][:Bo], foot0[:Bo], bt["goal"][:Bo], leg[:Bo], bt["cir"][:Bo], bt["nc"][:Bo],
                             steps=1, f_cyc=40, nthreads=a.threads)
    rep["oracle"] = {"episodes": Bo, "status": counts(ro["status"]), "s": time.time() - t0}
    for k in dev:
        rep["oracle"][f"{k}_same_subset"] = counts(dev[k]["status"][:Bo])
    print("oracle", rep["oracle"], flush=True)

    # host-driven loop: every tick's solve on the GPU (lane fp32), -3 inputs recorded
    rec = {k: [] for k in ("x0", "goal", "leg", "cir", "nc", "u0", "iters")}
    orig = C.solve_batch

    def gpu_solve(cfg, x0, goal, leg_, cir, nc, elp, ne, u0, nthreads=1):
        r = s32.solve(x0, goal, leg_, cir, nc, u0=u0)
        r["restorations"] = np.zeros(len(x0), np.int32)
        m = r["status"] == -3
        if m.any():
            for key, v in (("x0", x0), ("goal", goal), ("leg", leg_), ("cir", cir), ("nc", nc), ("u0", u0),
                           ("iters", r["iters"])):
                rec[key].append(np.asarray(v)[m])
        return r
    C.solve_batch = gpu_solve
    t0 = time.time()
    rh = C.closed_loop_batch(co, bt["x0"], foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=1, f_cyc=40)
    C.solve_batch = orig
    rep["host_driven_" + a.record] = {"status": counts(rh["status"]), "s": time.time() - t0,
                                    "same_as_device": float((rh["status"] == dev[a.record]["status"]).mean())}
    print("host-driven", rep["host_driven_" + a.record], flush=True)
    if rec["x0"]:
        R = {k: np.concatenate(v) for k, v in rec.items()}
        np.savez(os.path.join(a.out, "m3_inputs.npz"), **R)
        nR = len(R["x0"])
        rep["replay"] = {"instances": nR}
        for k, s in solvers.items():
            for mi in (30, 100):
                if mi == 100:
                    c = s.cfg
                    s2 = alipmpc.Solver(alipmpc.default_cfg(0, 3, nc_max=5, ne_max=0, max_iter=100, **progs[k]))
                else:
                    s2 = s
                r = s2.solve(R["x0"], R["goal"], R["leg"], R["cir"], R["nc"], u0=R["u0"])
                rep["replay"][f"{k}_it{mi}"] = counts(r["status"])
                if k == a.record and mi == 30:
                    rep["replay"]["reproduces_m3"] = float((r["status"] == -3).mean())
        for mi in (30, 100):
            co2 = C.default_cfg(0, 3, nc_max=5, ne_max=0, max_iter=mi)
            r = C.solve_batch(co2, R["x0"], R["goal"], R["leg"], R["cir"], R["nc"], None, None, R["u0"],
                              nthreads=a.threads)
            rep["replay"][f"oracle_it{mi}"] = counts(r["status"])
        print("replay", rep["replay"], flush=True)
    with open(os.path.join(a.out, "m3_report.json"), "w") as fh:
        json.dump(rep, fh, indent=1)
    print(json.dumps(rep))


if __name__ == "__main__":
    main()
