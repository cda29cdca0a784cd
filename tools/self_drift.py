#!/usr/bin/env python3
"""The closed loop's own sensitivity (CPU): oracle.closed_loop_batch against ITSELF with the initial
states moved by one ulp, on the episodes of tests/test_gpu.py::test_closed_loop_matches_oracle (same seeds, sizes and
tolerances per parametrisation).  Two loops that differ only by rounding at the start drift apart the way the GPU loop
and the oracle's loop do (a warm start on the tolerance boundary takes one iteration more, an unconverged iterate moves,
and the episode follows another path), so these statistics are the principled floor for the GPU-vs-oracle bars: the
test asserts each GPU statistic >= this table's value - 0.03.  The fp32 case is also run with the initial states
rounded to fp32 ("_f32round"), the perturbation scale of an fp32 program.  "_jitter": one ulp on every tick's warm start
(oracle.closed_loop_batch(jitter=True)) — two implementations differ by rounding at every solve, not only at the start;
the bars use the smaller of the two fp64 perturbations; the fp32 case's bar is its "_f32jitter" row (every tick's warm
start moved by 2^-24 relative: an fp32 iterate's rounding at every solve).  "_toljitter": every returned iterate moved
by the solve's tolerance (relative) — where two implementations may stop inside the convergence ball.

  python tools/self_drift.py [--out profiles/r6/parity/self_drift.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import oracle as C  # noqa: E402
from alipmpc import scenes  # noqa: E402

# (variant, kick, program, prec) as test_closed_loop_matches_oracle; fp32: the fp32 defaults' tolerances (N <= 3)
CASES = [(0, 0.0, 0, 0), (0, 0.05, 0, 0), (1, 0.05, 0, 0), (0, 0.05, 1, 0), (0, 0.05, 1, 1)]
FP32_TOL = (1e-4, 1e-3)


def stats(o, ref):
    err = np.abs(o["foot"] - ref["foot"]).max(-1)
    conv = (o["status"][:, :, -1] == 0) & (ref["status"][:, :, -1] == 0)
    return {"status_agree": float((o["status"] == ref["status"]).mean()),
            "iters_within_1": float((np.abs(o["iters"] - ref["iters"]) <= 1).mean()),
            "steps_to_goal_agree": float((o["steps_to_goal"] == ref["steps_to_goal"]).mean()),
            "foot_le_1e-3": float((err[conv] <= 1e-3).mean()), "foot_le_1e-4": float((err[conv] <= 1e-4).mean()),
            "converged_steps": int(conv.sum())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r6", "parity", "self_drift.json"))
    a = ap.parse_args()
    B, S, F = 48, 4, 40
    rep = {"episodes": B, "steps": S, "f_cyc": F, "perturbation": "x0 moved by one ulp (np.nextafter toward +inf)",
           "cases": {}}
    for variant, kick, program, prec in CASES:
        bt = scenes.make_batch(B, seed=520 + variant + int(kick * 100), n_cir=5)
        x0 = bt["x0"].copy()
        x0[:12, 0:2] = bt["goal"][:12] - (np.array([1.0, 0.8]) if variant == 1 else np.array([0.6, 0.5]))
        leg = bt["leg"].astype(np.int8)
        co = C.default_cfg(variant, 3, nc_max=5, ne_max=0)
        foot0 = C.solve_batch(co, x0, bt["goal"], leg, bt["cir"], bt["nc"], None, None, np.tile(x0, (1, 3)))["foot"][:, 0:2]
        if prec:
            co = C.default_cfg(variant, 3, nc_max=5, ne_max=0, tol=FP32_TOL[0], acceptable_tol=FP32_TOL[1])
        run = lambda x: C.closed_loop_batch(co, x, foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=S, f_cyc=F,  # noqa: E731
                                            kick=kick, seed=7)
        ref = run(x0)
        pert = run(np.nextafter(x0, np.inf))
        tag = f"{variant}_{kick}_{program}" + ("_fp32" if prec else "")
        rep["cases"][tag] = stats(pert, ref)
        # one ulp at EVERY solve (each tick's warm start): the rounding differences two implementations accumulate
        rep["cases"][tag + "_jitter"] = stats(C.closed_loop_batch(co, x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"],
                                                                  steps=S, f_cyc=F, kick=kick, seed=7, jitter=True), ref)
        print(tag + "_jitter", json.dumps(rep["cases"][tag + "_jitter"]), flush=True)
        if prec:   # the fp32 program's own perturbation scale: the initial states rounded to fp32 (~6e-8 relative), and
            # every tick's warm start moved by 2^-24 relative (fp32 rounding of the iterate at every solve)
            rep["cases"][tag + "_f32round"] = stats(run(x0.astype(np.float32).astype(np.float64)), ref)
            print(tag + "_f32round", json.dumps(rep["cases"][tag + "_f32round"]), flush=True)
            rep["cases"][tag + "_f32jitter"] = stats(C.closed_loop_batch(co, x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"],
                                                                         steps=S, f_cyc=F, kick=kick, seed=7,
                                                                         jitter=2.0 ** -24), ref)
            print(tag + "_f32jitter", json.dumps(rep["cases"][tag + "_f32jitter"]), flush=True)
        # the returned iterate moved by the solve's tolerance (relative): where two implementations may stop inside the
        # convergence ball (fp64 1e-8, fp32 1e-4)
        rep["cases"][tag + "_toljitter"] = stats(C.closed_loop_batch(co, x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"],
                                                                     steps=S, f_cyc=F, kick=kick, seed=7,
                                                                     jitter=float(co.tol)), ref)
        print(tag + "_toljitter", json.dumps(rep["cases"][tag + "_toljitter"]), flush=True)
        print(tag, json.dumps(rep["cases"][tag]), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(rep, fh, indent=1)


if __name__ == "__main__":
    main()
