#!/usr/bin/env python3 -B
"""Golden-fixture generator (DEV-ONLY, runs in the build container, never on the GPU box).

Imports the reference planner modules from /root/reference with a stub ``cyipopt`` module
(cyipopt / IPOPT / HSL are not installed and there is no network), evaluates the reference's own
``LIP_Prob`` callbacks and ``MPCCBF`` setup code on seeded inputs, and writes small ``.npz``
fixtures to ``tests/golden/``.  Nothing from the reference (source, bytecode, pickles) is copied:
only numeric inputs and the outputs the reference produced for them.

Fixtures written
  g1_callbacks_{modi,sig_step,dd}.npz  f, grad f, c, J of the reference LIP_Prob at seeded (x0, scene, goal, u)
                                       MPC_LIP_modi.py:430-583, MPC_LIP_sig_step.py:372-496, MPC_DD_sig_step.py:351-477
  g1_callbacks_modi_n5.npz             f and c for N=5 (reference objective/constraints loop over N;
                                       its gradient/jacobian are N=3-only, so N=5 derivatives are FD-pinned)
  g2_setup_{modi,sig_step}.npz         cl, cu, selected obstacles, detour goal captured from solveMPCCBF
                                       (MPC_LIP_modi.py:197-283, 325-338; MPC_LIP_sig_step.py:184-265)
  g3_sup_learn.npz                     the 640 recorded cyipopt MPC calls of sup_learn/*.csv, with the
                                       reconstructed solve inputs and a flag for rows a converged solve of
                                       the reference NLP reproduces (<1e-6)
  g3_synthetic_{modi,sig_step,dd}.npz  random 5-obstacle scenes solved to a tight KKT point by two scipy
                                       methods on the reference callbacks; kept where both agree
  g4_aux.npz                           get_next_states, xk_track_det, alip_des_vel, cal_foot_with_veldes,
                                       constant matrices A, B, W, M_A, M_B, dx_du, dP_du

Run:  PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python3 -B tools/gen_goldens.py [--quick]
"""
import os
import sys
import types
import random
import argparse
import warnings

sys.dont_write_bytecode = True          # never write __pycache__ into /root/reference
os.environ.setdefault("MPLBACKEND", "Agg")

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


class _StubProblem:
    """Captures what solveMPCCBF hands to cyipopt.Problem; solve() is pluggable."""
    last = None
    solver = None          # callable(problem) -> (u, status)

    def __init__(self, n, m, problem_obj, lb, ub, cl, cu):
        self.n, self.m, self.problem_obj = n, m, problem_obj
        self.lb, self.ub = lb, ub
        self.cl, self.cu = np.asarray(cl, float), np.asarray(cu, float)
        self.options = {}
        _StubProblem.last = self

    def add_option(self, k, v):
        self.options[k] = v

    def solve(self, u0):
        self.u0 = np.asarray(u0, float).copy()
        if _StubProblem.solver is None:
            return self.u0.copy(), {"status": 0}
        u, st = _StubProblem.solver(self)
        return u, {"status": st}


def import_reference():
    stub = types.ModuleType("cyipopt")
    stub.Problem = _StubProblem
    sys.modules["cyipopt"] = stub
    sys.path.insert(0, REF)
    warnings.filterwarnings("ignore")
    import MPC_LIP_modi as modi
    import MPC_LIP_sig_step as sig
    import MPC_DD_sig_step as dd
    import rand_obs
    return modi, sig, dd, rand_obs


# ----------------------------------------------------------------------------------------------
# scipy solves of the reference NLP (the stand-in for IPOPT, which cannot be installed offline)
# ----------------------------------------------------------------------------------------------
def _split_bounds(cl, cu):
    lo = np.isfinite(cl)
    hi = np.isfinite(cu)
    return lo, hi


def solve_slsqp(prob, u0, cl, cu, lb=None, ub=None, fd_deriv=False):
    from scipy.optimize import minimize
    lo, hi = _split_bounds(cl, cu)
    f = prob.objective
    c = prob.constraints
    if fd_deriv:
        g = lambda u: _cfd(lambda v: np.atleast_1d(f(v)), u)[0]
        J = lambda u: _cfd(c, u)
    else:
        g = lambda u: np.ravel(prob.gradient(u))
        J = lambda u: np.asarray(prob.jacobian(u)).reshape(len(cl), -1)
    cons = [
        {"type": "ineq", "fun": lambda u: np.asarray(c(u))[lo] - cl[lo], "jac": lambda u: J(u)[lo]},
        {"type": "ineq", "fun": lambda u: cu[hi] - np.asarray(c(u))[hi], "jac": lambda u: -J(u)[hi]},
    ]
    bounds = None if lb is None else list(zip(lb, ub))
    r = minimize(f, u0, jac=g, constraints=cons, method="SLSQP", bounds=bounds,
                 options={"ftol": 1e-15, "maxiter": 1000})
    return r.x, (0 if r.success else -1)


def solve_trust(prob, u0, cl, cu, lb=None, ub=None, fd_deriv=False):
    from scipy.optimize import minimize, NonlinearConstraint, BFGS, Bounds
    f = prob.objective
    c = lambda u: np.asarray(prob.constraints(u), float)
    if fd_deriv:
        g = lambda u: _cfd(lambda v: np.atleast_1d(f(v)), u)[0]
        J = lambda u: _cfd(c, u)
    else:
        g = lambda u: np.ravel(prob.gradient(u))
        J = lambda u: np.asarray(prob.jacobian(u)).reshape(len(cl), -1)
    nlc = NonlinearConstraint(c, cl, cu, jac=J, hess=BFGS())
    bounds = None if lb is None else Bounds(lb, ub)
    r = minimize(f, u0, jac=g, hess=BFGS(), constraints=[nlc], bounds=bounds, method="trust-constr",
                 options={"gtol": 1e-12, "xtol": 1e-14, "maxiter": 3000, "barrier_tol": 1e-12})
    return r.x, (0 if r.status in (1, 2) else -1)


def _cfd(fun, u, h=1e-6):
    u = np.asarray(u, float)
    f0 = np.asarray(fun(u), float)
    J = np.zeros((f0.size, u.size))
    for j in range(u.size):
        e = np.zeros_like(u)
        e[j] = h
        J[:, j] = (np.asarray(fun(u + e), float) - np.asarray(fun(u - e), float)) / (2 * h)
    return J


def violation(c, cl, cu):
    return float(np.max(np.concatenate([[0.0], cl - c, c - cu])))


# ----------------------------------------------------------------------------------------------
# scene / state sampling (same distribution the bench uses)
# ----------------------------------------------------------------------------------------------
def sample_scene(rand_obs, seed, num, typ):
    random.seed(seed)
    cir, elp = rand_obs.gen_ran_obs_list(num, typ)
    return np.array(cir, float).reshape(-1, 3), np.array(elp, float).reshape(-1, 5)


def sample_state(rng, cir_safe, elp_safe, goal=(10.0, 10.0)):
    while True:
        pos = rng.uniform(0.0, 10.0, 2)
        ok = True
        for c in cir_safe:
            if np.hypot(*(pos - c[:2])) < c[2] + 0.2:
                ok = False
        for e in elp_safe:
            if np.hypot(*(pos - e[:2])) < max(e[2], e[3]) + 0.2:
                ok = False
        if ok and np.hypot(*(pos - np.asarray(goal))) > 0.5:
            break
    leg = int(rng.choice([-1, 1]))
    th = np.arctan2(goal[1] - pos[1], goal[0] - pos[0]) + rng.normal(0.0, 0.2)
    vbx = rng.uniform(0.45, 0.75)
    vby = -leg * rng.uniform(0.17, 0.33)
    c, s = np.cos(th), np.sin(th)
    vx = c * vbx - s * vby
    vy = s * vbx + c * vby
    return np.array([pos[0], pos[1], vx, vy, th]), leg


def inflate(cir, elp, safe=0.4):
    cs = cir + np.array([0, 0, safe]) if len(cir) else cir
    es = elp + np.array([0, 0, safe, safe, 0]) if len(elp) else elp
    return cs, es


# ----------------------------------------------------------------------------------------------
def gen_g1(modi, sig, dd, rand_obs, n_cases):
    rng = np.random.default_rng(1234)
    goal = [[10.0, 10.0]]
    margin = [-0.5, 10.5]
    out = {}
    # ---- modi, N=3: circles only, ellipses only, mixed, no obstacles
    recs = {k: [] for k in ["x0", "goal", "cir", "nc", "elp", "ne", "u", "f", "grad", "c", "J", "m"]}
    NCM, NEM = 6, 6
    for t in range(n_cases):
        kind = t % 4
        if kind == 0:
            cir, elp = sample_scene(rand_obs, 100 + t, 5, "cir")
        elif kind == 1:
            cir, elp = sample_scene(rand_obs, 100 + t, 6, "mix")
        elif kind == 2:
            cir, elp = sample_scene(rand_obs, 100 + t, 4, "mix")
            cir = cir[:0]
        else:
            cir, elp = np.zeros((0, 3)), np.zeros((0, 5))
        cs, es = inflate(cir, elp)
        x0, leg = sample_state(rng, cs, es)
        g = np.array([10.0, 10.0]) if t % 3 else rng.uniform(2, 10, 2)
        mpc = modi.MPCCBF(goal, cir, cs, elp, es, margin)
        u = np.tile(x0, 3) + rng.normal(0, 0.3, 15)
        prob = modi.LIP_Prob(np.matrix(x0).T, mpc.M_A, mpc.M_B, mpc.A, mpc.W, mpc.dx_du, mpc.dP_du,
                             list(cs), list(es), np.matrix(g).T, 3)
        f = prob.objective(u)
        gr = np.ravel(prob.gradient(u))
        c = np.asarray(prob.constraints(u), float)
        J = np.asarray(prob.jacobian(u), float)
        _store(recs, x0, g, cs, es, NCM, NEM, u, f, gr, c, J)
    out["modi"] = recs

    # ---- sig_step, N=3: all obstacles used, 0 and 4/5 circles
    recs = {k: [] for k in ["x0", "goal", "cir", "nc", "elp", "ne", "u", "f", "grad", "c", "J", "m"]}
    for t in range(n_cases):
        if t % 3 == 0:
            cir = np.zeros((0, 3))
        else:
            cir, _ = sample_scene(rand_obs, 300 + t, 4 + (t % 2), "cir")
        cs, _ = inflate(cir, np.zeros((0, 5)))
        x0, leg = sample_state(rng, cs, [])
        g = np.array([10.0, 10.0])
        mpc = sig.MPCCBF(goal, cir, cs, margin)
        u = np.tile(x0, 3) + rng.normal(0, 0.3, 15)
        prob = sig.LIP_Prob(np.matrix(x0).T, mpc.M_A, mpc.M_B, mpc.A, mpc.W, mpc.dx_du, mpc.dP_du,
                            cs, np.matrix(g).T, 3)
        f = prob.objective(u)
        gr = np.ravel(prob.gradient(u))
        c = np.asarray(prob.constraints(u), float)
        J = np.asarray(prob.jacobian(u), float).reshape(len(c), 15)
        _store(recs, x0, g, cs, np.zeros((0, 5)), NCM, NEM, u, f, gr, c, J)
    out["sig_step"] = recs

    # ---- modi N=5: f and c only from the reference (its derivatives are N=3-only)
    recs = {k: [] for k in ["x0", "goal", "cir", "nc", "elp", "ne", "u", "f", "c", "m"]}
    for t in range(n_cases // 2):
        # 10 non-overlapping obstacles rarely fit rand_obs' spacing rule (its rejection loop does
        # not terminate), so take 5 circles + 5 ellipses built from two independent 5-circle draws
        cir, _ = sample_scene(rand_obs, 500 + t, 5, "cir")
        c2, _ = sample_scene(rand_obs, 600 + t, 5, "cir")
        r2 = np.random.default_rng(600 + t)
        elp = np.array([[c[0], c[1], c[2], c[2] * r2.uniform(0.5, 1.0), r2.integers(0, 181) * np.pi / 180]
                        for c in c2])
        cs, es = inflate(cir, elp)
        x0, leg = sample_state(rng, cs, es)
        g = np.array([10.0, 10.0])
        mpc = modi.MPCCBF(goal, cir, cs, elp, es, margin, step=5)
        u = np.tile(x0, 5) + rng.normal(0, 0.3, 25)
        prob = modi.LIP_Prob(np.matrix(x0).T, mpc.M_A, mpc.M_B, mpc.A, mpc.W, None, None,
                             list(cs), list(es), np.matrix(g).T, 5)
        f = prob.objective(u)
        c = np.asarray(prob.constraints(u), float)
        recs["x0"].append(x0); recs["goal"].append(g)
        recs["cir"].append(_pad(cs, 10, 3)); recs["nc"].append(len(cs))
        recs["elp"].append(_pad(es, 10, 5)); recs["ne"].append(len(es))
        recs["u"].append(u); recs["f"].append(f); recs["c"].append(_pad1(c, 5 * 25)); recs["m"].append(len(c))
    out["modi_n5"] = recs

    # ---- DD (unicycle), N=3
    recs = {k: [] for k in ["x0", "goal", "cir", "nc", "elp", "ne", "u", "last_u", "f", "grad", "c", "J", "m"]}
    for t in range(n_cases):
        cir, elp = sample_scene(rand_obs, 700 + t, 5 if t % 2 else 6, "cir" if t % 2 else "mix")
        cs, es = inflate(cir, elp)
        p0, leg = sample_state(rng, cs, es)
        x0 = np.array([p0[0], p0[1], p0[4]])
        g = np.array([10.0, 10.0])
        mpc = dd.MPCCBF(goal, cir, cs, elp, es, margin)
        u = np.tile([rng.uniform(0.4, 0.8), rng.uniform(-0.2, 0.2)], 3) + rng.normal(0, 0.05, 6)
        if t % 5 == 0:
            u[1] = 0.0                        # exercise sign(0) = 0 in den_du
        last_u = np.array([rng.uniform(0.4, 0.8), rng.uniform(-0.2, 0.2)])
        prob = dd.LIP_Prob(np.matrix(x0).T, mpc.A, mpc.dt, list(cs), list(es), np.matrix(g).T, 3, last_u)
        f = prob.objective(u)
        gr = np.ravel(prob.gradient(u))
        c = np.asarray(prob.constraints(u), float)
        J = np.asarray(prob.jacobian(u), float).reshape(len(c), 6)
        recs["last_u"].append(last_u)
        _store(recs, x0, g, cs, es, NCM, NEM, u, f, gr, c, J, nvar=6)
    out["dd"] = recs
    for name, recs in out.items():
        np.savez_compressed(os.path.join(OUT, f"g1_callbacks_{name}.npz"),
                            **{k: np.asarray(v) for k, v in recs.items()})
        print(f"g1 {name}: {len(recs['f'])} cases", flush=True)


def _pad(a, rows, cols):
    out = np.zeros((rows, cols))
    if len(a):
        out[:len(a)] = a
    return out


def _pad1(a, n):
    out = np.full(n, np.nan)
    out[:len(a)] = a
    return out


def _store(recs, x0, g, cs, es, NCM, NEM, u, f, gr, c, J, nvar=15):
    m = len(c)
    MM = 3 * (5 + NCM + NEM)
    recs["x0"].append(x0); recs["goal"].append(g)
    recs["cir"].append(_pad(cs, NCM, 3)); recs["nc"].append(len(cs))
    recs["elp"].append(_pad(es, NEM, 5)); recs["ne"].append(len(es))
    recs["u"].append(u); recs["f"].append(f); recs["grad"].append(gr)
    recs["c"].append(_pad1(c, MM))
    Jp = np.full((MM, nvar), np.nan)
    Jp[:m] = J
    recs["J"].append(Jp); recs["m"].append(m)


# ----------------------------------------------------------------------------------------------
def gen_g2(modi, sig, rand_obs, n_cases):
    """Setup goldens: cl/cu, selected obstacles, detour goal (stub Problem capture, no solve)."""
    rng = np.random.default_rng(4321)
    margin = [-0.5, 10.5]
    _StubProblem.solver = None
    for variant in ["modi", "sig_step"]:
        R = {k: [] for k in ["x0", "leg", "goal", "cir", "nc", "elp", "ne", "cl", "cu", "m",
                             "goal_eff", "sel_cir", "sel_elp"]}
        for t in range(n_cases):
            typ = "mix" if (variant == "modi" and t % 2) else "cir"
            cir, elp = sample_scene(rand_obs, 900 + t, 6 if typ == "mix" else 5, typ)
            if variant == "sig_step":
                elp = np.zeros((0, 5))
            cs, es = inflate(cir, elp)
            x0, leg = sample_state(rng, cs, es)
            if t % 4 == 1 and len(cs):
                # put the robot between a circle and the goal so the detour heuristic fires
                c0 = cs[t % len(cs)]
                d = np.array([10.0, 10.0]) - c0[:2]
                d /= np.linalg.norm(d) + 1e-12
                # off the circle-goal line by 1..10 degrees: exactly collinear starts make the sign of the
                # reference's (theta - alpha) a matter of atan2 rounding
                ang = rng.uniform(np.deg2rad(1.0), np.deg2rad(10.0)) * rng.choice([-1, 1])
                ca, sa = np.cos(ang), np.sin(ang)
                d = np.array([ca * d[0] - sa * d[1], sa * d[0] + ca * d[1]])
                pos = c0[:2] - d * (c0[2] + 0.3 + 0.8 * rng.random())
                x0[:2] = pos
            g = [[10.0, 10.0]] if t % 5 else [[rng.uniform(4, 10), rng.uniform(4, 10)]]
            if variant == "modi":
                mpc = modi.MPCCBF(g, cir, cs, elp, es, margin)
                mpc.select_obs(np.matrix(x0).T)
                mpc.solveMPCCBF(np.matrix(x0).T, leg, np.tile(x0, 3))
                sel_c = [_row_index(cs, r) for r in mpc.sel_cir]
                sel_e = [_row_index(es, r) for r in mpc.sel_elp]
            else:
                mpc = sig.MPCCBF(g, cir, cs, margin)
                mpc.solveMPCCBF(np.matrix(x0).T, leg, None)
                sel_c = list(range(len(cs)))
                sel_e = []
            P = _StubProblem.last
            MM = 3 * (5 + 6 + 6)
            R["x0"].append(x0); R["leg"].append(leg); R["goal"].append(np.ravel(g))
            R["cir"].append(_pad(cs, 6, 3)); R["nc"].append(len(cs))
            R["elp"].append(_pad(es, 6, 5)); R["ne"].append(len(es))
            R["cl"].append(_pad1(P.cl, MM)); R["cu"].append(_pad1(P.cu, MM)); R["m"].append(P.m)
            R["goal_eff"].append(np.ravel(P.problem_obj.goal))
            R["sel_cir"].append(_mask(sel_c, 6)); R["sel_elp"].append(_mask(sel_e, 6))
        np.savez_compressed(os.path.join(OUT, f"g2_setup_{variant}.npz"),
                            **{k: np.asarray(v) for k, v in R.items()})
        nd = int(np.sum(np.any(np.asarray(R["goal_eff"]) != np.asarray(R["goal"]), axis=1)))
        print(f"g2 {variant}: {n_cases} cases, detour fired in {nd}")


def _row_index(arr, row):
    for i, r in enumerate(arr):
        if np.array_equal(np.asarray(r, float), np.asarray(row, float)):
            return i
    raise ValueError("selected obstacle not found")


def _mask(idx, n):
    m = np.zeros(n, np.int8)
    m[idx] = 1
    return m


# ----------------------------------------------------------------------------------------------
def gen_g3_sup_learn(modi, quick):
    """The 640 recorded cyipopt calls (logger_iml.py:342-401) and a converged reference re-solve."""
    X = np.loadtxt(os.path.join(REF, "sup_learn", "X_data.csv"), delimiter=",")
    Y = np.loadtxt(os.path.join(REF, "sup_learn", "y_mpc_data.csv"), delimiter=",")
    goal = [[10.0, 10.0]]
    margin = [-0.5, 10.5]
    cir = X[0, 0:18].reshape(6, 3)
    cs = cir + np.array([0, 0, 0.4])                       # main_sim_mpc.py:11,14 safe_dis = 0.4
    mpc = modi.MPCCBF(goal, cir, cs, [], [], margin)
    n = len(X)
    R = {k: [] for k in ["x_nex", "leg", "u0", "foot_logged", "x_nex_logged", "foot_ref",
                         "u_ref", "ok_ref", "status_ref"]}
    # heading at the start of each walking step (rest_t == 0.4 row) -> hd_input_pr = y[3] - that
    start_hd = None
    for i in range(n):
        rest_t = X[i, 28]
        if abs(rest_t - 0.4) < 1e-12 or start_hd is None:
            start_hd = X[i, 22]
        hd_pr = Y[i, 3] - start_hd
        x_nex, _ = mpc.get_next_states(X[i, 18:20], X[i, 20:22], X[i, 22],
                                       np.array([X[i, 23], X[i, 24], hd_pr]), rest_t)
        leg = -int(X[i, 27])
        u0 = np.tile(x_nex, 3)
        R["x_nex"].append(x_nex); R["leg"].append(leg); R["u0"].append(u0)
        R["foot_logged"].append(Y[i, 0:2]); R["x_nex_logged"].append(Y[i, 4:6])
    if quick:
        idx = range(0, n, 8)
    else:
        idx = range(n)

    _StubProblem.solver = _wrap_solver(lambda P: solve_slsqp(P.problem_obj, P.u0, P.cl, P.cu))
    fr = np.full((n, 3), np.nan)
    ur = np.full((n, 15), np.nan)
    ok = np.zeros(n, np.int8)
    stv = np.full(n, -9, np.int32)
    for i in idx:
        x_nex = R["x_nex"][i]
        _, p0, _, _, feasi, _ = mpc.gen_control_test(x_nex, R["leg"][i], R["u0"][i])
        fr[i] = p0
        ur[i] = _last_solution[0]
        stv[i] = feasi
        ok[i] = int(np.max(np.abs(p0[:2] - Y[i, 0:2])) < 1e-6)
    _StubProblem.solver = None
    R["foot_ref"] = fr; R["u_ref"] = ur; R["ok_ref"] = ok; R["status_ref"] = stv
    R["cir_safe"] = cs
    np.savez_compressed(os.path.join(OUT, "g3_sup_learn.npz"), **{k: np.asarray(v) for k, v in R.items()})
    print(f"g3 sup_learn: {n} rows, re-solved {len(list(idx))}, reproduced <1e-6: {int(ok.sum())}")
    err = np.max(np.abs(np.asarray(R['x_nex'])[:, :2] - np.asarray(R['x_nex_logged'])), axis=1)
    print(f"   get_next_states vs logged x_nex: max err {err.max():.3e}")


_last_solution = []


def _wrap_solver(fn):
    def s(P):
        u, st = fn(P)
        _last_solution.clear()
        _last_solution.append(u)
        return u, st
    return s


# ----------------------------------------------------------------------------------------------
def gen_g3_synthetic(modi, sig, rand_obs, n_cases, variant):
    """Random 5-obstacle scenes; converged by SLSQP and trust-constr on the reference callbacks."""
    rng = np.random.default_rng(777 if variant == "modi" else 778)
    margin = [-0.5, 10.5]
    R = {k: [] for k in ["x0", "leg", "goal", "cir", "nc", "elp", "ne", "u0", "u_ref", "foot_ref",
                         "agree", "viol"]}
    kept = 0
    for t in range(n_cases):
        if variant == "modi":
            cir, elp = sample_scene(rand_obs, 2000 + t, 5, "cir" if t % 3 else "mix")
        else:
            cir, elp = sample_scene(rand_obs, 3000 + t, 5, "cir")
            elp = np.zeros((0, 5))
        cs, es = inflate(cir, elp)
        x0, leg = sample_state(rng, cs, es)
        goal = [[10.0, 10.0]]
        res = []
        for fn in (solve_slsqp, solve_trust):
            _StubProblem.solver = _wrap_solver(lambda P, fn=fn: fn(P.problem_obj, P.u0, P.cl, P.cu))
            if variant == "modi":
                mpc = modi.MPCCBF(goal, cir, cs, elp, es, margin)
                u0 = np.tile(x0, 3)
                out = mpc.gen_control_test(x0, leg, u0)
                p0 = out[1]
            else:
                mpc = sig.MPCCBF(goal, cir, cs, margin)
                u0 = np.tile(x0, 3)
                out = mpc.gen_control_test(x0, leg, None)
                p0 = out[1]
            P = _StubProblem.last
            u = _last_solution[0].copy()
            c = np.asarray(P.problem_obj.constraints(u), float)
            res.append((u, np.ravel(p0), violation(c, P.cl, P.cu)))
        _StubProblem.solver = None
        (ua, pa, va), (ub_, pb, vb) = res
        agree = float(np.max(np.abs(pa - pb)))
        R["x0"].append(x0); R["leg"].append(leg); R["goal"].append(np.array([10.0, 10.0]))
        R["cir"].append(_pad(cs, 6, 3)); R["nc"].append(len(cs))
        R["elp"].append(_pad(es, 6, 5)); R["ne"].append(len(es))
        R["u0"].append(u0); R["u_ref"].append(ua); R["foot_ref"].append(pa)
        R["agree"].append(agree); R["viol"].append(max(va, vb))
        if agree < 1e-8 and max(va, vb) < 1e-8:
            kept += 1
    np.savez_compressed(os.path.join(OUT, f"g3_synthetic_{variant}.npz"),
                        **{k: np.asarray(v) for k, v in R.items()})
    print(f"g3 synthetic {variant}: {n_cases} scenes, both scipy methods agree <1e-8 on {kept}")


def gen_g3_synthetic_dd(dd, rand_obs, n_cases):
    """DD (unicycle) scenes solved by SLSQP and trust-constr on the reference DD callbacks, with the
    reference's variable bounds v in [0.4, 0.8], w in [-pi/16, pi/16] (MPC_DD_sig_step.py:123-193)."""
    rng = np.random.default_rng(779)
    margin = [-0.5, 10.5]
    R = {k: [] for k in ["x0", "goal", "cir", "nc", "elp", "ne", "u0", "last_u", "u_ref", "agree", "viol",
                         "f_ref"]}
    kept = 0
    for t in range(n_cases):
        cir, elp = sample_scene(rand_obs, 4000 + t, 5, "cir" if t % 3 else "mix")
        cs, es = inflate(cir, elp)
        p0, _ = sample_state(rng, cs, es)
        x0 = np.array([p0[0], p0[1], p0[4]])
        last_u = np.array([rng.uniform(0.45, 0.75), rng.uniform(-0.15, 0.15)])
        u0 = np.tile(last_u, 3)
        goal = [[10.0, 10.0]]
        res = []
        for fn in (solve_slsqp, solve_trust):
            _StubProblem.solver = _wrap_solver(lambda P, fn=fn: fn(P.problem_obj, P.u0, P.cl, P.cu,
                                                                    np.asarray(P.lb, float), np.asarray(P.ub, float)))
            mpc = dd.MPCCBF(goal, cir, cs, elp, es, margin)
            import contextlib, io
            with contextlib.redirect_stdout(io.StringIO()):
                mpc.gen_dd_control(x0, u0, last_u)
            P = _StubProblem.last
            u = _last_solution[0].copy()
            c = np.asarray(P.problem_obj.constraints(u), float)
            vb = max(0.0, float(np.max(np.concatenate([np.asarray(P.lb) - u, u - np.asarray(P.ub)]))))
            res.append((u, max(violation(c, P.cl, P.cu), vb), float(P.problem_obj.objective(u))))
        _StubProblem.solver = None
        (ua, va, fa), (ub_, vb_, fb) = res
        agree = float(np.max(np.abs(ua - ub_)))
        R["x0"].append(x0); R["goal"].append(np.array([10.0, 10.0]))
        R["cir"].append(_pad(cs, 6, 3)); R["nc"].append(len(cs))
        R["elp"].append(_pad(es, 6, 5)); R["ne"].append(len(es))
        R["u0"].append(u0); R["last_u"].append(last_u); R["u_ref"].append(ua)
        R["agree"].append(agree); R["viol"].append(max(va, vb_)); R["f_ref"].append(fa)
        if agree < 1e-8 and max(va, vb_) < 1e-8:
            kept += 1
    np.savez_compressed(os.path.join(OUT, "g3_synthetic_dd.npz"), **{k: np.asarray(v) for k, v in R.items()})
    print(f"g3 synthetic dd: {n_cases} scenes, both scipy methods agree <1e-8 on {kept}")


def _oracle_derivs(P, N):
    """Analytic gradient / Jacobian of the reference LIP_Prob at horizon N (the reference's own
    gradient/jacobian are N=3-only).  Built from what solveMPCCBF handed to cyipopt (selected obstacles,
    goal after the detour, x0) by the numpy restatement, whose derivatives the CPU suite pins to central
    finite differences of the reference objective/constraints (tests/test_oracle.py)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
    import np_oracle as O
    po = P.problem_obj
    cfg = O.default_cfg(O.VARIANT_MODI, N, select_obs=0, detour=0, nc_max=12, ne_max=12)
    cir = np.asarray(po.cir_modi_pram, float).reshape(-1, 3)
    elp = np.asarray(po.elp_modi_pram, float).reshape(-1, 5)
    prob = O.Problem(cfg, np.ravel(po.xk), np.ravel(po.goal), 1, cir, elp)
    return prob.gradient, prob.jacobian


def _sample_scene_bounded(rand_obs, seed, num, typ, seconds=2):
    """sample_scene, or None when rand_obs' rejection loop does not finish within `seconds`."""
    import signal

    def _raise(*_):
        raise TimeoutError

    old = signal.signal(signal.SIGALRM, _raise)
    signal.alarm(seconds)
    try:
        return sample_scene(rand_obs, seed, num, typ)
    except TimeoutError:
        return None
    finally:
        signal.alarm(0)
        signal.signal(signal.SIGALRM, old)


def gen_g3_synthetic_modi_n5(modi, rand_obs, n_cases):
    """BASELINE cfg3 shape (N = 5, 5 circles + 5 ellipses): scenes solved by SLSQP and trust-constr on the
    reference objective/constraints (MPC_LIP_modi.py:430-500, which loop over N) built by the reference's
    own MPCCBF(step=5) set-up (select_obs, cl/cu, detour goal); derivatives from _oracle_derivs."""
    rng = np.random.default_rng(780)
    margin = [-0.5, 10.5]
    N = 5
    R = {k: [] for k in ["x0", "leg", "goal", "cir", "nc", "elp", "ne", "u0", "u_ref", "foot_ref", "agree",
                         "viol"]}
    kept = 0
    t = -1
    while len(R["x0"]) < n_cases:
        t += 1
        scene = _sample_scene_bounded(rand_obs, 5000 + t, 10, "mix")
        if scene is None:      # rejection sampling of 10 separated circles can fail to terminate
            continue
        cir, elp = scene
        cs, es = inflate(cir, elp)
        x0, leg = sample_state(rng, cs, es)
        goal = [[10.0, 10.0]]
        u0 = np.tile(x0, N)
        res = []
        for fn in (solve_slsqp, solve_trust):
            def run(P, fn=fn):
                g, J = _oracle_derivs(P, N)
                po = P.problem_obj

                class _Prob:   # reference f and c, analytic derivatives at any N
                    objective = staticmethod(po.objective)
                    constraints = staticmethod(po.constraints)
                    gradient = staticmethod(g)
                    jacobian = staticmethod(J)
                return fn(_Prob, P.u0, P.cl, P.cu)
            _StubProblem.solver = _wrap_solver(run)
            mpc = modi.MPCCBF(goal, cir, cs, elp, es, margin, step=N)
            out = mpc.gen_control_test(x0, leg, u0)
            P = _StubProblem.last
            u = _last_solution[0].copy()
            c = np.asarray(P.problem_obj.constraints(u), float)
            res.append((u, np.ravel(out[1]), violation(c, P.cl, P.cu)))
        _StubProblem.solver = None
        (ua, pa, va), (ub_, pb, vb) = res
        agree = float(np.max(np.abs(pa - pb)))
        R["x0"].append(x0); R["leg"].append(leg); R["goal"].append(np.array([10.0, 10.0]))
        R["cir"].append(_pad(cs, 5, 3)); R["nc"].append(len(cs))
        R["elp"].append(_pad(es, 5, 5)); R["ne"].append(len(es))
        R["u0"].append(u0); R["u_ref"].append(ua); R["foot_ref"].append(pa)
        R["agree"].append(agree); R["viol"].append(max(va, vb))
        if agree < 1e-8 and max(va, vb) < 1e-8:
            kept += 1
    np.savez_compressed(os.path.join(OUT, "g3_synthetic_modi_n5.npz"), **{k: np.asarray(v) for k, v in R.items()})
    print(f"g3 synthetic modi N=5: {n_cases} scenes, both scipy methods agree <1e-8 on {kept}")


def gen_g3_sig_step_nobs(sig, n_cases):
    """BASELINE cfg1 (MPC_LIP_sig_step.py, N = 3, no obstacles): the reference set-up and callbacks
    (MPC_LIP_sig_step.py:184-278, 372-496), solved by SLSQP and trust-constr; warm start None ->
    [x0, x0, x0] as the reference does (:186-187)."""
    rng = np.random.default_rng(781)
    margin = [-0.5, 10.5]
    R = {k: [] for k in ["x0", "leg", "goal", "u0", "u_ref", "foot_ref", "agree", "viol"]}
    kept = 0
    for t in range(n_cases):
        x0, leg = sample_state(rng, np.zeros((0, 3)), np.zeros((0, 5)))
        goal = [[10.0, 10.0]] if t % 4 else [list(rng.uniform(3.0, 10.0, 2))]
        res = []
        for fn in (solve_slsqp, solve_trust):
            _StubProblem.solver = _wrap_solver(lambda P, fn=fn: fn(P.problem_obj, P.u0, P.cl, P.cu))
            mpc = sig.MPCCBF(goal, [], [], margin)
            out = mpc.gen_control_test(x0, leg, None)
            P = _StubProblem.last
            u = _last_solution[0].copy()
            c = np.asarray(P.problem_obj.constraints(u), float)
            res.append((u, np.ravel(out[1]), violation(c, P.cl, P.cu)))
        _StubProblem.solver = None
        (ua, pa, va), (ub_, pb, vb) = res
        agree = float(np.max(np.abs(pa - pb)))
        R["x0"].append(x0); R["leg"].append(leg); R["goal"].append(np.ravel(goal))
        R["u0"].append(np.tile(x0, 3)); R["u_ref"].append(ua); R["foot_ref"].append(pa)
        R["agree"].append(agree); R["viol"].append(max(va, vb))
        if agree < 1e-8 and max(va, vb) < 1e-8:
            kept += 1
    np.savez_compressed(os.path.join(OUT, "g3_synthetic_sig_step_nobs.npz"),
                        **{k: np.asarray(v) for k, v in R.items()})
    print(f"g3 synthetic sig_step, no obstacles: {n_cases} scenes, both scipy methods agree <1e-8 on {kept}")


# ----------------------------------------------------------------------------------------------
def gen_g4(modi, sig):
    rng = np.random.default_rng(99)
    mpc = modi.MPCCBF([[10, 10]], [], [], [], [], [-0.5, 10.5])
    R = {"A": np.asarray(mpc.A), "B": np.asarray(mpc.B), "W": np.asarray(mpc.W),
         "M_A": np.asarray(mpc.M_A), "M_B": np.asarray(mpc.M_B), "dx_du": np.asarray(mpc.dx_du),
         "dP_du": np.asarray(mpc.dP_du), "sigma": mpc.sigma, "inv_B_vel_shr": np.asarray(mpc.inv_B_vel_shr)}
    gns_in, gns_out, trk = [], [], []
    for t in range(24):
        pos = rng.uniform(0, 10, 2); vel = rng.uniform(-0.5, 0.8, 2); hd = rng.uniform(-1, 1.5)
        p = np.array([*(pos + rng.normal(0, 0.1, 2)), rng.uniform(-0.2, 0.2)])
        tr = [0.4, 0.35, 0.3, 0.0125, 0.01, 0.0][t % 6] if t < 6 else rng.uniform(0.0, 0.4)
        xn, det = mpc.get_next_states(pos, vel, hd, p, tr)
        gns_in.append(np.concatenate([pos, vel, [hd], p, [tr]])); gns_out.append(xn)
        trk.append(_pad(det, 50, 2)); R.setdefault("trk_len", []).append(len(det))
    R["gns_in"] = np.array(gns_in); R["gns_out"] = np.array(gns_out); R["trk"] = np.array(trk)
    R["trk_len"] = np.array(R["trk_len"])
    adv = []
    for vx in [0.4, 0.6, 0.8]:
        for leg in [-1, 1]:
            adv.append([vx, leg, *mpc.alip_des_vel(vx, leg)])
    R["alip_des_vel"] = np.array(adv)
    cf_in, cf_out = [], []
    for t in range(10):
        x = rng.normal(0, 1, 5); v = rng.normal(0, 0.5, 2)
        cf_in.append(np.concatenate([x, v])); cf_out.append(mpc.cal_foot_with_veldes(x, v))
    R["cfv_in"] = np.array(cf_in); R["cfv_out"] = np.array(cf_out)
    hl, tv, tout = [], [], []
    for t in range(8):
        h = rng.normal(0, 0.3, 6); v0 = rng.normal(0, 0.2)
        hl.append(h); tv.append(v0); tout.append(mpc.tube_func(h, v0))
    R["tube_in"] = np.array(hl); R["tube_init"] = np.array(tv); R["tube_out"] = np.array(tout)
    np.savez_compressed(os.path.join(OUT, "g4_aux.npz"), **R)
    print("g4 aux written")


def gen_g5_logger():
    """Caller-side helpers of the planner -> controller interface in data_procs/logger_mpc.py (Logger):
    angle_A_minus_B (:169-175), tube_func (:283-300), avg_hd (:208-215), the frame transforms
    pos/vel_map_glo_2_robo_glo (:134-150), the foot-frame inputs of gen_nex_foot_input (:349-360, inline
    code: restated on the same attributes) and gen_tsc_control (:374-384)."""
    import contextlib
    import io
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_logger_mpc", os.path.join(REF, "data_procs", "logger_mpc.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    rng = np.random.default_rng(123)
    R = {}
    lg = mod.Logger(0.4, [0.3, -0.2], 0.25, [[10, 10]], [-0.5, 10.5])
    ab = rng.uniform(-7, 7, (40, 2))
    R["amb_in"] = ab
    R["amb_out"] = np.array([lg.angle_A_minus_B(a, b) for a, b in ab])
    tin = np.concatenate([rng.uniform(-0.4, 0.4, (30, 2)), [[0.0, 0.3], [0.15, 0.1], [-0.15, 0.2]]])
    R["tube_in"] = tin
    with contextlib.redirect_stdout(io.StringIO()):
        R["tube_out"] = np.array([lg.tube_func(t, v) for t, v in tin])
    av_in, av_out = [], []
    for _ in range(20):
        cur, turn = rng.uniform(-3, 3), rng.uniform(-0.2, 0.2)
        hds = rng.uniform(-3.5, 3.5, 3)
        lg.nex_turn = turn
        lg.mpc_hds_list = list(hds)
        av_in.append([cur, turn, *hds]); av_out.append(lg.avg_hd(cur))
    R["avg_in"] = np.array(av_in); R["avg_out"] = np.array(av_out)
    pv = rng.normal(0, 3, (12, 2))
    R["frame_in"] = pv
    R["pos_m2r"] = np.array([lg.pos_map_glo_2_robo_glo(v) for v in pv])
    R["vel_m2r"] = np.array([lg.vel_map_glo_2_robo_glo(v) for v in pv])
    ts_in, ts_out = [], []
    for t in range(16):
        lg.foot_input = rng.normal(0, 0.3, 2); lg.nex_pos_fot_loc = rng.normal(0, 0.2, 2)
        lg.nex_vel_fot_loc = rng.normal(0, 0.5, 2); lg.hd_input_pr = rng.uniform(-0.3, 0.3)
        lg.hd_input_cos = rng.uniform(-3, 3)
        i, n_cyc = int(rng.integers(0, 40)), 40
        ts_in.append([*lg.foot_input, *lg.nex_pos_fot_loc, *lg.nex_vel_fot_loc, lg.hd_input_pr, lg.hd_input_cos, i,
                      n_cyc])
        ts_out.append(lg.gen_tsc_control(i, n_cyc))
    R["tsc_in"] = np.array(ts_in); R["tsc_out"] = np.array(ts_out)
    np.savez_compressed(os.path.join(OUT, "g5_logger.npz"), **R)
    print("g5 logger written")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    if not os.path.isdir(REF):
        print("reference not present; nothing to do")
        return 0
    os.makedirs(OUT, exist_ok=True)
    modi, sig, dd, rand_obs = import_reference()
    only = set(a.only.split(",")) if a.only else None
    if not only or "g1" in only:
        gen_g1(modi, sig, dd, rand_obs, 24 if a.quick else 64)
    if not only or "g2" in only:
        gen_g2(modi, sig, rand_obs, 24 if a.quick else 64)
    if not only or "g4" in only:
        gen_g4(modi, sig)
    if not only or "g5" in only:
        gen_g5_logger()
    if not only or "g3s" in only:
        gen_g3_sup_learn(modi, a.quick)
    if not only or "g3y" in only:
        gen_g3_synthetic(modi, sig, rand_obs, 16 if a.quick else 48, "modi")
        gen_g3_synthetic(modi, sig, rand_obs, 16 if a.quick else 48, "sig_step")
    if not only or "g3dd" in only:
        gen_g3_synthetic_dd(dd, rand_obs, 16 if a.quick else 48)
    if not only or "g3n5" in only:
        gen_g3_synthetic_modi_n5(modi, rand_obs, 12 if a.quick else 128)
    if not only or "g3nobs" in only:
        gen_g3_sig_step_nobs(sig, 12 if a.quick else 48)
    return 0


if __name__ == "__main__":
    sys.exit(main())
