"""CPU: the oracle (numpy + C restatements) pinned against the reference's own outputs (tests/golden,
generated from /root/reference by tools/gen_goldens.py) and the recorded cyipopt solutions (sup_learn)."""
import math

import numpy as np
import pytest

import np_oracle as O

REL = 1e-12


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b) / (1.0 + np.abs(b)))) if a.size else 0.0


@pytest.mark.parametrize("name,variant", [("modi", 0), ("sig_step", 1)])
def test_numpy_callbacks_match_reference(golden, name, variant):
    g = golden(f"g1_callbacks_{name}")
    cfg = O.default_cfg(variant, select_obs=0, detour=0)
    for t in range(len(g["f"])):
        nc, ne, m = g["nc"][t], g["ne"][t], g["m"][t]
        pr = O.Problem(cfg, g["x0"][t], g["goal"][t], 1, g["cir"][t][:nc], g["elp"][t][:ne])
        u = g["u"][t]
        assert rel(pr.objective(u), g["f"][t]) < REL
        assert rel(pr.gradient(u), g["grad"][t]) < REL
        assert rel(pr.constraints(u), g["c"][t][:m]) < REL
        assert rel(pr.jacobian(u), g["J"][t][:m]) < REL


@pytest.mark.parametrize("name,variant", [("modi", 0), ("sig_step", 1)])
def test_c_oracle_eval_matches_reference(golden, coracle, name, variant):
    g = golden(f"g1_callbacks_{name}")
    cfg = coracle.default_cfg(variant, select_obs=0, detour=0)
    B = len(g["f"])
    o = coracle.eval_batch(cfg, g["x0"], g["goal"], np.ones(B), g["cir"], g["nc"], g["elp"], g["ne"], g["u"])
    assert rel(o["f"], g["f"]) < REL
    assert rel(o["grad"], g["grad"]) < REL
    for t in range(B):
        act = o["row_active"][t].astype(bool)
        m = g["m"][t]
        assert act.sum() == m
        assert rel(o["c"][t][act], g["c"][t][:m]) < REL
        assert rel(o["J"][t][act], g["J"][t][:m]) < REL


def test_horizon5_values_and_fd_derivatives(golden, coracle):
    """N=5: the reference objective/constraints loop over N (pinned exactly); its gradient/jacobian are
    N=3-only, so the generalised derivatives are pinned by central differences."""
    g = golden("g1_callbacks_modi_n5")
    cfg = O.default_cfg(0, N=5, select_obs=0, detour=0)
    for t in range(len(g["f"])):
        nc, ne, m = g["nc"][t], g["ne"][t], g["m"][t]
        pr = O.Problem(cfg, g["x0"][t], g["goal"][t], 1, g["cir"][t][:nc], g["elp"][t][:ne])
        u = g["u"][t]
        assert rel(pr.objective(u), g["f"][t]) < REL
        assert rel(pr.constraints(u), g["c"][t][:m]) < REL
        if t < 6:
            h = 1e-6
            E = np.eye(pr.n)
            gfd = np.array([(pr.objective(u + h * e) - pr.objective(u - h * e)) / (2 * h) for e in E])
            Jfd = np.array([(pr.constraints(u + h * e) - pr.constraints(u - h * e)) / (2 * h) for e in E]).T
            assert np.max(np.abs(gfd - pr.gradient(u))) < 1e-5 * (1 + np.max(np.abs(gfd)))
            assert np.max(np.abs(Jfd - pr.jacobian(u))) < 1e-5 * (1 + np.max(np.abs(Jfd)))
    # the C oracle agrees with the numpy restatement at N=5
    cc = coracle.default_cfg(0, 5, nc_max=10, ne_max=10, select_obs=0, detour=0)
    B = len(g["f"])
    o = coracle.eval_batch(cc, g["x0"], g["goal"], np.ones(B), g["cir"], g["nc"], g["elp"], g["ne"], g["u"])
    assert rel(o["f"], g["f"]) < REL


def test_hessian_matches_finite_differences(golden):
    g = golden("g1_callbacks_modi")
    rng = np.random.default_rng(3)
    for t in [1, 5, 9]:
        cfg = O.default_cfg(0, select_obs=0, detour=0)
        nc, ne = g["nc"][t], g["ne"][t]
        pr = O.Problem(cfg, g["x0"][t], g["goal"][t], 1, g["cir"][t][:nc], g["elp"][t][:ne])
        u = g["u"][t]
        y = rng.normal(size=pr.m)
        L = lambda v: pr.gradient(v) - pr.jacobian(v).T @ y
        h = 1e-6
        Hfd = np.array([(L(u + h * e) - L(u - h * e)) / (2 * h) for e in np.eye(pr.n)])
        assert np.max(np.abs(Hfd - pr.hessian(u, y))) < 1e-5 * (1 + np.max(np.abs(Hfd)))


@pytest.mark.parametrize("name,variant", [("modi", 0), ("sig_step", 1)])
def test_setup_matches_reference(golden, coracle, name, variant):
    """cl/cu with leg parity, select_obs, detour goal (MPC_LIP_modi.py:197-271, 325-338)."""
    g = golden(f"g2_setup_{name}")
    cfg = O.default_cfg(variant)
    B = len(g["m"])
    for t in range(B):
        nc, ne, m = g["nc"][t], g["ne"][t], g["m"][t]
        pr = O.Problem(cfg, g["x0"][t], g["goal"][t], g["leg"][t], g["cir"][t][:nc], g["elp"][t][:ne])
        assert pr.m == m
        assert np.array_equal(pr.cl, g["cl"][t][:m]) and np.array_equal(pr.cu, g["cu"][t][:m])
        assert np.allclose(pr.goal, g["goal_eff"][t], rtol=0, atol=1e-14)
        assert list(pr.sel_cir) == list(np.nonzero(g["sel_cir"][t])[0])
        assert list(pr.sel_elp) == list(np.nonzero(g["sel_elp"][t])[0])
    cc = coracle.default_cfg(variant)
    o = coracle.eval_batch(cc, g["x0"], g["goal"], g["leg"], g["cir"], g["nc"], g["elp"], g["ne"],
                           np.tile(g["x0"], (1, 3)))
    for t in range(B):
        act = o["row_active"][t].astype(bool)
        m = g["m"][t]
        assert act.sum() == m
        assert np.array_equal(o["cl"][t][act], g["cl"][t][:m])
        assert np.array_equal(o["cu"][t][act], g["cu"][t][:m])
        assert np.allclose(o["goal_eff"][t], g["goal_eff"][t], rtol=0, atol=1e-14)
    assert np.sum(np.any(g["goal_eff"] != g["goal"], axis=1)) > 0     # the detour branch is exercised


def test_constants_match_reference(golden):
    g = golden("g4_aux")
    K = O.Consts(O.default_cfg(0))
    for name, ours in [("A", K.A), ("B", K.B), ("W", K.W), ("M_A", K.MA), ("M_B", K.MB)]:
        assert rel(ours, g[name]) < 1e-14, name
    dx = np.concatenate([K.Phi[k] for k in range(4)])
    dp = np.concatenate([K.Psi[k] for k in range(3)])
    assert rel(dx, g["dx_du"]) < 1e-14
    assert rel(dp, g["dP_du"]) < 1e-14


def test_sup_learn_recorded_cyipopt_solutions(golden, coracle):
    """The 640 recorded cyipopt calls (logger_iml.py:342-401).  On the rows a converged solve of the
    reference NLP reproduces (ok_ref), the oracle's foothold matches the LOGGED cyipopt foothold to 1e-4
    except where it lands in a different local minimum (nonconvex CBF/atan2 terms); status 2 only where
    the reference solve is infeasible too."""
    d = golden("g3_sup_learn")
    B = len(d["leg"])
    cfg = coracle.default_cfg(0, nc_max=6, ne_max=0, max_iter=100)   # to convergence (reference cap: 30)
    cir = np.tile(d["cir_safe"], (B, 1, 1))
    r = coracle.solve_batch(cfg, d["x_nex"], [10, 10], d["leg"], cir, np.full(B, 6), None, None, d["u0"], nthreads=8)
    ok = d["ok_ref"].astype(bool)
    err = np.max(np.abs(r["foot"][:, :2] - d["foot_logged"]), axis=1)
    assert (err[ok] < 1e-4).sum() >= int(0.97 * ok.sum()), ((err[ok] < 1e-4).sum(), ok.sum())
    assert (err < 1e-4).sum() >= 470
    assert (r["status"] == 0).sum() >= 530


@pytest.mark.parametrize("variant,name", [(0, "modi"), (1, "sig_step")])
def test_synthetic_scipy_solutions(golden, coracle, variant, name):
    d = golden(f"g3_synthetic_{name}")
    good = (d["agree"] < 1e-8) & (d["viol"] < 1e-8)
    B = len(d["leg"])
    cfg = coracle.default_cfg(variant, nc_max=6, ne_max=6, max_iter=100)   # to convergence
    r = coracle.solve_batch(cfg, d["x0"], d["goal"], d["leg"], d["cir"], d["nc"], d["elp"], d["ne"], d["u0"])
    err = np.max(np.abs(r["foot"] - d["foot_ref"]), axis=1)
    assert good.sum() >= 20
    assert np.all(err[good] < 1e-4), err[good].max()


def test_synthetic_scipy_solutions_horizon5(golden, coracle):
    """BASELINE cfg3 shape (N = 5, 5 circles + 5 ellipses): the C oracle lands on the KKT point SLSQP and
    trust-constr find on the reference objective/constraints (g3_synthetic_modi_n5, tools/gen_goldens.py)."""
    d = golden("g3_synthetic_modi_n5")
    good = (d["agree"] < 1e-8) & (d["viol"] < 1e-8)
    cfg = coracle.default_cfg(0, 5, nc_max=5, ne_max=5, max_iter=100)
    r = coracle.solve_batch(cfg, d["x0"], d["goal"], d["leg"], d["cir"], d["nc"], d["elp"], d["ne"], d["u0"])
    err = np.max(np.abs(r["foot"] - d["foot_ref"]), axis=1)
    assert good.sum() >= 30
    assert np.all(r["status"][good] == 0)
    assert np.all(err[good] < 1e-6), err[good].max()


def test_sig_step_no_obstacle_solutions(golden, coracle):
    """BASELINE cfg1 (sig_step, N = 3, no obstacles): C oracle vs SLSQP / trust-constr on the reference."""
    d = golden("g3_synthetic_sig_step_nobs")
    good = (d["agree"] < 1e-8) & (d["viol"] < 1e-8)
    B = len(d["x0"])
    cfg = coracle.default_cfg(1, 3, nc_max=0, ne_max=0, max_iter=100)
    r = coracle.solve_batch(cfg, d["x0"], d["goal"], d["leg"], np.zeros((B, 0, 3)), np.zeros(B, np.int32),
                            None, None, d["u0"])
    err = np.max(np.abs(r["foot"] - d["foot_ref"]), axis=1)
    assert good.sum() >= 30
    assert np.all(err[good] < 1e-6), err[good].max()


def test_numpy_and_c_oracles_agree(golden, coracle):
    d = golden("g3_sup_learn")
    idx = np.arange(0, 640, 16)
    cfg = coracle.default_cfg(0, nc_max=6, ne_max=0)
    cir = np.tile(d["cir_safe"], (len(idx), 1, 1))
    r = coracle.solve_batch(cfg, d["x_nex"][idx], [10, 10], d["leg"][idx], cir, np.full(len(idx), 6), None, None,
                            d["u0"][idx])
    pcfg = O.default_cfg(0)
    agree = 0
    for j, i in enumerate(idx):
        pr = O.Problem(pcfg, d["x_nex"][i], [10, 10], d["leg"][i], d["cir_safe"], np.zeros((0, 5)))
        u, st, it = O.solve_footholds(pr, d["u0"][i])
        if st == r["status"][j] and (st != 0 or np.max(np.abs(u - r["u"][j])) < 1e-6):
            agree += 1
    assert agree >= int(0.9 * len(idx))


# ---------------------------------------------------------------- DD variant (MPC_DD_sig_step.py)
def test_dd_callbacks_match_reference(golden, coracle):
    """numpy + C restatements of the DD LIP_Prob callbacks (MPC_DD_sig_step.py:351-477) vs the goldens."""
    g = golden("g1_callbacks_dd")
    cfg = O.default_cfg(2)
    for t in range(len(g["f"])):
        nc, ne, m = g["nc"][t], g["ne"][t], g["m"][t]
        pr = O.DDProblem(cfg, g["x0"][t], g["goal"][t], g["cir"][t][:nc], g["elp"][t][:ne], g["last_u"][t])
        u = g["u"][t]
        assert rel(pr.objective(u), g["f"][t]) < REL
        assert rel(pr.gradient(u), g["grad"][t]) < REL
        assert rel(pr.constraints(u), g["c"][t][:m]) < REL
        assert rel(pr.jacobian(u), g["J"][t][:m]) < REL
    cc = coracle.default_cfg(2, nc_max=6, ne_max=6)
    r = coracle.eval_batch_dd(cc, g["x0"], g["goal"], g["cir"], g["nc"], g["elp"], g["ne"], g["u"], g["last_u"])
    assert rel(r["f"], g["f"]) < REL and rel(r["grad"], g["grad"]) < REL
    for t in range(len(g["f"])):
        act = r["row_active"][t].astype(bool)
        assert rel(r["c"][t][act], g["c"][t][:g["m"][t]]) < REL
        assert rel(r["J"][t][act], g["J"][t][:g["m"][t]]) < REL


def test_dd_hessian_matches_finite_differences(golden):
    g = golden("g1_callbacks_dd")
    cfg = O.default_cfg(2)
    rng = np.random.default_rng(5)
    for t in range(8):
        nc, ne = g["nc"][t], g["ne"][t]
        pr = O.DDProblem(cfg, g["x0"][t], g["goal"][t], g["cir"][t][:nc], g["elp"][t][:ne], g["last_u"][t],
                         split=True)
        u, y = g["u"][t], rng.normal(0, 1, pr.m)
        H = pr.hessian(u, y)
        L = lambda v: pr.gradient(v) - pr.jacobian(v).T @ y
        Hf = np.stack([(L(u + e) - L(u - e)) / 2e-6 for e in np.eye(pr.n) * 1e-6], 1)
        assert np.max(np.abs(H - Hf)) / (1 + np.max(np.abs(Hf))) < 1e-7


def test_dd_solutions_match_scipy_goldens(golden, coracle):
    """DD scenes solved by SLSQP and trust-constr on the reference callbacks (tools/gen_goldens.py g3dd)."""
    d = golden("g3_synthetic_dd")
    good = (d["agree"] < 1e-6) & (d["viol"] < 1e-8)
    assert good.sum() >= 20
    cfg = coracle.default_cfg(2, nc_max=6, ne_max=6, max_iter=100)   # to convergence (reference cap: 40)
    r = coracle.solve_batch_dd(cfg, d["x0"], d["goal"], d["cir"], d["nc"], d["elp"], d["ne"], d["u0"], d["last_u"])
    err = np.max(np.abs(r["u"] - d["u_ref"]), axis=1)
    assert np.all(err[good] < 1e-4), err[good].max()
    # numpy restatement agrees with the C one
    pcfg = O.default_cfg(2)
    for t in range(0, len(d["u0"]), 4):
        pr = O.DDProblem(pcfg, d["x0"][t], d["goal"][t], d["cir"][t][:d["nc"][t]], d["elp"][t][:d["ne"][t]],
                         d["last_u"][t])
        u, st, it = O.dd_solve(pr, d["u0"][t], max_iter=100)
        assert st == r["status"][t]
        if st == 0:
            assert np.max(np.abs(u - r["u"][t])) < 1e-6


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_rollout_oracle_semantics(coracle, variant):
    """Closed-loop rollout: step 0 is the plain solve, the plant executes the first planned
    step (x <- x_pred[0] = A x + B p_0, i.e. get_next_states over a full step), stance and warm start follow
    the reference drivers, and a goal-reached instance is retired."""
    import sys
    import math
    from alipmpc import scenes
    from alipmpc.planner import next_state
    dd = variant == 2
    N = 3
    bt = scenes.make_batch(24, seed=31 + variant, n_cir=3, N=N)
    cfg = coracle.default_cfg(variant, N, nc_max=3, ne_max=0)
    if dd:
        x0 = bt["x0"][:, [0, 1, 4]]
        u0 = np.tile([0.6, 0.0], (24, N))
        lu = np.tile([0.6, 0.0], (24, 1))
    else:
        x0, u0, lu = bt["x0"], bt["u0"], None
    # put a few instances right next to the goal so that they retire inside the horizon
    x0 = x0.copy()
    x0[:4, 0:2] = bt["goal"][:4] - np.array([0.25, 0.25])
    if not dd:
        u0 = np.tile(x0, (1, N))
    ro = coracle.rollout_batch(cfg, x0, bt["goal"], bt["leg"], bt["cir"], bt["nc"], None, None, u0, lu, steps=4,
                               nthreads=4)
    if dd:
        first = coracle.solve_batch_dd(cfg, x0, bt["goal"], bt["cir"], bt["nc"], None, None, u0, lu)
    else:
        first = coracle.solve_batch(cfg, x0, bt["goal"], bt["leg"], bt["cir"], bt["nc"], None, None, u0)
    assert np.array_equal(ro["foot"][:, 0], first["foot"])
    assert np.array_equal(ro["status"][:, 0], first["status"])
    assert np.array_equal(ro["x"][:, 1], first["x_pred"][:, 0])
    beta = math.sqrt(9.81)
    for b in range(24):
        for t in range(4):
            if ro["status"][b, t] == -10:
                assert np.isnan(ro["foot"][b, t]).all()
                assert np.array_equal(ro["x"][b, t + 1], ro["x"][b, t])
                continue
            if not dd:   # ideal ALIP plant == the reference's continuous flow over a full step
                xs = ro["x"][b, t]
                xn, _ = next_state(beta, 0.4, xs[0:2], xs[2:4], xs[4], ro["foot"][b, t], 0.4)
                assert np.allclose(xn, ro["x"][b, t + 1], rtol=0, atol=1e-12)
    reached = ro["steps_to_goal"] > 0
    assert reached[:4].any()
    for b in np.nonzero(reached)[0]:
        k = ro["steps_to_goal"][b]
        assert (ro["status"][b, k:] == -10).all() and (ro["status"][b, :k] != -10).all()


@pytest.mark.parametrize("variant", [0, 1])
def test_closed_loop_oracle_semantics(coracle, variant):
    """Closed loop at the control rate (main_sim_mpc.py:65-135): tick 0 solves at
    get_next_states(x, stance, rest_t = T) with od_ev = -leg_ind and the warm start [x_nex] x 3; the plant's f_cyc
    flows of T / f_cyc compose to one flow over T about the stance foot with the step's heading input hd_pr
    (= 0 on the first step: mpc_hds_list starts at the initial heading); touchdown moves the stance to the last
    solve's first foothold; an episode stops after the step on which close_2_goal first held."""
    import math
    from alipmpc import scenes
    from alipmpc.planner import next_state
    B, S, F = 16, 3, 8
    bt = scenes.make_batch(B, seed=41 + variant, n_cir=3)
    cfg = coracle.default_cfg(variant, 3, nc_max=3, ne_max=0)
    x0 = bt["x0"].copy()
    x0[:4, 0:2] = bt["goal"][:4] - np.array([0.5, 0.4])
    leg = bt["leg"].astype(np.int8)
    foot0 = coracle.solve_batch(cfg, x0, bt["goal"], leg, bt["cir"], bt["nc"], None, None,
                                np.tile(x0, (1, 3)))["foot"][:, 0:2]
    r = coracle.closed_loop_batch(cfg, x0, foot0, bt["goal"], leg, bt["cir"], bt["nc"], steps=S, f_cyc=F, nthreads=4)
    beta = math.sqrt(9.81)
    assert np.array_equal(r["hd"][:, 0, 0], np.zeros(B)) and np.array_equal(r["hd"][:, 0, 1], x0[:, 4])
    xn0 = np.stack([next_state(beta, 0.4, x0[b, 0:2], x0[b, 2:4], x0[b, 4], [*foot0[b], 0.0], 0.4)[0]
                    for b in range(B)])
    first = coracle.solve_batch(cfg, xn0, bt["goal"], -leg, bt["cir"], bt["nc"], None, None, np.tile(xn0, (1, 3)))
    assert np.array_equal(r["status"][:, 0, 0], first["status"])
    assert np.array_equal(r["iters"][:, 0, 0], first["iters"])
    # tick 0's controller command = the Logger's formulas (alipmpc.tsc, pinned to g5_logger) on the same inputs:
    # robot frame at the initial pose, vel_des = alip_des_vel(0.6, leg_ind), base angle 0 in that frame
    from alipmpc import tsc
    mp_des = np.stack([np.full(B, 0.0), np.zeros(B)], 1)
    beta_ = math.sqrt(9.81)
    sig = beta_ / math.tanh(0.4 * beta_ / 2)
    mp_des[:, 0] = sig * 0.6 * 0.4 / 2
    mp_des[:, 1] = 0.5 * (-0.5 * leg.astype(float) * 0.3) * (beta_ * math.sinh(beta_ * 0.4)) / (math.cosh(beta_ * 0.4) + 1)
    nex_stf = tsc.map_to_robot_pos(first["foot"][:, 0:2], x0[:, 0:2], x0[:, 4])
    cur_stf = tsc.map_to_robot_pos(foot0, x0[:, 0:2], x0[:, 4])
    nex_pos = tsc.map_to_robot_pos(xn0[:, 0:2], x0[:, 0:2], x0[:, 4])
    nex_vel = tsc.map_to_robot_vel(mp_des, x0[:, 4])
    fi, npf, nvf = tsc.foot_frame_inputs(nex_stf, cur_stf, np.zeros(B), nex_pos, nex_vel)
    act0 = tsc.gen_tsc_control(fi, npf, nvf, r["hd"][:, 0, 0], r["hd"][:, 0, 1] - x0[:, 4], 0, F)
    np.testing.assert_allclose(r["action"][:, 0, 0], act0, rtol=0, atol=1e-12)
    for b in range(B):
        stance = foot0[b]
        for s in range(S):
            if r["status"][b, s, 0] == -10:
                assert (r["status"][b, s] == -10).all() and np.array_equal(r["x"][b, s + 1], r["x"][b, s])
                continue
            xs = r["x"][b, s]
            xn, _ = next_state(beta, 0.4, xs[0:2], xs[2:4], xs[4], [*stance, r["hd"][b, s, 0]], 0.4)
            assert np.allclose(xn, r["x"][b, s + 1], rtol=0, atol=1e-9)
            stance = r["foot"][b, s, 0:2]
    reached = r["steps_to_goal"] > 0
    assert reached[:4].any()
    for b in np.nonzero(reached)[0]:
        k = r["steps_to_goal"][b]
        assert (r["status"][b, k:] == -10).all() and (r["status"][b, :k] != -10).all()


@pytest.mark.parametrize("variant", [0, 1])
def test_goal_singularity_guard(golden, coracle, variant):
    """where a planned state sits exactly on the goal, the target heading atan2(g - p) has
    0 / 0 derivatives (the reference's cal_dtar_ang_du, MPC_LIP_modi.py:650-655, returns NaN there); every
    implementation takes them as 0 — numpy and C oracles agree, gradient and Hessian finite — and a solve warm-started
    at such a plan proceeds (the r3 fp32 closed loop had stayed at Error_In_Step_Computation there).  Away from the
    goal nothing changes (the g1 goldens above)."""
    g = golden("g1_callbacks_modi")
    cfg = O.default_cfg(variant, select_obs=0, detour=0)
    x0, goal = g["x0"][0].copy(), np.array([10.0, 10.0])
    u = np.tile(x0, 3)
    u[10:12] = goal                                   # x_3 = u_3 (positions) exactly on the goal
    pr = O.Problem(cfg, x0, goal, 1, np.zeros((0, 3)), np.zeros((0, 5)))
    gr = pr.gradient(u)
    assert np.isfinite(gr).all() and np.isfinite(pr.hessian(u, np.zeros(pr.m))).all()
    cc = coracle.default_cfg(variant, 3, nc_max=0, ne_max=0, select_obs=0, detour=0)
    o = coracle.eval_batch(cc, x0[None], goal[None], np.ones(1), np.zeros((1, 0, 3)), np.zeros(1, np.int32), None,
                           None, u[None])
    assert rel(o["grad"][0], gr) < REL
    r = coracle.solve_batch(cc, x0[None], goal[None], np.ones(1, np.int8), np.zeros((1, 0, 3)), np.zeros(1, np.int32),
                            None, None, u[None])
    assert r["status"][0] != -3 and np.isfinite(r["u"]).all()


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_goal_singular_abort_semantics(coracle, variant):
    """cfg.goal_singular (include/alipmpc.h).  At a planned state exactly on the goal the reference's
    cal_dtar_ang_du (MPC_LIP_modi.py:650-655, MPC_DD_sig_step.py:527-531) divides 0 by 0: its gradient is NaN, which
    IPOPT's gradient evaluation rejects (Eval_Error) — Invalid_Number_Detected (-13) with that iterate returned.
    GOAL_SINGULAR_ABORT reproduces that path in both oracles; the default (ZERO) takes the derivatives as 0 and solves
    on.  The instance starts ON the singular point (x0 at the goal, zero warm start: every planned state at the goal
    with exact arithmetic)."""
    dd = variant == 2
    N = 3
    sd = 3 if dd else 5
    n = 2 * N if dd else 5 * N
    x0, goal, u0 = np.zeros(sd), np.zeros(2), np.zeros(n)
    cir = np.array([[3.0, 3.0, 0.5]])
    res = {}
    for gs in (0, 1):
        c = coracle.default_cfg(variant, N, nc_max=1, ne_max=0, goal_singular=gs)
        o = O.default_cfg(variant, N, nc_max=1, ne_max=0, goal_singular=gs)
        if dd:
            r = coracle.solve_batch_dd(c, x0[None], goal[None], cir[None], np.ones(1, np.int32), None, None,
                                       u0[None], np.zeros((1, 2)))
            pu, pst, pit = O.dd_solve(O.DDProblem(o, x0, goal, cir, np.zeros((0, 5)), np.zeros(2)), u0)
        else:
            r = coracle.solve_batch(c, x0[None], goal[None], np.ones(1, np.int8), cir[None], np.ones(1, np.int32),
                                    None, None, u0[None])
            pu, pst, pit = O.solve_footholds(O.Problem(o, x0, goal, 1, cir, np.zeros((0, 5))), u0)
        assert r["status"][0] == pst and r["iters"][0] == pit, (gs, r["status"][0], pst, r["iters"][0], pit)
        res[gs] = (r, pu)
    r1, pu1 = res[1]
    assert r1["status"][0] == -13 and r1["iters"][0] == 0
    # the starting iterate is returned (LIP: u_k = x_{k+1} of the zero footholds; DD: the controls)
    assert np.array_equal(r1["u"][0], np.zeros(n)) and np.array_equal(pu1, np.zeros(n))
    r0, pu0 = res[0]
    assert r0["status"][0] != -13 and r0["iters"][0] > 0 and np.isfinite(r0["u"]).all()
    assert np.abs(r0["u"][0] - pu0).max() <= 1e-6


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_nlp_scaling_semantics(coracle, variant):
    """IPOPT's default NLP scaling (nlp_scaling_method = gradient-based, nlp_scaling_max_gradient = 100; the reference
    sets no scaling option, MPC_LIP_modi.py:284-290, MPC_DD_sig_step.py:181-189): at the starting point, the objective is
    scaled by df = 100 / max|grad f(u0)| (the gradient in the reference's u) where that exceeds 100.  An instance started
    near the goal facing away from it (heading error ~2.5 rad: gradient > 100): both oracles scale, agree, and solve
    the same NLP as the unscaled oracle with weights q, p, r (and DD's smoothness weight) times df — the objective is
    linear in them.  Constraint gradients stay far below 100 in u, so no row is scaled (dc = 1, as both oracles assume)."""
    dd = variant == 2
    N = 3
    goal = np.array([5.0, 5.0])
    cir = np.array([[7.0, 4.0, 0.4], [3.0, 6.5, 0.3]])
    if dd:
        x0 = np.array([4.7, 4.8, np.pi + 0.9])
        last_u = np.array([0.5, 0.0])
        u0 = np.tile(last_u, N)
        o = O.default_cfg(variant, N, nc_max=2, ne_max=0)
        pr = O.DDProblem(o, x0, goal, cir, np.zeros((0, 5)), last_u, split=True)
        sp = O.ScaledProblem(pr, u0)
    else:
        x0 = np.array([4.7, 4.8, -0.3, -0.1, np.pi + 0.9])
        u0 = np.tile(x0, N)
        o = O.default_cfg(variant, N, nc_max=2, ne_max=0)
        pr = O.Problem(o, x0, goal, 1, cir, np.zeros((0, 5)))
        fp = O.FootholdProblem(pr.split_copy())
        sp = O.ScaledProblem(fp, fp.p_of_u(u0))
    df = sp.df
    assert 0.0 < df < 1.0, df
    assert sp.max_constraint_gradient < 10.0, sp.max_constraint_gradient
    c = coracle.default_cfg(variant, N, nc_max=2, ne_max=0)
    if dd:
        r = coracle.solve_batch_dd(c, x0[None], goal[None], cir[None], np.array([2], np.int32), None, None, u0[None],
                                   last_u[None])
        pu, pst, pit = O.dd_solve(O.DDProblem(o, x0, goal, cir, np.zeros((0, 5)), last_u), u0)
    else:
        r = coracle.solve_batch(c, x0[None], goal[None], np.ones(1, np.int8), cir[None], np.array([2], np.int32), None,
                                None, u0[None])
        pu, pst, pit = O.solve_footholds(pr, u0)
    assert r["status"][0] == pst and r["iters"][0] == pit
    assert np.abs(r["u"][0] - pu).max() <= 1e-9
    # the same NLP with the objective's weights scaled by df, solved without scaling (its gradient is then 100)
    kw = dict(q=o.q * df, p=o.p * df, r=o.r * df) | (dict(dd_t=o.dd_t * df) if dd else {})
    cs = coracle.default_cfg(variant, N, nc_max=2, ne_max=0, **kw)
    if dd:
        rs = coracle.solve_batch_dd(cs, x0[None], goal[None], cir[None], np.array([2], np.int32), None, None,
                                    u0[None], last_u[None])
    else:
        rs = coracle.solve_batch(cs, x0[None], goal[None], np.ones(1, np.int8), cir[None], np.array([2], np.int32),
                                 None, None, u0[None])
    assert rs["status"][0] == r["status"][0] and abs(int(rs["iters"][0]) - int(r["iters"][0])) <= 1
    assert np.abs(rs["u"][0] - r["u"][0]).max() <= 1e-6


def _chain(coracle, d, restoration, max_iter=30):
    """the 640 recorded calls as the warm-started chain the reference ran (logger_iml.py:333-342), C oracle"""
    cc = coracle.default_cfg(0, 3, nc_max=6, ne_max=0, max_iter=max_iter)
    cc.restoration = restoration
    n = len(d["leg"])
    feet, st, u = np.zeros((n, 3)), np.zeros(n, np.int32), d["u0"][0]
    for i in range(n):
        o = coracle.solve_batch(cc, d["x_nex"][i:i + 1], np.array([[10.0, 10.0]]), d["leg"][i:i + 1],
                                d["cir_safe"][None], np.array([6]), np.zeros((1, 0, 5)), np.zeros(1), u[None])
        feet[i], st[i], u = o["foot"][0], o["status"][0], o["u"][0]
    return np.max(np.abs(feet[:, :2] - d["foot_logged"]), axis=1), st


def test_restoration_phase_reproduces_recorded_calls(golden, coracle):
    """IPOPT's feasibility restoration phase (cfg.restoration = IPOPT, the default; np_oracle._resto / alipmpc_oracle.c
    oresto) against the rounds-1-5 substitute on the 640 recorded cyipopt calls of sup_learn replayed as the reference's
    warm-started chain: the restoration phase reproduces >= 30 more recorded footholds (<= 1e-4) than the substitute and
    loses none (measured 532 vs 479, profiles/r6/resto/resto_chain.json); the statuses the reference labels as
    failures (2) stay the same rows' (its Infeasible_Problem_Detected is what the logs call a failed plan)."""
    d = golden("g3_sup_learn")
    e_ip, s_ip = _chain(coracle, d, 0)
    e_sub, s_sub = _chain(coracle, d, 1)
    r_ip, r_sub = e_ip <= 1e-4, e_sub <= 1e-4
    assert r_ip.sum() >= 520 and r_sub.sum() >= 470, (r_ip.sum(), r_sub.sum())
    assert r_ip.sum() >= r_sub.sum() + 30
    assert not np.any(r_sub & ~r_ip), np.nonzero(r_sub & ~r_ip)[0]
    assert ((s_ip == 2) == (s_sub == 2)).mean() >= 0.97


def test_restoration_phase_numpy_and_c_agree(coracle):
    """The numpy and C restatements of the restoration phase agree on a batch with infeasible scenes (cfg2's shape):
    statuses equal, footholds within 1e-6 on >= 97 % (rounding-level differences in a nonconvex solve)."""
    import alipmpc.scenes as scenes
    B = 96
    bt = scenes.make_batch(B, seed=0, n_cir=5, N=3)
    cc = coracle.default_cfg(0, 3, nc_max=5, ne_max=0)
    ref = coracle.solve_batch(cc, bt["x0"], bt["goal"], bt["leg"], bt["cir"], bt["nc"], np.zeros((B, 0, 5)),
                              np.zeros(B), bt["u0"], nthreads=4)
    assert (ref["restorations"] > 0).sum() >= 5   # the batch exercises the phase
    feet, st = np.zeros((B, 3)), np.zeros(B, np.int32)
    cfg = O.default_cfg(0, 3, nc_max=5, ne_max=0)
    for i in range(B):
        pr = O.Problem(cfg, bt["x0"][i], bt["goal"][i], bt["leg"][i], bt["cir"][i][:bt["nc"][i]], np.zeros((0, 5)))
        u, st[i], _ = O.solve_footholds(pr, bt["u0"][i])
        feet[i] = O.plan(pr, u)[1]
    assert (st == ref["status"]).mean() >= 0.97
    assert np.mean(np.max(np.abs(feet - ref["foot"]), axis=1) <= 1e-6) >= 0.97


def test_restoration_phase_semantics():
    """The restoration phase's own contract (np_oracle._resto): from the failed point it returns either a point the
    original filter accepts with violation <= 0.9 theta_R ("ok"), a converged restoration problem with violation above
    1e-4 ("infeasible"), or the iteration cap; the iterations it used are counted in the solve's total."""
    import alipmpc.scenes as scenes
    bt = scenes.make_batch(64, seed=0, n_cir=5, N=3)
    cfg = O.default_cfg(0, 3, nc_max=5, ne_max=0)
    seen = {}
    orig = O._resto

    def spy(prob, x, s, zl, zu, mu_o, cl, cu, hl, hu, filt_o, theta_R, orig_phi, it, max_iter, tol, stats):
        r = orig(prob, x, s, zl, zu, mu_o, cl, cu, hl, hu, filt_o, theta_R, orig_phi, it, max_iter, tol, stats)
        code, x1, s1, _, _, it1 = r
        seen[code] = seen.get(code, 0) + 1
        assert it1 >= it and it1 <= max_iter
        c1 = prob.constraints(x1)
        if code == "ok" and it1 > it:
            th = float(np.abs(c1 - s1).sum())
            assert th <= 0.9 * theta_R * (1 + 1e-12) or th <= 1e-12
        return r
    O._resto = spy
    try:
        for i in range(64):
            pr = O.Problem(cfg, bt["x0"][i], bt["goal"][i], bt["leg"][i], bt["cir"][i][:bt["nc"][i]], np.zeros((0, 5)))
            O.solve_footholds(pr, bt["u0"][i])
    finally:
        O._resto = orig
    assert seen.get("ok", 0) >= 5, seen


def test_row_scaling_region():
    """IPOPT's gradient-based scaling would also scale a constraint row whose gradient at the starting point exceeds 100
    (nlp_scaling_max_gradient): the build scales the objective only.  Pinned here:
    (a) on the benchmark scene generators (cfg2 modi, cfg3 N = 5 with ellipses, sig_step with select_obs = 0) every row
    gradient stays below 4 in the reference's u (measured max 3.5 over 512 instances each), so no row would be scaled;
    (b) the region where the deviation applies exists and is flagged: a 4 x 5 m ellipse 25 m away with obstacle
    selection off (select_obs = 0) has a row gradient of ~190, and ScaledProblem.rows_over_max_gradient reports it;
    the same scene with the reference's modi selection drops the obstacle (no such row)."""
    from dataclasses import replace
    from alipmpc import scenes
    for variant, N, n_elp in ((0, 3, 0), (0, 5, 5), (1, 3, 0)):
        bt = scenes.make_batch(32, seed=0, n_cir=5, n_elp=n_elp, N=N)
        o = O.default_cfg(variant, N, nc_max=5, ne_max=n_elp)
        for i in range(32):
            elp = bt["elp"][i][:bt["ne"][i]] if n_elp else np.zeros((0, 5))
            pr = O.Problem(o, bt["x0"][i], bt["goal"][i], bt["leg"][i], bt["cir"][i][:bt["nc"][i]], elp)
            fp = O.FootholdProblem(pr.split_copy())
            sp = O.ScaledProblem(fp, fp.p_of_u(bt["u0"][i]))
            assert sp.max_constraint_gradient < 4.0 and sp.rows_over_max_gradient == 0, (variant, N, i)
    x0 = np.array([0.0, 0.0, 0.1, 0.0, 0.0])
    elp = np.array([[25.0, 3.0, 4.0, 5.0, 0.3]])
    over = {}
    for so in (0, 1):
        o = replace(O.default_cfg(0, 3, nc_max=0, ne_max=1), select_obs=so)
        pr = O.Problem(o, x0, np.array([5.0, 0.5]), 1, np.zeros((0, 3)), elp)
        fp = O.FootholdProblem(pr.split_copy())
        sp = O.ScaledProblem(fp, fp.p_of_u(np.tile(x0, 3)))
        over[so] = (sp.rows_over_max_gradient, sp.max_constraint_gradient)
    assert over[0][0] >= 1 and over[0][1] > 100.0, over
    assert over[1] == (0, over[1][1]) and over[1][1] < 4.0, over
