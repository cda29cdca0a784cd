"""Plan traces (gen_control_test pos_det, MPC_LIP_modi.py:102-122, 304-322) and data_log-compatible episode
logs (logger_mpc.py:439-474) — host side: numpy plan_traces, the writer/reader, on oracle rollouts."""
import numpy as np
import pytest

from alipmpc import datalog, planner


def test_alip_constants_match_reference(golden):
    g = golden("g4_aux")
    k = planner.alip_constants()
    for name in ("A", "B", "W", "M_A", "M_B"):
        assert np.max(np.abs(k[name] - g[name])) < 1e-14, name


def _consts():
    k = planner.alip_constants()
    return k["beta"], 0.4, k["A"], k["W"], k["M_A"], k["M_B"]


def test_plan_traces_shape_and_continuity(coracle):
    from alipmpc import scenes
    bt = scenes.make_batch(16, seed=5, n_cir=5)
    o = coracle.solve_batch(coracle.default_cfg(0, 3, nc_max=5, ne_max=0), bt["x0"], bt["goal"], bt["leg"],
                            bt["cir"], bt["nc"], None, None, bt["u0"])
    tr = planner.plan_traces(*_consts(), bt["x0"], o["u"])
    assert tr.shape == (16, 3, 42, 2)                       # 126 x 2 per plan, as the data_log pickles
    assert np.array_equal(tr[:, 0, 0], bt["x0"][:, 0:2])    # row 0 = x_k[0:2]
    assert np.max(np.abs(tr[:, :, 1] - tr[:, :, 0])) < 1e-15   # t = 0 sample = x_k
    # the t = dt sample (row 41) is the next planned state x_{k+1} (= u_k)
    xp = o["x_pred"]
    assert np.max(np.abs(tr[:, :, 41] - xp[:, :, 0:2])) < 1e-12
    assert np.max(np.abs(tr[:, 1:, 0] - xp[:, :-1, 0:2])) < 1e-12
    # a gen_control_test-style concatenation of xk_track_det per step gives the same rows
    k = planner.alip_constants()
    xk, rows = bt["x0"][3], []
    for i in range(3):
        uk = o["u"][3, 5 * i:5 * i + 5]
        rows.append(planner.track_det(k["beta"], xk, k["W"] @ (uk - k["A"] @ xk), 0.4))
        xk = k["M_A"] @ xk + k["M_B"] @ uk
    assert np.array_equal(np.concatenate(rows), tr[3].reshape(126, 2))


def test_episode_logs_roundtrip(coracle, tmp_path):
    from alipmpc import scenes
    bt = scenes.make_batch(6, seed=8, n_cir=5)
    x0 = bt["x0"].copy()
    x0[0, 0:2] = bt["goal"][0] - np.array([0.5, 0.4])       # episode 0 reaches the goal quickly
    S = 5
    roll = coracle.rollout_batch(coracle.default_cfg(0, 3, nc_max=5, ne_max=0), x0, bt["goal"], bt["leg"],
                                 bt["cir"], bt["nc"], None, None, np.tile(x0, (1, 3)), steps=S)
    assert roll["u"].shape == (6, S, 15)
    c = _consts()
    for b in range(6):
        logs = datalog.episode_logs(roll, b, lambda xs, us: planner.plan_traces(*c, xs, us),
                                    cir=bt["cir"][b] - np.array([0, 0, 0.4]))
        T = roll["steps_to_goal"][b] if roll["steps_to_goal"][b] > 0 else S
        assert len(logs["pred_full_end"]) == T
        assert all(p.shape == (126, 2) for p in logs["pred_full_end"])
        assert len(logs["pred_feasi_end"]) + len(logs["pred_fail_end"]) == T
        assert logs["pos"].shape == (40 * T, 2) and logs["time"].shape == (40 * T,)
        assert logs["foot"].shape == (40 * T, 2) and logs["heading"].shape == (40 * T,)
        assert np.array_equal(logs["real_end"], roll["x"][b, 1:T + 1, 0:2])
        assert np.allclose(logs["pos"][::40], roll["x"][b, :T, 0:2], rtol=0, atol=1e-12)
        # the tick after the last of step t continues into step t + 1 (the CoM path is continuous)
        if T > 1:
            nxt = planner.track_det(c[0], roll["x"][b, 0], roll["foot"][b, 0], 0.4)[41]
            assert np.allclose(nxt, logs["pos"][40], rtol=0, atol=1e-12)
        paths = datalog.write_data_log(str(tmp_path / f"ep{b}_"), logs)
        assert len(paths) == 13
        back = datalog.read_data_log(str(tmp_path / f"ep{b}_"))
        for k in datalog.NAMES:
            a, r = back[k], logs[k]
            if isinstance(r, list):
                assert len(a) == len(r) and all(np.array_equal(x, y) for x, y in zip(a, r))
            else:
                assert np.array_equal(np.asarray(a), np.asarray(r))
    assert (roll["steps_to_goal"][0] > 0)


def test_tsc_command_packing_matches_reference(golden):
    """Batched planner -> TSC command helpers against the reference Logger (logger_mpc.py), golden g5."""
    from alipmpc import tsc
    g = golden("g5_logger")
    assert np.max(np.abs(tsc.angle_a_minus_b(g["amb_in"][:, 0], g["amb_in"][:, 1]) - g["amb_out"])) < 1e-15
    assert np.max(np.abs(tsc.tube_step(g["tube_in"][:, 0], g["tube_in"][:, 1]) - g["tube_out"])) < 1e-15
    a = g["avg_in"]
    assert np.max(np.abs(tsc.avg_hd(a[:, 0], a[:, 1], a[:, 2:5]) - g["avg_out"])) < 1e-15
    assert np.max(np.abs(tsc.map_to_robot_pos(g["frame_in"], [0.3, -0.2], 0.25) - g["pos_m2r"])) < 1e-14
    assert np.max(np.abs(tsc.map_to_robot_vel(g["frame_in"], 0.25) - g["vel_m2r"])) < 1e-14
    t = g["tsc_in"]
    out = tsc.gen_tsc_control(t[:, 0:2], t[:, 2:4], t[:, 4:6], t[:, 6], t[:, 7], t[:, 8], t[:, 9])
    assert out.shape == (16, 8) and np.max(np.abs(out - g["tsc_out"])) < 1e-15


def test_foot_frame_inputs_geometry():
    from alipmpc import tsc
    rng = np.random.default_rng(4)
    nex, cur, pos, vel = (rng.normal(size=(10, 2)) for _ in range(4))
    ang = rng.uniform(-3, 3, 10)
    fi, npf, nvf = tsc.foot_frame_inputs(nex, cur, ang, pos, vel)
    for b in range(10):
        M_T = np.array([[np.cos(ang[b]), np.sin(ang[b])], [-np.sin(ang[b]), np.cos(ang[b])]])
        assert np.allclose(fi[b], M_T @ (nex[b] - cur[b]), rtol=0, atol=1e-15)
        assert np.allclose(npf[b], M_T @ (pos[b] - cur[b]), rtol=0, atol=1e-15)
        assert np.allclose(nvf[b], M_T @ vel[b], rtol=0, atol=1e-15)
