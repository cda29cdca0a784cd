"""Planner -> task-space-controller command packing, batched.

The reference's caller turns each MPC solve into the 8-vector high-level action of the (closed-source)
Digit task-space controller inside data_procs/logger_mpc.py (Logger).  These are the same formulas
vectorised over a batch of B robots (numpy; they are per-solve O(1) work next to the batched solve):

  angle_a_minus_b      Logger.angle_A_minus_B      logger_mpc.py:169-175
  tube_step            Logger.tube_func            logger_mpc.py:283-300 (heading tube of set_stf_head)
  avg_hd               Logger.avg_hd               logger_mpc.py:208-215 (turn command hd_input_pr)
  map_to_robot_pos/vel Logger.pos/vel_map_glo_2_robo_glo  logger_mpc.py:134-150
  foot_frame_inputs    gen_nex_foot_input's foot_input / nex_pos_fot_loc / nex_vel_fot_loc
                                                   logger_mpc.py:349-360
  gen_tsc_control      Logger.gen_tsc_control      logger_mpc.py:374-384
"""
import numpy as np


def angle_a_minus_b(a, b):
    """A - B wrapped once into [-pi, pi] as the reference does (one 2 pi correction)."""
    r = np.asarray(a, float) - np.asarray(b, float)
    big = np.abs(r) > np.pi
    return np.where(big & (r < 0), r + 2 * np.pi, np.where(big & (r > 0), r - 2 * np.pi, r))


def tube_step(turning, init_tube_value):
    """One heading-tube update: +0.4 * turn inside |turn| < 0.15, +0.7 * turn outside; returned relative to
    init_tube_value (angle_A_minus_B)."""
    d = np.asarray(turning, float)
    v0 = np.asarray(init_tube_value, float)
    inside = np.where(d > 0, 0.15 > d, -0.15 < d)
    tube = v0 + np.where(d == 0, 0.0, np.where(inside, 0.4, 0.7) * d)
    return angle_a_minus_b(tube, v0)


def avg_hd(cur_hd, nex_turn, mpc_hds):
    """Turn command: (nex_turn + sum_i angle(mpc_hds[i] - [cur_hd, mpc_hds[0], mpc_hds[1]][i])) / 4.
    cur_hd (B,), nex_turn (B,), mpc_hds (B, >=3) = the plan's headings (hd_list of gen_control_test)."""
    h = np.asarray(mpc_hds, float)
    cur = np.asarray(cur_hd, float)
    prev = np.stack([cur, h[..., 0], h[..., 1]], axis=-1)
    return (np.asarray(nex_turn, float) + angle_a_minus_b(h[..., :3], prev).sum(-1)) / 4.0


def _rot(theta):
    c, s = np.cos(theta), np.sin(theta)
    return np.stack([np.stack([c, s], -1), np.stack([-s, c], -1)], -2)   # [[c, s], [-s, c]]


def map_to_robot_pos(pos_map, map_init, hd_init):
    return np.einsum("...ij,...j->...i", _rot(np.asarray(hd_init, float)), np.asarray(pos_map, float) -
                     np.asarray(map_init, float))


def map_to_robot_vel(vel_map, hd_init):
    return np.einsum("...ij,...j->...i", _rot(np.asarray(hd_init, float)), np.asarray(vel_map, float))


def foot_frame_inputs(nex_stf_rob, cur_stf_rob, cur_base_ang, nex_pos_rob, nex_vel_rob):
    """Next foothold / CoM position / CoM velocity in the current stance-foot frame rotated by the base
    heading: foot_input = M_T (p_next - p_stance), nex_pos_fot_loc = M_T (x_pos - p_stance),
    nex_vel_fot_loc = M_T v_des, M_T = [[cos, sin], [-sin, cos]](base angle)."""
    M = _rot(np.asarray(cur_base_ang, float))
    cur = np.asarray(cur_stf_rob, float)
    mv = lambda v: np.einsum("...ij,...j->...i", M, v)   # noqa: E731
    return (mv(np.asarray(nex_stf_rob, float) - cur), mv(np.asarray(nex_pos_rob, float) - cur),
            mv(np.asarray(nex_vel_rob, float)))


def gen_tsc_control(foot_input, nex_pos_fot_loc, nex_vel_fot_loc, hd_input_pr, hd_input_cos, i, n_cyc):
    """High-level action [foot x, foot y, 0, heading(i), com x, com y, com vx, 0] for control tick i of
    n_cyc; heading ramps as hd_input_pr / n_cyc * (i + 4.5) + hd_input_cos.  Returns (B, 8)."""
    fi = np.asarray(foot_input, float)
    npf = np.asarray(nex_pos_fot_loc, float)
    nvf = np.asarray(nex_vel_fot_loc, float)
    hd = np.asarray(hd_input_pr, float) / np.asarray(n_cyc, float) * (np.asarray(i, float) + 4.5) + \
        np.asarray(hd_input_cos, float)
    z = np.zeros_like(hd)
    return np.stack([fi[..., 0], fi[..., 1], z, hd, npf[..., 0], npf[..., 1], nvf[..., 0], z], axis=-1)
