"""data_log-compatible episode logs from batched closed-loop rollouts.

The reference driver (main_sim_mpc.py:48-146) records one episode per run and pickles it through
Logger.plot_each_pre_trajects (logger_mpc.py:439-474) as <path>{pos,time,foot,heading,turning,body_vel,
ellp,cir,real_end,pred_end,pred_feasi_end,pred_fail_end,pred_full_end}.pkl, which plot_data_cir.py reads.
Here an episode comes from alipmpc_rollout_batch (every instance of the batch is one episode on the ideal
ALIP plant) and the per-step predicted plans from alipmpc_trace_batch (the gen_control_test pos_det traces).

Correspondence (ideal plant: the executed step is the plan's first step, so "real" = predicted step 0):
  pos        CoM position at every control tick (f_cyc = 40 ticks of step_t / f_cyc = 0.01 s per step):
             rows 1..40 of the step-0 trace of each plan (the ALIP flow from the touchdown state)
  time       tick times 0, 0.01, ...                              (Logger.t_list)
  foot       stance foot per tick (foot_traj[t, 0:2])             (list_pos_stf_map_glo_frame)
  heading    theta(t) = theta_t + (t / T) dtheta_t per tick       (the ALIP B-matrix heading row)
  turning    the turn command dtheta_t per tick                   (list_hd_input_pr)
  body_vel   CoM velocity rotated into the heading frame per tick (list_vel_com_fot_fram)
  real_end   CoM position at each foot switch = x^(t+1)[0:2]      (real_str_traj)
  pred_end   [[CoM at switch], [plan's predicted x_1 position]]   (pred_str_traj_list)
  pred_full_end / pred_feasi_end / pred_fail_end
             the plan traces (N * 42 x 2 each, 126 x 2 at N = 3), all / status != 2 / status == 2
  cir, ellp  the obstacle lists as given (the driver stores the un-inflated lists)
Container types follow the reference: numpy arrays for the per-tick series and real_end, python lists of
arrays for pred_* and for ellp when it is empty.
"""
import math
import os
import pickle

import numpy as np

NAMES = ("pos", "time", "foot", "heading", "turning", "body_vel", "ellp", "cir", "real_end", "pred_end",
         "pred_feasi_end", "pred_fail_end", "pred_full_end")


def episode_logs(roll, b, trace_fn, cir=None, elp=None, dt=0.4, f_cyc=40, beta=math.sqrt(9.81 / 1.0)):
    """Build the data_log arrays of episode b of a rollout.

    roll: dict from Solver.rollout (x (B,S+1,5), foot (B,S,3), status (B,S), u (B,S,5N), steps_to_goal (B,)).
    trace_fn(x0s (T,5), us (T,5N)) -> (T, N, rows, 2): Solver.trace on the GPU (or planner.plan_traces).
    """
    stg = int(roll["steps_to_goal"][b])
    S = roll["foot"].shape[1]
    T = stg if stg > 0 else S
    x = np.asarray(roll["x"][b, :T + 1], float)
    foot = np.asarray(roll["foot"][b, :T], float)
    status = np.asarray(roll["status"][b, :T])
    u = np.asarray(roll["u"][b, :T], float)
    tr = np.asarray(trace_fn(x[:T], u))                                   # (T, N, rows, 2)
    N = tr.shape[1]
    plans = [tr[t].reshape(N * tr.shape[2], 2) for t in range(T)]
    ticks = f_cyc
    pos = np.concatenate([tr[t, 0, 1:1 + ticks] for t in range(T)]) if T else np.zeros((0, 2))
    tick_t = np.arange(ticks) * (dt / f_cyc)
    time = np.arange(T * ticks) * (dt / f_cyc)
    stance = np.repeat(foot[:, 0:2], ticks, axis=0)
    heading = np.concatenate([x[t, 4] + tick_t / dt * foot[t, 2] for t in range(T)]) if T else np.zeros(0)
    turning = np.repeat(foot[:, 2], ticks)
    body = []
    for t in range(T):
        ch, sh = np.cosh(beta * tick_t), np.sinh(beta * tick_t)
        vx = sh * beta * (x[t, 0] - foot[t, 0]) + ch * x[t, 2]
        vy = sh * beta * (x[t, 1] - foot[t, 1]) + ch * x[t, 3]
        th = x[t, 4] + tick_t / dt * foot[t, 2]
        c, s = np.cos(th), np.sin(th)
        body.append(np.stack([c * vx + s * vy, -s * vx + c * vy], 1))
    body_vel = np.concatenate(body) if body else np.zeros((0, 2))
    real_end = x[1:T + 1, 0:2].copy()
    pred_end = [np.array([x[t + 1, 0:2], u[t, 0:2]]) for t in range(T)]
    feasi = [plans[t] for t in range(T) if status[t] != 2]
    fail = [plans[t] for t in range(T) if status[t] == 2]
    return {
        "pos": pos, "time": time, "foot": stance, "heading": heading, "turning": turning, "body_vel": body_vel,
        "ellp": [] if elp is None or len(elp) == 0 else np.asarray(elp, float),
        "cir": np.zeros((0, 3)) if cir is None else np.asarray(cir, float),
        "real_end": real_end, "pred_end": pred_end, "pred_feasi_end": feasi, "pred_fail_end": fail,
        "pred_full_end": plans,
    }


def write_data_log(path, logs):
    """Write <path><name>.pkl for every data_log entry (logger_mpc.py:449-474 file names)."""
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    for name in NAMES:
        with open(path + name + ".pkl", "wb") as fh:
            pickle.dump(logs[name], fh)
    return [path + name + ".pkl" for name in NAMES]


def read_data_log(path):
    """Read back logs written by write_data_log (our own files only)."""
    out = {}
    for name in NAMES:
        with open(path + name + ".pkl", "rb") as fh:
            out[name] = pickle.load(fh)
    return out
