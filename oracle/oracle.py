"""ORACLE (test infrastructure only) — ctypes wrapper of oracle/liboracle.so, the C restatement of the
reference NLP and of the interior-point solve (see alipmpc_oracle.c header for reference anchors).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module, as the
checker or the reported CPU baseline; the product (libalipmpc.so) never touches it.
"""
import ctypes
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

VARIANT_MODI, VARIANT_SIG_STEP, VARIANT_DD = 0, 1, 2


class Cfg(ctypes.Structure):
    """Mirror of alipmpc_cfg (include/alipmpc.h)."""
    _fields_ = [(k, ctypes.c_int32) for k in
                ("N", "nc_max", "ne_max", "variant", "max_iter", "precision", "select_obs", "detour")] + \
               [(k, ctypes.c_double) for k in
                ("tol", "acceptable_tol", "dt", "H", "g", "leg2_max", "bvx_lo", "bvx_hi", "bvy_lo", "bvy_hi",
                 "dtheta_max", "q", "p", "r", "gamma", "s", "detect_r2", "dd_t", "mu_init")] + \
               [("program", ctypes.c_int32), ("goal_singular", ctypes.c_int32), ("restoration", ctypes.c_int32),
                ("reserved_", ctypes.c_int32)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.oracle_default_cfg.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(Cfg)]
        P = ctypes.c_void_p
        L.oracle_solve_batch.argtypes = [ctypes.POINTER(Cfg), ctypes.c_int64] + [P] * 14 + [ctypes.c_int]
        L.oracle_solve_batch.restype = ctypes.c_int
        L.oracle_eval_batch.argtypes = [ctypes.POINTER(Cfg), ctypes.c_int64] + [P] * 16
        L.oracle_eval_batch.restype = ctypes.c_int
        L.oracle_solve_batch_dd.argtypes = [ctypes.POINTER(Cfg), ctypes.c_int64] + [P] * 14 + [ctypes.c_int]
        L.oracle_solve_batch_dd.restype = ctypes.c_int
        L.oracle_eval_batch_dd.argtypes = [ctypes.POINTER(Cfg), ctypes.c_int64] + [P] * 15
        L.oracle_eval_batch_dd.restype = ctypes.c_int
        _lib = L
    return _lib


def default_cfg(variant=VARIANT_MODI, N=3, **kw):
    c = Cfg()
    lib().oracle_default_cfg(variant, N, ctypes.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def n_vars(cfg):
    return 2 * cfg.N if cfg.variant == VARIANT_DD else 5 * cfg.N


def rows_per_step(cfg):
    if cfg.variant == VARIANT_DD:
        return cfg.nc_max + cfg.ne_max + 1
    return 4 + cfg.nc_max + cfg.ne_max + (1 if cfg.variant == VARIANT_MODI else 0)


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _batch_inputs(cfg, x0, goal, leg, cir, nc, elp, ne):
    B = len(x0)
    x0 = np.ascontiguousarray(x0, np.float64).reshape(B, 5)
    goal = np.ascontiguousarray(np.broadcast_to(np.asarray(goal, np.float64), (B, 2)))
    leg = np.ascontiguousarray(leg, np.int8).reshape(B)
    cir = np.ascontiguousarray(cir, np.float64).reshape(B, cfg.nc_max, 3)
    nc = np.ascontiguousarray(nc, np.int32).reshape(B)
    if cfg.ne_max > 0 and elp is not None:
        elp = np.ascontiguousarray(elp, np.float64).reshape(B, cfg.ne_max, 5)
        ne = np.ascontiguousarray(ne, np.int32).reshape(B)
    else:
        elp = None
        ne = np.zeros(B, np.int32)
    return B, x0, goal, leg, cir, nc, elp, ne


def solve_batch(cfg, x0, goal, leg, cir, nc, elp, ne, u0, nthreads=1):
    B, x0, goal, leg, cir, nc, elp, ne = _batch_inputs(cfg, x0, goal, leg, cir, nc, elp, ne)
    n = n_vars(cfg)
    u0 = np.ascontiguousarray(u0, np.float64).reshape(B, n)
    out = dict(u=np.zeros((B, n)), foot=np.zeros((B, 3)), x_pred=np.zeros((B, cfg.N, 5)),
               status=np.zeros(B, np.int32), iters=np.zeros(B, np.int32), restorations=np.zeros(B, np.int32))
    rc = lib().oracle_solve_batch(ctypes.byref(cfg), B, _p(x0), _p(goal), _p(leg), _p(cir), _p(nc), _p(elp), _p(ne),
                                  _p(u0), _p(out["u"]), _p(out["foot"]), _p(out["x_pred"]), _p(out["status"]),
                                  _p(out["iters"]), _p(out["restorations"]), nthreads)
    if rc != 0:
        raise RuntimeError(f"oracle_solve_batch failed: {rc}")
    return out


def eval_batch(cfg, x0, goal, leg, cir, nc, elp, ne, u):
    B, x0, goal, leg, cir, nc, elp, ne = _batch_inputs(cfg, x0, goal, leg, cir, nc, elp, ne)
    n = n_vars(cfg)
    mm = cfg.N * rows_per_step(cfg)
    u = np.ascontiguousarray(u, np.float64).reshape(B, n)
    out = dict(f=np.zeros(B), grad=np.zeros((B, n)), c=np.zeros((B, mm)), J=np.zeros((B, mm, n)),
               cl=np.zeros((B, mm)), cu=np.zeros((B, mm)), goal_eff=np.zeros((B, 2)),
               row_active=np.zeros((B, mm), np.int8))
    rc = lib().oracle_eval_batch(ctypes.byref(cfg), B, _p(x0), _p(goal), _p(leg), _p(cir), _p(nc), _p(elp), _p(ne),
                                 _p(u), _p(out["f"]), _p(out["grad"]), _p(out["c"]), _p(out["J"]), _p(out["cl"]),
                                 _p(out["cu"]), _p(out["goal_eff"]), _p(out["row_active"]))
    if rc != 0:
        raise RuntimeError(f"oracle_eval_batch failed: {rc}")
    return out


def _dd_inputs(cfg, x0, goal, cir, nc, elp, ne, last_u):
    B = len(x0)
    x0 = np.ascontiguousarray(x0, np.float64).reshape(B, 3)
    goal = np.ascontiguousarray(np.broadcast_to(np.asarray(goal, np.float64), (B, 2)))
    cir = np.ascontiguousarray(cir, np.float64).reshape(B, cfg.nc_max, 3)
    nc = np.ascontiguousarray(nc, np.int32).reshape(B)
    if cfg.ne_max > 0 and elp is not None:
        elp = np.ascontiguousarray(elp, np.float64).reshape(B, cfg.ne_max, 5)
        ne = np.ascontiguousarray(ne, np.int32).reshape(B)
    else:
        elp = None
        ne = np.zeros(B, np.int32)
    last_u = np.ascontiguousarray(np.broadcast_to(np.asarray(last_u, np.float64), (B, 2)))
    return B, x0, goal, cir, nc, elp, ne, last_u


def solve_batch_dd(cfg, x0, goal, cir, nc, elp, ne, u0, last_u, nthreads=1):
    """DD (unicycle) solves; foot = first control [v, w, 0], x_pred = x_1..x_N (B x N x 3)."""
    B, x0, goal, cir, nc, elp, ne, last_u = _dd_inputs(cfg, x0, goal, cir, nc, elp, ne, last_u)
    n = n_vars(cfg)
    u0 = np.ascontiguousarray(u0, np.float64).reshape(B, n)
    out = dict(u=np.zeros((B, n)), foot=np.zeros((B, 3)), x_pred=np.zeros((B, cfg.N, 3)),
               status=np.zeros(B, np.int32), iters=np.zeros(B, np.int32), restorations=np.zeros(B, np.int32))
    rc = lib().oracle_solve_batch_dd(ctypes.byref(cfg), B, _p(x0), _p(goal), _p(cir), _p(nc), _p(elp), _p(ne),
                                     _p(u0), _p(last_u), _p(out["u"]), _p(out["foot"]), _p(out["x_pred"]),
                                     _p(out["status"]), _p(out["iters"]), _p(out["restorations"]), nthreads)
    if rc != 0:
        raise RuntimeError(f"oracle_solve_batch_dd failed: {rc}")
    return out


def eval_batch_dd(cfg, x0, goal, cir, nc, elp, ne, u, last_u):
    B, x0, goal, cir, nc, elp, ne, last_u = _dd_inputs(cfg, x0, goal, cir, nc, elp, ne, last_u)
    n = n_vars(cfg)
    mm = cfg.N * rows_per_step(cfg)
    u = np.ascontiguousarray(u, np.float64).reshape(B, n)
    out = dict(f=np.zeros(B), grad=np.zeros((B, n)), c=np.zeros((B, mm)), J=np.zeros((B, mm, n)),
               cl=np.zeros((B, mm)), cu=np.zeros((B, mm)), row_active=np.zeros((B, mm), np.int8))
    rc = lib().oracle_eval_batch_dd(ctypes.byref(cfg), B, _p(x0), _p(goal), _p(cir), _p(nc), _p(elp), _p(ne), _p(u),
                                    _p(last_u), _p(out["f"]), _p(out["grad"]), _p(out["c"]), _p(out["J"]),
                                    _p(out["cl"]), _p(out["cu"]), _p(out["row_active"]))
    if rc != 0:
        raise RuntimeError(f"oracle_eval_batch_dd failed: {rc}")
    return out


def rollout_batch(cfg, x0, goal, leg, cir, nc, elp, ne, u0, last_u=None, steps=8, nthreads=1):
    """Closed-loop receding-horizon rollout on an ideal ALIP plant (oracle of alipmpc_rollout_batch).
    Per step: solve the active instances (C oracle); x <- x_pred[0] (the touchdown state = get_next_states
    over a full step, MPC_LIP_modi.py:149-178); stance switch leg <- -leg (main_sim_mpc.py:111); warm start
    modi: previous x_mpc_tar unshifted (logger_mpc.py:325-331), sig_step: [g2..gN, gN]
    (MPC_LIP_sig_step.py:186-189), DD: previous controls + last_u <- first control; retire after
    close_2_goal (modi |pos_1-goal| <= 0.15, MPC_LIP_modi.py:108-115; sig_step any step <= 0.35,
    MPC_LIP_sig_step.py:104-111; DD |pos_1-goal| <= 0.35, MPC_DD_sig_step.py:92-98; the episode stops after
    that step, main_sim_mpc.py:121-131)."""
    dd = cfg.variant == VARIANT_DD
    sd = 3 if dd else 5
    N, n = cfg.N, n_vars(cfg)
    x = np.array(x0, np.float64).reshape(-1, sd).copy()
    B = len(x)
    goal = np.ascontiguousarray(np.broadcast_to(np.asarray(goal, np.float64), (B, 2)))
    u0 = np.array(u0, np.float64).reshape(B, n).copy()
    legv = None if dd else np.array(leg, np.int8).reshape(B).copy()
    lu = np.zeros((B, 2)) if last_u is None else np.array(np.broadcast_to(np.asarray(last_u, np.float64), (B, 2)))
    S = int(steps)
    foot = np.full((B, S, 3), np.nan)
    xs = np.zeros((B, S + 1, sd))
    xs[:, 0] = x
    status = np.full((B, S), -10, np.int32)
    iters = np.zeros((B, S), np.int32)
    stg = np.full(B, -1, np.int32)
    uts = np.full((B, S, n), np.nan)
    active = np.ones(B, bool)
    elp_a = None if elp is None else np.asarray(elp)
    ne_a = None if ne is None else np.asarray(ne)
    for t in range(S):
        idx = np.nonzero(active)[0]
        if len(idx):
            sub = lambda a: None if a is None else np.asarray(a)[idx]
            if dd:
                o = solve_batch_dd(cfg, x[idx], goal[idx], sub(cir), sub(nc), sub(elp_a), sub(ne_a), u0[idx], lu[idx],
                                   nthreads=nthreads)
            else:
                o = solve_batch(cfg, x[idx], goal[idx], legv[idx], sub(cir), sub(nc), sub(elp_a), sub(ne_a), u0[idx],
                                nthreads=nthreads)
            foot[idx, t] = o["foot"]
            status[idx, t] = o["status"]
            iters[idx, t] = o["iters"]
            xp = o["x_pred"]
            x[idx] = xp[:, 0]
            u = o["u"]
            uts[idx, t] = u
            if cfg.variant == VARIANT_SIG_STEP:
                blk = n // N
                ub = u.reshape(len(idx), N, blk)
                u0[idx] = np.concatenate([ub[:, 1:], ub[:, -1:]], axis=1).reshape(len(idx), n)
            else:
                u0[idx] = u
            if dd:
                lu[idx] = u[:, 0:2]
            else:
                legv[idx] = -legv[idx]
            d = np.sqrt(((xp[:, :, 0:2] - goal[idx, None, :]) ** 2).sum(-1))
            if cfg.variant == VARIANT_SIG_STEP:
                close = (d <= 0.35).any(1)
            else:
                close = d[:, 0] <= (0.15 if cfg.variant == VARIANT_MODI else 0.35)
            done = idx[close]
            active[done] = False
            stg[done] = t + 1
        xs[:, t + 1] = x
    return dict(foot=foot, x=xs, status=status, iters=iters, steps_to_goal=stg, u=uts)


# ---------------------------------------------------------------- closed loop at the control rate (test oracle)
def _ang_diff(A, B):
    """Logger.angle_A_minus_B (data_procs/logger_mpc.py:169-175)."""
    r = A - B
    if r < 0 and abs(r) > math.pi:
        r += 2 * math.pi
    elif r > 0 and abs(r) > math.pi:
        r -= 2 * math.pi
    return r


def _tube_turn(turning, init):
    """Logger.tube_func (data_procs/logger_mpc.py:283-300)."""
    tv = init
    if turning > 0:
        tv += (0.4 if 0.15 > turning else 0.7) * turning
    elif turning < 0:
        tv += (0.4 if -0.15 < turning else 0.7) * turning
    return _ang_diff(tv, init)


_M64 = (1 << 64) - 1


def cl_uniform(seed, b, s, i, axis):
    """splitmix64 uniform [0, 1) of (episode, step, tick, axis): the closed loop's velocity kicks (the same
    integer recipe as cl_uniform in csrc/alipmpc.hip)."""
    key = ((((b * 1048576 + s) * 1024 + i) * 2 + axis) + 1) & _M64
    z = (seed + 0x9E3779B97F4A7C15 * key) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    z = z ^ (z >> 31)
    return (z >> 11) * (1.0 / 9007199254740992.0)


def closed_loop_batch(cfg, x0, foot0, goal, leg, cir, nc, elp=None, ne=None, steps=8, f_cyc=40, kick=0.0, seed=0,
                      nthreads=8, jitter=False):
    """Oracle of alipmpc_closed_loop_batch (include/alipmpc.h): the reference driver's per-tick loop
    (main_sim_mpc.py:65-135; Logger.set_stf_head / gen_nex_foot_input, data_procs/logger_mpc.py:270-371) on an
    ALIP plant, every solve by the C oracle.  jitter (study only, tools/self_drift.py): every solve's returned plan —
    the next tick's warm start — moved by one ulp (True) or by a relative amount (a float), the size of the difference
    between two implementations' returned iterates."""
    N, n = cfg.N, 5 * cfg.N
    x = np.array(x0, np.float64).reshape(-1, 5).copy()
    B = len(x)
    pst = np.array(foot0, np.float64).reshape(B, 2).copy()
    goal = np.ascontiguousarray(np.broadcast_to(np.asarray(goal, np.float64), (B, 2)))
    legv = np.array(leg, np.int8).reshape(B).copy()
    hdv = np.zeros((B, 3))     # nex_turn, hd_input_pr, hd_input_cos
    mhd = np.repeat(x[:, 4:5], 3, axis=1)   # mpc_hds_list: 0 in the Logger's robot frame = the initial heading here
    plan = np.zeros((B, n))
    active = np.ones(B, bool)
    has_plan = np.zeros(B, bool)
    rclose = np.zeros(B, bool)
    S, F = int(steps), int(f_cyc)
    beta, T = math.sqrt(cfg.g / cfg.H), cfg.dt
    dt = T / F
    ch_d, shb_d, bsh_d, td = math.cosh(beta * dt), math.sinh(beta * dt) / beta, math.sinh(beta * dt) * beta, dt / T
    foot = np.full((B, S, 3), np.nan)
    xs = np.zeros((B, S + 1, 5))
    xs[:, 0] = x
    hd = np.zeros((B, S, 2))
    # controller command per tick (Logger.gen_nex_foot_input / gen_tsc_control, logger_mpc.py:318-384): the
    # robot-global frame is the map frame moved to the initial pose (pos/vel_map_glo_2_robo_glo, :134-150);
    # vel_des = alip_des_vel(0.6, leg_ind) first (main_sim_mpc.py:54), then mpc_state_tar[0][2:4] after each
    # solve and [1][2:4] at touchdown (:88, :112)
    action = np.full((B, S, F, 8), np.nan)
    pose0 = np.concatenate([x[:, 0:2], x[:, 4:5]], axis=1).copy()
    beta_ = math.sqrt(cfg.g / cfg.H)
    sh_, ch_ = math.sinh(beta_ * cfg.dt), math.cosh(beta_ * cfg.dt)
    vdx = beta_ / math.tanh(cfg.dt * beta_ / 2) * 0.6 * cfg.dt / 2
    vdes = np.stack([np.full(B, vdx), 0.5 * (-0.5 * legv.astype(float) * 0.3) * ((beta_ * sh_) / (ch_ + 1))], 1)

    def rot(th, vx, vy):
        c, s_ = np.cos(th), np.sin(th)
        return c * vx + s_ * vy, -s_ * vx + c * vy
    status = np.full((B, S, F), -10, np.int32)
    iters = np.zeros((B, S, F), np.int32)
    stg = np.full(B, -1, np.int32)
    cir = np.asarray(cir)
    nc = np.asarray(nc)
    for s in range(S):
        for i in range(F):
            idx = np.nonzero(active)[0]
            if len(idx) == 0:
                continue
            rest = T - i * (T / F)
            ch_r, shb_r, bsh_r, tr = math.cosh(beta * rest), math.sinh(beta * rest) / beta, \
                math.sinh(beta * rest) * beta, rest * (1.0 / T)
            if i == 0:
                for b in idx:
                    cur = x[b, 4]
                    hdv[b, 2] = cur
                    hdv[b, 0] = _tube_turn(hdv[b, 0], cur)
                    ssum = hdv[b, 0]
                    ncur = [cur, mhd[b, 0], mhd[b, 1]]
                    for k in range(3):
                        ssum += _ang_diff(mhd[b, k], ncur[k])
                    hdv[b, 1] = ssum / 4.0
                    hd[b, s] = hdv[b, 1], hdv[b, 2]
            xi, fx, fy, hp = x[idx], pst[idx, 0], pst[idx, 1], hdv[idx, 1]
            xn = np.stack([ch_r * xi[:, 0] + shb_r * xi[:, 2] + (1.0 - ch_r) * fx,
                           ch_r * xi[:, 1] + shb_r * xi[:, 3] + (1.0 - ch_r) * fy,
                           bsh_r * xi[:, 0] + ch_r * xi[:, 2] - bsh_r * fx,
                           bsh_r * xi[:, 1] + ch_r * xi[:, 3] - bsh_r * fy,
                           xi[:, 4] + tr * hp], axis=1)
            u0 = np.tile(xn, (1, N))
            hp_ = has_plan[idx]
            if cfg.variant == VARIANT_SIG_STEP:
                pb = plan[idx].reshape(len(idx), N, 5)
                sh = np.concatenate([pb[:, 1:], pb[:, -1:]], axis=1).reshape(len(idx), n)
                u0[hp_] = sh[hp_]
            else:
                u0[hp_] = plan[idx][hp_]
            sub = lambda a: None if a is None else np.asarray(a)[idx]  # noqa: E731
            o = solve_batch(cfg, xn, goal[idx], -legv[idx], cir[idx], nc[idx], sub(elp), sub(ne), u0,
                            nthreads=nthreads)
            status[idx, s, i] = o["status"]
            iters[idx, s, i] = o["iters"]
            plan[idx] = (np.nextafter(o["u"], np.inf) if jitter is True else o["u"] * (1.0 + float(jitter))) if jitter \
                else o["u"]
            has_plan[idx] = True
            hdv[idx, 0] = o["foot"][:, 2]
            xp = o["x_pred"]
            mhd[idx] = xp[:, :3, 4]
            d = np.sqrt(((xp[:, :, 0:2] - goal[idx, None, :]) ** 2).sum(-1))
            if cfg.variant == VARIANT_SIG_STEP:
                close = (d <= 0.35).any(1)
            else:
                close = d[:, 0] <= (0.15 if cfg.variant == VARIANT_MODI else 0.35)
            p0 = pose0[idx]
            nsx, nsy = rot(p0[:, 2], o["foot"][:, 0] - p0[:, 0], o["foot"][:, 1] - p0[:, 1])
            csx, csy = rot(p0[:, 2], fx - p0[:, 0], fy - p0[:, 1])
            npx, npy = rot(p0[:, 2], xn[:, 0] - p0[:, 0], xn[:, 1] - p0[:, 1])
            nvx, nvy = rot(p0[:, 2], vdes[idx, 0], vdes[idx, 1])
            fi = rot(xi[:, 4] - p0[:, 2], nsx - csx, nsy - csy)
            npf = rot(xi[:, 4] - p0[:, 2], npx - csx, npy - csy)
            nvf = rot(xi[:, 4] - p0[:, 2], nvx, nvy)
            z = np.zeros(len(idx))
            action[idx, s, i] = np.stack([fi[0], fi[1], z, hp / F * (i + 4.5) + (hdv[idx, 2] - p0[:, 2]), npf[0], npf[1],
                                          nvf[0], z], axis=1)
            kv = 1 if (i == F - 1 and N > 1) else 0
            vdes[idx] = xp[:, kv, 2:4]
            xa = np.stack([ch_d * xi[:, 0] + shb_d * xi[:, 2] + (1.0 - ch_d) * fx,
                           ch_d * xi[:, 1] + shb_d * xi[:, 3] + (1.0 - ch_d) * fy,
                           bsh_d * xi[:, 0] + ch_d * xi[:, 2] - bsh_d * fx,
                           bsh_d * xi[:, 1] + ch_d * xi[:, 3] - bsh_d * fy,
                           xi[:, 4] + td * hp], axis=1)
            if kick > 0:
                for j, b in enumerate(idx):
                    xa[j, 2] += kick * (2.0 * cl_uniform(seed, int(b), s, i, 0) - 1.0)
                    xa[j, 3] += kick * (2.0 * cl_uniform(seed, int(b), s, i, 1) - 1.0)
            x[idx] = xa
            if i == F - 1:
                pst[idx] = o["foot"][:, 0:2]
                legv[idx] = -legv[idx]
                foot[idx, s] = o["foot"]
                stop = idx[rclose[idx]]
                active[stop] = False
                stg[stop] = s + 1
            rclose[idx] |= close
        xs[:, s + 1] = x
    return dict(foot=foot, x=xs, hd=hd, status=status, iters=iters, steps_to_goal=stg, action=action)
