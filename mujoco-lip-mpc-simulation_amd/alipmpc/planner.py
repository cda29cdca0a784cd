"""MPCCBF drop-in: the reference planner API (MPC_LIP_modi.MPCCBF / MPC_LIP_sig_step.MPCCBF) dispatching
the NLP solve to libalipmpc.so through ctypes, plus a batched entry point.

Reference surface reproduced (file:line):
  MPCCBF.__init__(goals, cir_param, cir_cbf, elp_param, elp_cbf, margin, step=3)    MPC_LIP_modi.py:14-87
  .gen_control_test(state, leg_ind, init_guess, plot=False, trajec=[])
        -> (xk_list[1:], p_list[0], hd_list, close_2_goal, feasi, pos_det)          MPC_LIP_modi.py:90-146
  .solveMPCCBF(xk, od_ev, init_guess) -> (u, feasi)                                MPC_LIP_modi.py:197-301
  .get_next_states(glo_pos, glo_vel, glo_hd, glo_p, t_rest, plot=False)            MPC_LIP_modi.py:149-178
  .alip_des_vel(vx_max, leg_ind) / .cal_foot_with_veldes(x_state, vel_des_glo)      MPC_LIP_modi.py:181-194
  .select_obs(xk) (sets sel_cir / sel_elp) / .xk_track_det / .solve_footdisp / .tube_func
  sig_step: MPCCBFSigStep(goals, obs_param, obs_cbf, margin, step=3); gen_control_test returns the
  4-tuple (xk_list[1:], p_list[0], hd_list, close_2_goal) and solveMPCCBF returns u   MPC_LIP_sig_step.py:14-278
  DD: MPCCBFDD(goals, cir_param, cir_cbf, elp_param, elp_cbf, margin, step=3); gen_dd_control(state,
  init_guess, last_u) -> (states, heading, control, close2goal, fesi)                  MPC_DD_sig_step.py:11-193
Errors: invalid arguments raise ValueError; a solver failure is NOT an exception (feasi = 2, iterate
returned), exactly like the reference.  Instances are stateful (sel_cir, init_state) and not re-entrant.
New: solve_batch(states, leg_inds, init_guesses, ...) solves many instances in one kernel launch.
"""
import math

import numpy as np

from . import _lib


def _alip_matrices(beta, t, T):
    ch, sh = math.cosh(beta * t), math.sinh(beta * t)
    A = np.array([[ch, 0, sh / beta, 0, 0], [0, ch, 0, sh / beta, 0], [sh * beta, 0, ch, 0, 0],
                  [0, sh * beta, 0, ch, 0], [0, 0, 0, 0, 1.0]])
    B = np.array([[1 - ch, 0, 0], [0, 1 - ch, 0], [-sh * beta, 0, 0], [0, -sh * beta, 0], [0, 0, t * (1 / T)]])
    return A, B


def next_state(beta, dt, glo_pos, glo_vel, glo_hd, glo_p, t_rest):
    """Continuous ALIP flow over the remaining step time (MPC_LIP_modi.py:149-178) -> (x_next, trace)."""
    A, B = _alip_matrices(beta, t_rest, dt)
    xk = np.concatenate([np.ravel(glo_pos), np.ravel(glo_vel), [glo_hd]]).astype(float)
    p = np.ravel(glo_p).astype(float)
    return A @ xk + B @ p, track_det(beta, xk, p, t_rest)


def track_det(beta, xk, contr, t_rest):
    """MPC_LIP_modi.py:304-322 vectorised: [x0[0:2]] + positions at t = 0, 0.01, ... (np.arange rule)."""
    t_det = np.arange(0, t_rest + 0.01, 0.01)
    xk = np.ravel(xk).astype(float)
    p = np.ravel(contr).astype(float)
    ch, sh = np.cosh(beta * t_det), np.sinh(beta * t_det)
    px = ch * xk[0] + sh / beta * xk[2] + (1 - ch) * p[0]
    py = ch * xk[1] + sh / beta * xk[3] + (1 - ch) * p[1]
    return np.concatenate([xk[None, 0:2], np.stack([px, py], 1)])


def alip_constants(dt=0.4, g=9.81, H=1.0):
    """MPCCBF.__init__ constants (MPC_LIP_modi.py:45-68): beta, A, B (B[4,2] = 1), W (a = 5, b = 1 weighted
    pseudo-inverse), M_A = A - B W A, M_B = B W."""
    beta = math.sqrt(g / H)
    A, B = _alip_matrices(beta, dt, dt)
    B[4, 2] = 1.0
    ch, sh = math.cosh(beta * dt), math.sinh(beta * dt)
    a, b = 5.0, 1.0
    D = a * (ch - 1) ** 2 + b * (sh * beta) ** 2
    Ch, Sh = -a * (ch - 1) / D, -b * sh * beta / D
    W = np.array([[Ch, 0, Sh, 0, 0], [0, Ch, 0, Sh, 0], [0, 0, 0, 0, 1.0]])
    return dict(beta=beta, A=A, B=B, W=W, M_A=A - B @ W @ A, M_B=B @ W)


def plan_traces(beta, dt, A, W, M_A, M_B, x0s, us):
    """numpy form of the pos_det traces of gen_control_test (MPC_LIP_modi.py:102-122) for many plans:
    x0s (T,5), us (T,5N) -> (T, N, rows, 2) — what alipmpc_trace_batch computes on the device."""
    x0s = np.asarray(x0s, float).reshape(-1, 5)
    us = np.asarray(us, float).reshape(len(x0s), -1)
    N = us.shape[1] // 5
    out = []
    for x0, u in zip(x0s, us):
        xk, rows = x0, []
        for i in range(N):
            uk = u[5 * i:5 * (i + 1)]
            pk = W @ (uk - A @ xk)
            rows.append(track_det(beta, xk, pk, dt))
            xk = M_A @ xk + M_B @ uk
        out.append(np.stack(rows))
    return np.stack(out) if out else np.zeros((0, N, 0, 2))


class _Base:
    variant = _lib.VARIANT_MODI

    def _setup(self, goals, margin, step, device, cfg_overrides, nc_max, ne_max):
        self.goal = np.asarray(goals, float).reshape(-1)[:2].reshape(2, 1)
        self.margin = margin
        self.N = step
        self.dt = 0.4
        self.beta = math.sqrt(9.81 / 1.0)
        self.step_gap = 0.3
        # sigma = beta * coth(dt * beta / 2)   (MPC_LIP_modi.py:45)
        self.sigma = self.beta / math.tanh(self.dt * self.beta / 2)
        k = alip_constants(self.dt)
        self.A, self.B, self.W, self.M_A, self.M_B = k["A"], k["B"], k["W"], k["M_A"], k["M_B"]
        self.B_vel_shr = self.B[2:4, 0:2]
        self.inv_B_vel_shr = np.linalg.inv(self.B_vel_shr)
        self.cfg = _lib.default_cfg(self.variant, step, nc_max=max(nc_max, 0), ne_max=max(ne_max, 0),
                                    **cfg_overrides)
        self.solver = _lib.Solver(self.cfg, device=device)
        self.leg = self.cfg.leg2_max
        self.bvx_max, self.bvx_min = self.cfg.bvx_hi, self.cfg.bvx_lo
        self.bvy_max, self.bvy_min = self.cfg.bvy_hi, self.cfg.bvy_lo
        self.ang_max = self.cfg.dtheta_max
        self.last_status = None
        self.last_iters = None

    # --- small host-side helpers of the reference (not the hot path) ------------------------------
    def get_next_states(self, glo_pos, glo_vel, glo_hd, glo_p, t_rest, plot=False):
        return next_state(self.beta, self.dt, glo_pos, glo_vel, glo_hd, glo_p, t_rest)

    def xk_track_det(self, xk, contr, t_rest):
        return track_det(self.beta, xk, contr, t_rest)

    def plan_traces(self, x0s, us, device=True):
        """pos_det traces of many plans: on the GPU (alipmpc_trace_batch) or with numpy (device=False)."""
        if device:
            return self.solver.trace(x0s, us)
        return plan_traces(self.beta, self.dt, self.A, self.W, self.M_A, self.M_B, x0s, us)

    def alip_des_vel(self, vx_max, leg_ind):
        vdes_x = self.sigma * vx_max * self.dt / 2
        vdes_y = 0.5 * (-0.5 * leg_ind * self.step_gap) * (self.beta * math.sinh(self.beta * self.dt)) / \
            (math.cosh(self.beta * self.dt) + 1)
        return np.array([vdes_x, vdes_y])

    def cal_foot_with_veldes(self, x_state, vel_des_glo):
        A_x = self.A @ np.ravel(x_state)
        return np.ravel(self.inv_B_vel_shr @ (np.ravel(vel_des_glo) - A_x[2:4]))

    def solve_footdisp(self, xk, u):
        return self.W @ (np.ravel(u) - self.A @ np.ravel(xk))

    def tube_func(self, heading_list, init_tube_value):
        new_heading = np.zeros_like(heading_list, dtype=float)
        tube = init_tube_value
        for i, h in enumerate(heading_list):
            d = h - tube
            if d > 0:
                tube += (0.5 if 0.15 > d else 0.7) * d
            elif d < 0:
                tube += (0.5 if -0.15 < d else 0.7) * d
            new_heading[i] = tube
        return new_heading

    # --- batched solve --------------------------------------------------------------------------
    def solve_batch(self, states, leg_inds, init_guesses, goals=None, cir=None, nc=None, elp=None, ne=None):
        """Solve many instances in one launch.  states (B,5); leg_inds (B,) = od_ev; init_guesses (B,5N).
        Obstacles default to this planner's inflated lists.  Returns dict(u, foot, x_pred, status, iters)."""
        states = np.asarray(states, float).reshape(-1, 5)
        Bn = len(states)
        goals = np.tile(np.ravel(self.goal), (Bn, 1)) if goals is None else goals
        if cir is None:
            cir, nc = self._padded_cir(Bn)
        if elp is None and self.cfg.ne_max > 0:
            elp, ne = self._padded_elp(Bn)
        return self.solver.solve(states, goals, np.asarray(leg_inds), cir, nc, elp, ne,
                                 u0=np.asarray(init_guesses, float).reshape(Bn, -1))

    def _padded_cir(self, Bn):
        nc = len(self.cir_safe)
        c = np.zeros((Bn, self.cfg.nc_max, 3))
        if nc:
            c[:, :nc] = self.cir_safe
        return c, np.full(Bn, nc, np.int32)

    def _padded_elp(self, Bn):
        ne = len(self.elp_safe)
        e = np.zeros((Bn, self.cfg.ne_max, 5))
        if ne:
            e[:, :ne] = self.elp_safe
        return e, np.full(Bn, ne, np.int32)

    def _solve_one(self, xk, od_ev, u0):
        cir, nc = self._padded_cir(1)
        elp, ne = self._padded_elp(1) if self.cfg.ne_max > 0 else (None, None)
        out = self.solver.solve(np.ravel(xk)[None], np.ravel(self.goal)[None], np.array([1 if od_ev > 0 else -1]),
                                cir, nc, elp, ne, u0=np.ravel(u0)[None])
        self.last_status = int(out["status"][0])
        self.last_iters = int(out["iters"][0])
        return out["u"][0], self.last_status


class MPCCBF(_Base):
    """Drop-in for MPC_LIP_modi.MPCCBF (circle + ellipse D-CBF, f_en row, select_obs, detour goal)."""
    variant = _lib.VARIANT_MODI

    def __init__(self, goals, cir_param, cir_cbf, elp_param, elp_cbf, margin, step=3, device=0, **cfg_overrides):
        self.cir_list = cir_param
        self.elp_list = elp_param
        self.cir_safe = np.asarray(cir_cbf, float).reshape(-1, 3)
        self.elp_safe = np.asarray(elp_cbf, float).reshape(-1, 5)
        self._setup(goals, margin, step, device, cfg_overrides, len(self.cir_safe), len(self.elp_safe))

    def select_obs(self, xk):
        """MPC_LIP_modi.py:325-338 (informational here: the kernel applies the same filter on device)."""
        xk = np.ravel(xk)
        self.sel_cir = [c for c in self.cir_safe if (xk[0] - c[0]) ** 2 + (xk[1] - c[1]) ** 2 - c[2] ** 2 <= 16]
        self.sel_elp = [e for e in self.elp_safe
                        if (xk[0] - e[0]) ** 2 + (xk[1] - e[1]) ** 2 - max(e[2], e[3]) ** 2 <= 16]

    def solveMPCCBF(self, xk, od_ev, init_guess):
        if init_guess is None:
            raise ValueError("modi solveMPCCBF needs an init_guess (MPC_LIP_modi.py:199)")
        u0 = np.ravel(np.asarray(init_guess, float))
        if u0.size != 5 * self.N:
            raise ValueError(f"init_guess must have {5 * self.N} entries")
        return self._solve_one(xk, od_ev, u0)

    def gen_control_test(self, state, leg_ind, init_guess, plot=False, trajec=[]):
        self.init_state = np.asarray(state, float).reshape(5, 1)
        xk = np.ravel(state).astype(float)
        self.select_obs(xk)
        u, feasi = self.solveMPCCBF(xk, leg_ind, init_guess)
        p_list, hd_list, xk_list = [], [], [xk]
        for i in range(self.N):
            uk = u[5 * i:5 * (i + 1)]
            pk = self.W @ (uk - self.A @ xk)
            xk = self.M_A @ xk + self.M_B @ uk
            if i == 0:
                dis2goal = math.sqrt(float((xk[0:2] - np.ravel(self.goal)) @ (xk[0:2] - np.ravel(self.goal))))
            p_list.append(pk)
            xk_list.append(xk)
            hd_list.append(float(xk[4]))
        close_2_goal = dis2goal <= 0.15
        pos_det = np.concatenate([self.xk_track_det(xk_list[j], p_list[j], self.dt) for j in range(self.N)])
        return xk_list[1:], p_list[0], hd_list, close_2_goal, feasi, pos_det


class MPCCBFSigStep(_Base):
    """Drop-in for MPC_LIP_sig_step.MPCCBF (circles only, all obstacles used, no f_en row)."""
    variant = _lib.VARIANT_SIG_STEP

    def __init__(self, goals, obs_param, obs_cbf, margin, step=3, device=0, **cfg_overrides):
        self.obs_list = obs_param
        self.cir_safe = np.asarray(obs_cbf, float).reshape(-1, 3)
        self.elp_safe = np.zeros((0, 5))
        self._setup(goals, margin, step, device, cfg_overrides, len(self.cir_safe), 0)

    def solveMPCCBF(self, xk, od_ev, init_guess):
        """MPC_LIP_sig_step.py:184-278: None -> [x0]*3, else [g1, g2, g2] from the previous plan."""
        xa = np.ravel(xk).astype(float)
        if init_guess is None:
            u0 = np.tile(xa, self.N)
        else:
            g = [np.ravel(v) for v in init_guess]
            u0 = np.concatenate(g[1:] + [g[-1]])      # N = 3: [g1, g2, g2]
        u, st = self._solve_one(xa, od_ev, u0)
        return u

    def gen_control_test(self, state, leg_ind, init_guess, plot=False, trajec=[]):
        self.init_state = np.asarray(state, float).reshape(5, 1)
        xk = np.ravel(state).astype(float)
        u = self.solveMPCCBF(xk, leg_ind, init_guess)
        p_list, hd_list, xk_list = [], [], [xk]
        close_2_goal = False
        for i in range(self.N):
            uk = u[5 * i:5 * (i + 1)]
            pk = self.W @ (uk - self.A @ xk)
            xk = self.M_A @ xk + self.M_B @ uk
            d = math.sqrt(float((xk[0:2] - np.ravel(self.goal)) @ (xk[0:2] - np.ravel(self.goal))))
            p_list.append(pk)
            xk_list.append(xk)
            hd_list.append(float(xk[4]))
            if d <= 0.35:
                close_2_goal = True
        return xk_list[1:], p_list[0], hd_list, close_2_goal


class MPCCBFDD(_Base):
    """Drop-in for MPC_DD_sig_step.MPCCBF (unicycle MPC-CBF, MPC_DD_sig_step.py:11-316): state [px, py, th],
    decision [v, w] x N with v in [0.4, 0.8], |w| <= pi/16, f_en = s|w| + v, smoothness to last_u.
      gen_dd_control(state, init_guess, last_u, plot=False, trajec=[])
          -> (states, heading, control, close2goal, fesi)                          :70-121
      solveMPCCBF(xk, init_guess, last_u) -> (u, fesi)                            :123-193
    All obstacles are used (select_obs is commented out, :75) and there is no detour goal."""
    variant = _lib.VARIANT_DD

    def __init__(self, goals, cir_param, cir_cbf, elp_param, elp_cbf, margin, step=3, device=0, **cfg_overrides):
        self.cir_list = cir_param
        self.elp_list = elp_param
        self.cir_safe = np.asarray(cir_cbf, float).reshape(-1, 3)
        self.elp_safe = np.asarray(elp_cbf, float).reshape(-1, 5)
        self._setup(goals, margin, step, device, cfg_overrides, len(self.cir_safe), len(self.elp_safe))
        self.v_max, self.v_min = self.cfg.bvx_hi, self.cfg.bvx_lo
        self.tot_time = 80

    def tube_func(self, heading_list, init_tube_value):
        """MPC_DD_sig_step.py:298-316 (its own thresholds: +-0.2, gains 0.3 / 0.7)."""
        new_heading = np.zeros_like(heading_list, dtype=float)
        tube = init_tube_value
        for i, h in enumerate(heading_list):
            d = h - tube
            if d > 0:
                tube += (0.3 if 0.2 > d else 0.7) * d
            elif d < 0:
                tube += (0.3 if -0.2 < d else 0.7) * d
            new_heading[i] = tube
        return new_heading

    def solveMPCCBF(self, xk, init_guess, last_u):
        u0 = np.ravel(np.asarray(init_guess, float))
        if u0.size != 2 * self.N:
            raise ValueError(f"init_guess must have {2 * self.N} entries")
        cir, nc = self._padded_cir(1)
        elp, ne = self._padded_elp(1) if self.cfg.ne_max > 0 else (None, None)
        out = self.solver.solve(np.ravel(xk)[None], np.ravel(self.goal)[None], None, cir, nc, elp, ne,
                                u0=u0[None], last_u=np.ravel(np.asarray(last_u, float))[None])
        self.last_status = int(out["status"][0])
        self.last_iters = int(out["iters"][0])
        return out["u"][0], self.last_status

    def gen_dd_control(self, state, init_guess, last_u, plot=False, trajec=[]):
        self.init_state = np.asarray(state, float).reshape(3, 1)
        xk = np.ravel(state).astype(float)
        u, fesi = self.solveMPCCBF(xk, init_guess, last_u)
        states, heading, control = [list(xk)], [], []
        g = np.ravel(self.goal)
        dis2goal = None
        for i in range(self.N):
            uk = np.array([u[2 * i:2 * i + 2]]).T
            xk = xk + np.array([self.dt * math.cos(xk[2]) * uk[0, 0], self.dt * math.sin(xk[2]) * uk[0, 0], uk[1, 0]])
            if i == 0:
                dis2goal = math.sqrt(float((xk[0:2] - g) @ (xk[0:2] - g)))
            states.append(list(xk))
            heading.append(float(xk[2]))
            control.append(uk)
        return states, heading, control, dis2goal <= 0.35, fesi

    def solve_batch(self, states, init_guesses, last_us, goals=None, cir=None, nc=None, elp=None, ne=None):
        """Many DD instances in one launch: states (B,3), init_guesses (B,2N), last_us (B,2)."""
        states = np.asarray(states, float).reshape(-1, 3)
        Bn = len(states)
        goals = np.tile(np.ravel(self.goal), (Bn, 1)) if goals is None else goals
        if cir is None:
            cir, nc = self._padded_cir(Bn)
        if elp is None and self.cfg.ne_max > 0:
            elp, ne = self._padded_elp(Bn)
        return self.solver.solve(states, goals, None, cir, nc, elp, ne,
                                 u0=np.asarray(init_guesses, float).reshape(Bn, -1),
                                 last_u=np.asarray(last_us, float).reshape(Bn, 2))
