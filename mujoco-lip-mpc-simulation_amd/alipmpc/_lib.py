"""ctypes binding of libalipmpc.so (include/alipmpc.h).

This is the reference-side binding a Python caller of the planner would add: plain
ctypes over the C ABI, numpy arrays for host-pointer calls, torch CUDA tensors (+ the current HIP stream)
for device-pointer calls.  There is no fallback: if the library or a gfx950 device is missing, the
calls raise.
"""
import ctypes
import os

import numpy as np

from . import build as _build

VARIANT_MODI, VARIANT_SIG_STEP, VARIANT_DD = 0, 1, 2
PREC_FP64, PREC_FP32 = 0, 1
PROGRAM_WAVE, PROGRAM_LANE = 0, 1   # cfg.program: one instance per wavefront / per lane (include/alipmpc.h)
GOAL_SINGULAR_ZERO, GOAL_SINGULAR_ABORT = 0, 1   # cfg.goal_singular (include/alipmpc.h)
RESTORATION_IPOPT, RESTORATION_SUBSTITUTE = 0, 1   # cfg.restoration (include/alipmpc.h)
INVALID_NUMBER_DETECTED = -13

STATUS_NAMES = {0: "Solve_Succeeded", 1: "Solved_To_Acceptable_Level", 2: "Infeasible_Problem_Detected",
                -1: "Maximum_Iterations_Exceeded", -3: "Error_In_Step_Computation",
                -13: "Invalid_Number_Detected (cfg.goal_singular = GOAL_SINGULAR_ABORT)",
                -10: "Rollout_Done (goal reached earlier, not solved)"}
ROLLOUT_DONE = -10

_ERRORS = {-1: "EINVAL", -2: "ENODEV (no visible gfx950 device)", -3: "EHIP", -4: "EUNSUPPORTED"}


class Cfg(ctypes.Structure):
    """alipmpc_cfg"""
    _fields_ = [(k, ctypes.c_int32) for k in
                ("N", "nc_max", "ne_max", "variant", "max_iter", "precision", "select_obs", "detour")] + \
               [(k, ctypes.c_double) for k in
                ("tol", "acceptable_tol", "dt", "H", "g", "leg2_max", "bvx_lo", "bvx_hi", "bvy_lo", "bvy_hi",
                 "dtheta_max", "q", "p", "r", "gamma", "s", "detect_r2", "dd_t", "mu_init")] + \
               [("program", ctypes.c_int32), ("goal_singular", ctypes.c_int32), ("restoration", ctypes.c_int32),
                ("reserved_", ctypes.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


EXPORTS = ("alipmpc_default_cfg", "alipmpc_rows_per_step", "alipmpc_num_vars", "alipmpc_create",
           "alipmpc_solve_batch", "alipmpc_eval_batch", "alipmpc_rollout_batch", "alipmpc_closed_loop_batch",
           "alipmpc_trace_len",
           "alipmpc_trace_batch", "alipmpc_nominal_gait_batch", "alipmpc_solve_slots", "alipmpc_solve_launches", "alipmpc_lane_handoffs", "alipmpc_solve_program", "alipmpc_last_kernel_ms",
           "alipmpc_build_id",
           "alipmpc_last_error", "alipmpc_destroy")

_lib = None


def lib_path():
    return _build.LIB


def build_id():
    """The loaded library's build id (include/alipmpc.h: alipmpc_build_id; "unknown" for builds without one)."""
    L = load()
    return L.alipmpc_build_id().decode() if hasattr(L, "alipmpc_build_id") else "unknown"


def load(build_if_missing=True):
    """Load libalipmpc.so (building it in-tree with hipcc if it is missing or stale)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("ALIPMPC_LIB")          # dev override (e.g. the phase-stamp diagnostic build)
    if path is None:
        if build_if_missing and _build.needs_build():
            _build.build()
        path = _build.LIB
    if not os.path.exists(path):
        raise RuntimeError(f"libalipmpc.so not found at {path}; run alipmpc.build.build()")
    L = ctypes.CDLL(path)
    P = ctypes.c_void_p
    L.alipmpc_default_cfg.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(Cfg)]
    L.alipmpc_default_cfg.restype = ctypes.c_int
    L.alipmpc_rows_per_step.argtypes = [ctypes.POINTER(Cfg)]
    L.alipmpc_rows_per_step.restype = ctypes.c_int32
    L.alipmpc_num_vars.argtypes = [ctypes.POINTER(Cfg)]
    L.alipmpc_num_vars.restype = ctypes.c_int32
    L.alipmpc_create.argtypes = [ctypes.POINTER(Cfg), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    L.alipmpc_create.restype = ctypes.c_int
    L.alipmpc_solve_batch.argtypes = [P, ctypes.c_int64] + [P] * 15
    L.alipmpc_solve_batch.restype = ctypes.c_int
    L.alipmpc_eval_batch.argtypes = [P, ctypes.c_int64] + [P] * 18
    L.alipmpc_eval_batch.restype = ctypes.c_int
    L.alipmpc_rollout_batch.argtypes = [P, ctypes.c_int64, ctypes.c_int32] + [P] * 16
    L.alipmpc_rollout_batch.restype = ctypes.c_int
    L.alipmpc_closed_loop_batch.argtypes = [P, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_double,
                                            ctypes.c_uint64] + [P] * 16
    L.alipmpc_closed_loop_batch.restype = ctypes.c_int
    L.alipmpc_trace_len.argtypes = [ctypes.POINTER(Cfg)]
    L.alipmpc_trace_len.restype = ctypes.c_int32
    L.alipmpc_trace_batch.argtypes = [P, ctypes.c_int64, P, P, P, P]
    L.alipmpc_trace_batch.restype = ctypes.c_int
    if hasattr(L, "alipmpc_nominal_gait_batch"):   # (absent from older dev builds used for A/B timing)
        L.alipmpc_nominal_gait_batch.argtypes = [P, ctypes.c_int64, ctypes.c_double, P, P, P, P, P, P]
        L.alipmpc_nominal_gait_batch.restype = ctypes.c_int
    if hasattr(L, "alipmpc_lane_handoffs"):
        L.alipmpc_lane_handoffs.argtypes = [P, P, ctypes.POINTER(ctypes.c_int64)]
        L.alipmpc_lane_handoffs.restype = ctypes.c_int
    if hasattr(L, "alipmpc_solve_launches"):
        L.alipmpc_solve_launches.argtypes = [P, ctypes.c_int64, ctypes.POINTER(ctypes.c_int32),
                                             ctypes.POINTER(ctypes.c_int32)]
        L.alipmpc_solve_launches.restype = ctypes.c_int
    if hasattr(L, "alipmpc_solve_slots"):     # (absent from older dev builds used for A/B timing)
        L.alipmpc_solve_slots.argtypes = [P, ctypes.POINTER(ctypes.c_int64)]
        L.alipmpc_solve_slots.restype = ctypes.c_int
    if hasattr(L, "alipmpc_solve_program"):
        L.alipmpc_solve_program.argtypes = [P]
        L.alipmpc_solve_program.restype = ctypes.c_char_p
    if hasattr(L, "alipmpc_build_id"):
        L.alipmpc_build_id.argtypes = []
        L.alipmpc_build_id.restype = ctypes.c_char_p
    L.alipmpc_last_kernel_ms.argtypes = [P]
    L.alipmpc_last_kernel_ms.restype = ctypes.c_double
    L.alipmpc_last_error.argtypes = [P]
    L.alipmpc_last_error.restype = ctypes.c_char_p
    L.alipmpc_destroy.argtypes = [P]
    L.alipmpc_destroy.restype = None
    _lib = L
    return L


# fp32 solve kernels (cfg.precision = PREC_FP32, BASELINE cfg5): the fp64 tolerance 1e-8 is below fp32
# resolution, so unless the caller sets them the fp32 tolerances are tol 1e-4 / acceptable 1e-3 for N <= 3
# and 3e-4 / 3e-3 for longer horizons, whose decision-space gradients (through A^k) are larger and put the
# fp32 stationarity floor higher.  tools/fp32_study.py (profiles/): N = 3 foothold within 1e-3 of the fp64
# solve on 99.8 % of the instances both converge on, same feasible fraction, 1.5x the fp64 throughput;
# N = 5 with ellipses 99 % within 1e-3, 1.7x.
FP32_TOL, FP32_ACCEPTABLE_TOL = 1e-4, 1e-3
FP32_TOL_LONG, FP32_ACCEPTABLE_TOL_LONG = 3e-4, 3e-3


def default_cfg(variant=VARIANT_MODI, N=3, **overrides):
    c = Cfg()
    rc = load().alipmpc_default_cfg(variant, N, ctypes.byref(c))
    if rc != 0:
        raise ValueError(f"alipmpc_default_cfg({variant}, {N}) -> {rc}")
    if overrides.get("precision") == PREC_FP32:
        long_h = N > 3
        overrides.setdefault("tol", FP32_TOL_LONG if long_h else FP32_TOL)
        overrides.setdefault("acceptable_tol", FP32_ACCEPTABLE_TOL_LONG if long_h else FP32_ACCEPTABLE_TOL)
    for k, v in overrides.items():
        if not hasattr(c, k):
            raise AttributeError(k)
        setattr(c, k, v)
    return c


def rows_per_step(cfg):
    return int(load().alipmpc_rows_per_step(ctypes.byref(cfg)))


def num_vars(cfg):
    return int(load().alipmpc_num_vars(ctypes.byref(cfg)))


def trace_len(cfg):
    return int(load().alipmpc_trace_len(ctypes.byref(cfg)))


STREAM_NULL = ctypes.c_void_p(ctypes.c_size_t(-1).value)   # ALIPMPC_STREAM_NULL


def _stream_arg(st):
    """Device-pointer mode needs a non-NULL stream argument: torch's default stream has handle 0, which the
    ABI reads as host-pointer mode, so it is passed as ALIPMPC_STREAM_NULL."""
    h = int(st.cuda_stream)
    return ctypes.c_void_p(h) if h else STREAM_NULL


def _ptr(a):
    if a is None:
        return None
    if hasattr(a, "data_ptr"):          # torch tensor (device mode)
        return ctypes.c_void_p(a.data_ptr())
    return a.ctypes.data_as(ctypes.c_void_p)


class Solver:
    """Owns one libalipmpc handle (one config, one device)."""

    def __init__(self, cfg, device=0):
        self.cfg = cfg
        self.device = device
        self._L = load()
        h = ctypes.c_void_p()
        rc = self._L.alipmpc_create(ctypes.byref(cfg), device, ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(f"alipmpc_create failed: {_ERRORS.get(rc, rc)}")
        self._h = h
        self.n = num_vars(cfg)
        self.rps = rows_per_step(cfg)
        self.m_max = cfg.N * self.rps
        self.sdim = 3 if cfg.variant == VARIANT_DD else 5

    def close(self):
        if getattr(self, "_h", None):
            self._L.alipmpc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = self._L.alipmpc_last_error(self._h).decode()
            raise RuntimeError(f"{what} failed ({_ERRORS.get(rc, rc)}): {msg}")

    def last_kernel_ms(self):
        return float(self._L.alipmpc_last_kernel_ms(self._h))

    def solve_program(self):
        """The device program this handle's solves run (include/alipmpc.h: alipmpc_solve_program)."""
        return self._L.alipmpc_solve_program(self._h).decode()

    def solve_slots(self):
        """Instances the solve kernel holds resident at once; larger batches run the persistent
        work-queue launch (include/alipmpc.h: alipmpc_solve_slots)."""
        v = ctypes.c_int64(0)
        self._check(self._L.alipmpc_solve_slots(self._h, ctypes.byref(v)), "alipmpc_solve_slots")
        return int(v.value)

    def solve_launches(self, B):
        """(kernel launches per solve of B instances, phase-2 team size) — 2 for a split launch
        (include/alipmpc.h: alipmpc_solve_launches)."""
        n, t = ctypes.c_int32(0), ctypes.c_int32(0)
        self._check(self._L.alipmpc_solve_launches(self._h, int(B), ctypes.byref(n), ctypes.byref(t)),
                    "alipmpc_solve_launches")
        return int(n.value), int(t.value)

    def lane_handoffs(self, stream=None):
        """Instances of the last lane-program or fp32 wave-program solve on `stream` (None: the handle's own stream, the
        host-pointer calls) that were handed to the fp64 wave program for IPOPT's restoration phase (include/alipmpc.h)."""
        v = ctypes.c_int64(0)
        st = None if stream is None else _stream_arg(stream)
        self._check(self._L.alipmpc_lane_handoffs(self._h, st, ctypes.byref(v)), "alipmpc_lane_handoffs")
        return int(v.value)

    # ---------------------------------------------------------------- host (numpy) calls
    def _inputs(self, x0, goal, leg, cir, nc, elp, ne):
        cfg = self.cfg
        x0 = np.ascontiguousarray(x0, np.float64).reshape(-1, self.sdim)
        B = x0.shape[0]
        goal = np.ascontiguousarray(np.broadcast_to(np.asarray(goal, np.float64), (B, 2)))
        leg = None if leg is None else np.ascontiguousarray(np.broadcast_to(np.asarray(leg), (B,)), np.int8)
        cir = np.ascontiguousarray(np.broadcast_to(np.asarray(cir, np.float64), (B, cfg.nc_max, 3))) \
            if cfg.nc_max else np.zeros((B, 0, 3))
        nc = np.ascontiguousarray(np.broadcast_to(np.asarray(nc), (B,)), np.int32)
        if cfg.ne_max:
            elp = np.ascontiguousarray(np.broadcast_to(np.asarray(elp, np.float64), (B, cfg.ne_max, 5)))
            ne = np.ascontiguousarray(np.broadcast_to(np.asarray(ne), (B,)), np.int32)
        else:
            elp, ne = None, None
        return B, x0, goal, leg, cir, nc, elp, ne

    def solve(self, x0, goal, leg, cir, nc, elp=None, ne=None, u0=None, last_u=None):
        """Solve a batch from host arrays; returns a dict of numpy outputs."""
        B, x0, goal, leg, cir, nc, elp, ne = self._inputs(x0, goal, leg, cir, nc, elp, ne)
        u0 = np.ascontiguousarray(u0, np.float64).reshape(B, self.n)
        lu = None if last_u is None else np.ascontiguousarray(np.broadcast_to(np.asarray(last_u, np.float64), (B, 2)))
        out = dict(u=np.zeros((B, self.n)), foot=np.zeros((B, 3)), x_pred=np.zeros((B, self.cfg.N, self.sdim)),
                   status=np.zeros(B, np.int32), iters=np.zeros(B, np.int32))
        rc = self._L.alipmpc_solve_batch(self._h, B, _ptr(x0), _ptr(goal), _ptr(leg), _ptr(cir), _ptr(nc), _ptr(elp),
                                         _ptr(ne), _ptr(u0), _ptr(lu), _ptr(out["u"]), _ptr(out["foot"]),
                                         _ptr(out["x_pred"]), _ptr(out["status"]), _ptr(out["iters"]), None)
        self._check(rc, "alipmpc_solve_batch")
        return out

    def eval(self, x0, goal, leg, cir, nc, elp=None, ne=None, u=None, last_u=None, want_J=True):
        B, x0, goal, leg, cir, nc, elp, ne = self._inputs(x0, goal, leg, cir, nc, elp, ne)
        u = np.ascontiguousarray(u, np.float64).reshape(B, self.n)
        lu = None if last_u is None else np.ascontiguousarray(np.broadcast_to(np.asarray(last_u, np.float64), (B, 2)))
        mm = self.m_max
        out = dict(f=np.zeros(B), grad=np.zeros((B, self.n)), c=np.zeros((B, mm)),
                   J=np.zeros((B, mm, self.n)) if want_J else None, cl=np.zeros((B, mm)), cu=np.zeros((B, mm)),
                   goal_eff=np.zeros((B, 2)), row_active=np.zeros((B, mm), np.int8))
        rc = self._L.alipmpc_eval_batch(self._h, B, _ptr(x0), _ptr(goal), _ptr(leg), _ptr(cir), _ptr(nc), _ptr(elp),
                                        _ptr(ne), _ptr(u), _ptr(lu), _ptr(out["f"]), _ptr(out["grad"]),
                                        _ptr(out["c"]), _ptr(out["J"]), _ptr(out["cl"]), _ptr(out["cu"]),
                                        _ptr(out["goal_eff"]), _ptr(out["row_active"]), None)
        self._check(rc, "alipmpc_eval_batch")
        return out

    def rollout(self, x0, goal, leg, cir, nc, elp=None, ne=None, u0=None, last_u=None, steps=8):
        """Closed-loop receding-horizon rollout (alipmpc_rollout_batch) from host arrays.  Returns
        dict(foot (B,S,3), x (B,S+1,sdim), status (B,S), iters (B,S), steps_to_goal (B,), u (B,S,n))."""
        B, x0, goal, leg, cir, nc, elp, ne = self._inputs(x0, goal, leg, cir, nc, elp, ne)
        u0 = np.ascontiguousarray(u0, np.float64).reshape(B, self.n)
        lu = None if last_u is None else np.ascontiguousarray(np.broadcast_to(np.asarray(last_u, np.float64), (B, 2)))
        S = int(steps)
        out = dict(foot=np.zeros((B, S, 3)), x=np.zeros((B, S + 1, self.sdim)), status=np.zeros((B, S), np.int32),
                   iters=np.zeros((B, S), np.int32), steps_to_goal=np.zeros(B, np.int32),
                   u=np.zeros((B, S, self.n)))
        rc = self._L.alipmpc_rollout_batch(self._h, B, S, _ptr(x0), _ptr(goal), _ptr(leg), _ptr(cir), _ptr(nc),
                                           _ptr(elp), _ptr(ne), _ptr(u0), _ptr(lu), _ptr(out["foot"]),
                                           _ptr(out["x"]), _ptr(out["status"]), _ptr(out["iters"]),
                                           _ptr(out["steps_to_goal"]), _ptr(out["u"]), None)
        self._check(rc, "alipmpc_rollout_batch")
        return out

    def closed_loop(self, x0, foot0, goal, leg, cir, nc, elp=None, ne=None, steps=8, f_cyc=40, kick=0.0, seed=0):
        """Closed loop at the reference's control rate (alipmpc_closed_loop_batch): B episodes, up to `steps`
        walking steps, f_cyc solves per step on an ALIP plant with an optional seeded velocity kick.
        Returns dict(foot (B,S,3), x (B,S+1,5), hd (B,S,2), status (B,S,f_cyc), iters (B,S,f_cyc),
        steps_to_goal (B,), action (B,S,f_cyc,8): the controller command of every tick)."""
        B, x0, goal, leg, cir, nc, elp, ne = self._inputs(x0, goal, leg, cir, nc, elp, ne)
        foot0 = np.ascontiguousarray(foot0, np.float64).reshape(B, 2)
        S, F = int(steps), int(f_cyc)
        out = dict(foot=np.zeros((B, S, 3)), x=np.zeros((B, S + 1, 5)), hd=np.zeros((B, S, 2)),
                   status=np.zeros((B, S, F), np.int32), iters=np.zeros((B, S, F), np.int32),
                   steps_to_goal=np.zeros(B, np.int32), action=np.zeros((B, S, F, 8)))
        rc = self._L.alipmpc_closed_loop_batch(self._h, B, S, F, float(kick), int(seed), _ptr(x0), _ptr(foot0),
                                               _ptr(goal), _ptr(leg), _ptr(cir), _ptr(nc), _ptr(elp), _ptr(ne),
                                               _ptr(out["foot"]), _ptr(out["x"]), _ptr(out["hd"]),
                                               _ptr(out["status"]), _ptr(out["iters"]), _ptr(out["steps_to_goal"]),
                                               _ptr(out["action"]), None)
        self._check(rc, "alipmpc_closed_loop_batch")
        return out

    def closed_loop_device(self, inp, out, steps, f_cyc=40, kick=0.0, seed=0, stream=None):
        """Asynchronous closed loop on device tensors: inp x0 (B,5), foot0 (B,2), goal, leg (int8), cir, nc
        [, elp, ne]; out dict with any of foot, x, hd, status, iters, steps_to_goal, action (shapes of
        closed_loop)."""
        import torch
        st = stream if stream is not None else torch.cuda.current_stream()
        B = inp["x0"].shape[0]
        rc = self._L.alipmpc_closed_loop_batch(
            self._h, B, int(steps), int(f_cyc), float(kick), int(seed), _ptr(inp["x0"]), _ptr(inp["foot0"]),
            _ptr(inp["goal"]), _ptr(inp["leg"]), _ptr(inp["cir"]), _ptr(inp["nc"]), _ptr(inp.get("elp")),
            _ptr(inp.get("ne")), _ptr(out.get("foot")), _ptr(out.get("x")), _ptr(out.get("hd")),
            _ptr(out.get("status")), _ptr(out.get("iters")), _ptr(out.get("steps_to_goal")), _ptr(out.get("action")),
            _stream_arg(st))
        self._check(rc, "alipmpc_closed_loop_batch")

    def nominal_gait(self, x, leg=None, vx_max=0.6, vel_des=None):
        """Nominal gait (alipmpc_nominal_gait_batch): returns (vel_des (B,2), foot (B,2)) — alip_des_vel(vx_max,
        leg_ind) per instance (or the given vel_des) and cal_foot_with_veldes(x, vel_des)."""
        x = np.ascontiguousarray(x, np.float64).reshape(-1, 5)
        B = x.shape[0]
        lg = None if leg is None else np.ascontiguousarray(np.broadcast_to(np.asarray(leg), (B,)), np.int8)
        vin = None if vel_des is None else np.ascontiguousarray(np.broadcast_to(vel_des, (B, 2)), np.float64)
        vout, foot = np.zeros((B, 2)), np.zeros((B, 2))
        rc = self._L.alipmpc_nominal_gait_batch(self._h, B, float(vx_max), _ptr(x), _ptr(lg), _ptr(vin), _ptr(vout),
                                                _ptr(foot), None)
        self._check(rc, "alipmpc_nominal_gait_batch")
        return vout, foot

    def trace(self, x0, u):
        """Dense plan traces (alipmpc_trace_batch): x0 (B,5), u (B,5N) -> (B, N, trace_len, 2)."""
        x0 = np.ascontiguousarray(x0, np.float64).reshape(-1, 5)
        B = x0.shape[0]
        u = np.ascontiguousarray(u, np.float64).reshape(B, self.n)
        out = np.zeros((B, self.cfg.N, trace_len(self.cfg), 2))
        rc = self._L.alipmpc_trace_batch(self._h, B, _ptr(x0), _ptr(u), _ptr(out), None)
        self._check(rc, "alipmpc_trace_batch")
        return out

    # ---------------------------------------------------------------- device (torch) calls
    def rollout_device(self, inp, out, steps, stream=None):
        """Asynchronous rollout on device tensors: inp as solve_device, out dict with any of foot (B,S,3),
        x (B,S+1,sdim), status (B,S), iters (B,S), steps_to_goal (B,), u (B,S,n)."""
        import torch
        st = stream if stream is not None else torch.cuda.current_stream()
        B = inp["x0"].shape[0]
        rc = self._L.alipmpc_rollout_batch(
            self._h, B, int(steps), _ptr(inp["x0"]), _ptr(inp["goal"]), _ptr(inp.get("leg")), _ptr(inp["cir"]),
            _ptr(inp["nc"]), _ptr(inp.get("elp")), _ptr(inp.get("ne")), _ptr(inp["u0"]), _ptr(inp.get("last_u")),
            _ptr(out.get("foot")), _ptr(out.get("x")), _ptr(out.get("status")), _ptr(out.get("iters")),
            _ptr(out.get("steps_to_goal")), _ptr(out.get("u")), _stream_arg(st))
        self._check(rc, "alipmpc_rollout_batch")

    def trace_device(self, x0, u, trace, stream=None):
        """Asynchronous dense plan traces on device tensors x0 (B,5), u (B,5N) -> trace (B,N,trace_len,2)."""
        import torch
        st = stream if stream is not None else torch.cuda.current_stream()
        rc = self._L.alipmpc_trace_batch(self._h, x0.shape[0], _ptr(x0), _ptr(u), _ptr(trace), _stream_arg(st))
        self._check(rc, "alipmpc_trace_batch")

    def solve_device(self, inp, out, stream=None):
        """Asynchronous solve on device tensors.  inp/out: dicts of torch CUDA tensors with the shapes of
        solve(); stream: torch.cuda.Stream (defaults to the current stream)."""
        import torch
        st = stream if stream is not None else torch.cuda.current_stream()
        B = inp["x0"].shape[0]
        rc = self._L.alipmpc_solve_batch(
            self._h, B, _ptr(inp["x0"]), _ptr(inp["goal"]), _ptr(inp["leg"]), _ptr(inp["cir"]), _ptr(inp["nc"]),
            _ptr(inp.get("elp")), _ptr(inp.get("ne")), _ptr(inp["u0"]), _ptr(inp.get("last_u")),
            _ptr(out["u"]), _ptr(out.get("foot")), _ptr(out.get("x_pred")), _ptr(out.get("status")),
            _ptr(out.get("iters")), _stream_arg(st))
        self._check(rc, "alipmpc_solve_batch")

    def eval_device(self, inp, out, stream=None):
        import torch
        st = stream if stream is not None else torch.cuda.current_stream()
        B = inp["x0"].shape[0]
        rc = self._L.alipmpc_eval_batch(
            self._h, B, _ptr(inp["x0"]), _ptr(inp["goal"]), _ptr(inp["leg"]), _ptr(inp["cir"]), _ptr(inp["nc"]),
            _ptr(inp.get("elp")), _ptr(inp.get("ne")), _ptr(inp["u"]), _ptr(inp.get("last_u")),
            _ptr(out.get("f")), _ptr(out.get("grad")), _ptr(out.get("c")), _ptr(out.get("J")), _ptr(out.get("cl")),
            _ptr(out.get("cu")), _ptr(out.get("goal_eff")), _ptr(out.get("row_active")),
            _stream_arg(st))
        self._check(rc, "alipmpc_eval_batch")
