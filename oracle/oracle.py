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
                 "dtheta_max", "q", "p", "r", "gamma", "s", "detect_r2", "dd_t", "mu_init")]


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
