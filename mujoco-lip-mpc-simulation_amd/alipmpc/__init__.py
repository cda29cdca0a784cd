"""alipmpc — MI355X-native batched ALIP-MPC-CBF footstep planner (HIP kernels behind a C ABI).

  Solver       one libalipmpc.so handle: batched solve / eval on host or device buffers
  default_cfg  the reference's constants per variant (modi / sig_step / dd)
  planner      MPCCBF drop-in (reference MPC_LIP_modi.MPCCBF signatures) + solve_batch
"""
from ._lib import (Cfg, Solver, default_cfg, load, lib_path, build_id, num_vars, rows_per_step, trace_len, EXPORTS, STATUS_NAMES,
                   VARIANT_MODI, VARIANT_SIG_STEP, VARIANT_DD, PREC_FP64, PREC_FP32, PROGRAM_WAVE, PROGRAM_LANE,
                   ROLLOUT_DONE, FP32_TOL,
                   FP32_ACCEPTABLE_TOL, FP32_TOL_LONG, FP32_ACCEPTABLE_TOL_LONG, GOAL_SINGULAR_ZERO,
                   GOAL_SINGULAR_ABORT, INVALID_NUMBER_DETECTED, RESTORATION_IPOPT, RESTORATION_SUBSTITUTE)

__all__ = ["Cfg", "Solver", "default_cfg", "load", "lib_path", "build_id", "num_vars", "rows_per_step", "trace_len", "EXPORTS",
           "STATUS_NAMES", "VARIANT_MODI", "VARIANT_SIG_STEP", "VARIANT_DD", "PREC_FP64", "PREC_FP32",
           "PROGRAM_WAVE", "PROGRAM_LANE", "ROLLOUT_DONE", "FP32_TOL", "FP32_ACCEPTABLE_TOL",
           "FP32_TOL_LONG", "FP32_ACCEPTABLE_TOL_LONG", "GOAL_SINGULAR_ZERO", "GOAL_SINGULAR_ABORT",
           "INVALID_NUMBER_DETECTED", "RESTORATION_IPOPT", "RESTORATION_SUBSTITUTE"]
