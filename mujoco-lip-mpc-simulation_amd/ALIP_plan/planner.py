"""ALIP_plan/planner.py — the C-ABI dispatch shim named by the north star.

The reference's ALIP_plan/planner.py (class ALIP, planner.py:14) is a legacy one-step planner that
nothing imports; the working planner surface callers use is MPCCBF (MPC_LIP_modi.py:13-391), so this
module exports that surface backed by libalipmpc.so (see alipmpc/planner.py for the signatures).
"""
from alipmpc.planner import MPCCBF, MPCCBFDD, MPCCBFSigStep  # noqa: F401

__all__ = ["MPCCBF", "MPCCBFSigStep", "MPCCBFDD"]
