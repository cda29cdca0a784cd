"""Dev: the bench's Jacobian sweep (bench.jacobian_sweep) at several batch sizes in one process."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import alipmpc  # noqa: E402
from alipmpc import scenes  # noqa: E402


class A:
    seed = 0


for bs in [int(x) for x in (sys.argv[1:] or ["65536", "131072", "262144", "524288"])]:
    A.sweep_batch = bs
    r = bench.jacobian_sweep(alipmpc, scenes, alipmpc.VARIANT_MODI, A, torch.device("cuda", 0), reps=20)
    print(bs, "kernel_ms %.4f" % r["kernel_ms"], "GB/s %.0f" % r["achieved"], "frac %.3f" % r["frac"], flush=True)
