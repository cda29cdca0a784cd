"""Dev: the bench's Jacobian sweep alone (eval_kernel on 65536 cfg2-shaped instances), for rocprofv3 passes."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import bench

class A:
    sweep_batch = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    seed = 0
sys.path.insert(0, os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd"))
import alipmpc
from alipmpc import scenes
r = bench.jacobian_sweep(alipmpc, scenes, alipmpc.VARIANT_MODI, A, torch.device("cuda", 0), reps=6)
print(r)
