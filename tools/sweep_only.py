"""Dev: time only the Jacobian sweep (eval_kernel, bench.jacobian_sweep) — the program for rocprofv3
kernel-trace / PMC passes of that kernel.   python tools/sweep_only.py [B] [reps]"""
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (puts the package on sys.path)
import torch  # noqa: E402
import alipmpc  # noqa: E402
from alipmpc import scenes  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
args = types.SimpleNamespace(sweep_batch=B, seed=0)
print(json.dumps(bench.jacobian_sweep(alipmpc, scenes, 0, args, torch.device("cuda", 0), reps=reps)))
