"""Dev: cfg2 launch time vs batch size at the reference iteration cap (is the launch tail-latency bound?)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from perf_sweep import run  # noqa: E402

if __name__ == "__main__":
    for B in [64, 256, 1024, 2048, 4096, 8192, 16384]:
        print(json.dumps(run(B, max_iter=30)), flush=True)
    # same instance replicated: every wave does identical work (no iteration-count spread)
