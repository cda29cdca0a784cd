#!/usr/bin/env python3
"""Per-group tick phases of the closed loop from a rocprofv3 kernel trace (tools/cl_trace.sh): for each HW queue (one
per episode group) the phase-1 and phase-2 solve dispatches of every tick and the small per-tick kernels.

  python tools/cl_trace_summary.py gpurun_out/clkt [label]
"""
import collections
import csv
import os
import sys

import numpy as np


def main(d, label=""):
    rows = list(csv.DictReader(open(os.path.join(d, "kt_kernel_trace.csv"))))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    inits = [i for i, r in enumerate(rows) if "cl_init" in r["Kernel_Name"]]
    seg = rows[inits[-1]:]   # the last loop of the process
    by, small = collections.defaultdict(list), collections.Counter()
    t0 = int(seg[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in seg if "copyBuffer" not in r["Kernel_Name"])
    for r in seg:
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "solve_kernel" in r["Kernel_Name"]:
            by[r["Queue_Id"]].append(dur)
        elif "copyBuffer" not in r["Kernel_Name"]:
            small[r["Queue_Id"]] += dur
    print(f"{label}: last loop {(t1 - t0) / 1e6:.2f} ms (first kernel start to last kernel end)")
    for q, v in by.items():
        p1, p2 = np.array(v[0::2]), np.array(v[1::2])
        print(f"  queue {q}: phase 1 mean {p1.mean():.1f} us, max {p1.max():.1f} us, sum {p1.sum() / 1e3:.2f} ms | "
              f"phase 2 mean {p2.mean():.1f} us, max {p2.max():.1f} us, sum {p2.sum() / 1e3:.2f} ms | "
              f"project + memset + update {small[q] / 1e3:.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else sys.argv[1])
