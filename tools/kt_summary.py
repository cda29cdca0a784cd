#!/usr/bin/env python3
"""Dev: mean duration per (kernel, grid) of a rocprofv3 kernel-trace csv.  python tools/kt_summary.py <dir>"""
import csv
import glob
import sys
from collections import defaultdict

for fn in sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)):
    d = defaultdict(list)
    with open(fn) as fh:
        for r in csv.DictReader(fh):
            k = (r["Kernel_Name"][:70], r.get("Grid_Size_X") or r.get("Grid_Size"))
            d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    print(fn)
    for (k, g), v in sorted(d.items(), key=lambda t: -sum(t[1])):
        print(f"  {k:70s} grid {g:>8s} n {len(v):4d} mean {sum(v) / len(v):9.1f} us")
