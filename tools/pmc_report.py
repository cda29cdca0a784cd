"""Summarise PMC passes (gpurun_out/<tag>_p*/pmc_counter_collection.csv) for one kernel: mean per dispatch."""
import csv, glob, sys, collections
tag = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "solve_kernel"
acc = collections.defaultdict(list)
for f in sorted(glob.glob(f"gpurun_out/{tag}_p*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(f"{k:32s} {sum(v)/len(v):16.1f}  (n={len(v)})")
