"""Mean per-dispatch PMC counters of one kernel over rocprofv3 --pmc passes: pmc_summary.py DIR [KERNEL] [SKIP]
(DIR holds pmc_*/pmc_counter_collection.csv; SKIP = leading dispatches of the kernel to ignore, e.g. warmup)."""
import csv, glob, sys, collections
d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "solve_kernel"
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 1
acc = collections.defaultdict(list)
meta = None
for f in sorted(glob.glob(f"{d}/pmc_*/pmc_counter_collection.csv")):
    rows = [r for r in csv.DictReader(open(f)) if kern in r["Kernel_Name"]]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})[skip:]
    for r in rows:
        if int(r["Dispatch_Id"]) in ids:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = meta or {k: r[k] for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                                               "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count")}
print(meta)
for k, v in sorted(acc.items()):
    print(f"{k:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
