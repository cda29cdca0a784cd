#!/usr/bin/env python3
"""Recompute the bench line's `roofline` fields from a committed profile directory.

  python tools/roofline.py profiles/r2/cfg2 [--write profiles/solve_kernel_counters.json]
  python tools/roofline.py profiles/r2/sweep/r2t --sweep 'sweep_kernel<5,true,32,2>' [--write ...]

The directory holds what tools/gpu_run.sh's `prof` step collects for ONE bench config:
  bench.json                       the bench line of the profiled build (kernel name, B, iterations, peaks)
  prof_kt/kt_kernel_stats.csv      rocprofv3 --kernel-trace --stats of `bench.py --steps 10`
  pmc_*/pmc_counter_collection.csv rocprofv3 --pmc passes of `bench.py --steps 3 --warmup 1` (one pass each)

Every record carries the alipmpc_build_id of the profiled library (bench.json config.build_id); bench.py attaches a
record to its line only when that id equals the id of the library it is timing.

Fields (per solve of the dominant solve kernel — a split launch's two dispatches summed, config.launches_per_solve; the
first solve of every pass is the warmup and skipped):
  kernel_ms          kernel-trace average duration (the bench's own HIP-event figure must agree)
  achieved / frac    algorithmic FP64 flops per launch (flops_per_iter x instance-iterations) / kernel_ms, / peak
  traffic            HBM bytes: 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md: FETCH_SIZE counts half the
                     bytes of wide reads on gfx950; both in KiB)
  valu_issue_frac    SQ_INSTS_VALU x 4 cycles / SIMD-cycles (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs): the share of
                     the chip's vector-issue slots the kernel used (a wave64 VALU op holds a SIMD >= 4 cycles)
  active_issue_frac  SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES: the share of resident-wave time spent issuing
  mfma_busy_share    SQ_VALU_MFMA_BUSY_CYCLES / SIMD-cycles
  insts_per_iter     SQ_INSTS / instance-iterations (VALU / SALU / LDS / MFMA split alongside)
  lds_conflict_share SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS, XCDS = 1024, 8


def counters(d, kern, skip=1):
    """Per-dispatch means of the kernel's counters over the dispatches of the benchmarked batch: the largest grid of
    the family (bench.py's latency probe and feasibility checks launch the same kernel on small grids)."""
    acc = defaultdict(list)
    meta = {}
    for f in sorted(glob.glob(os.path.join(d, "pmc_*", "pmc_counter_collection.csv"))):
        rows = [r for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith(kern)]
        if rows:
            g = max(int(r["Grid_Size"]) for r in rows)
            rows = [r for r in rows if int(r["Grid_Size"]) == g]
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})[skip:]
        for r in rows:
            if int(r["Dispatch_Id"]) in ids:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta = meta or {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size",
                                                   "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count")}
    return {k: sum(v) / len(v) for k, v in acc.items()}, meta


def kernel_ms(d, kern, launches=1):
    """Mean duration per SOLVE of the kernel family: launches per solve x the mean dispatch (a split launch runs
    phase 1 and phase 2 of every solve as two dispatches of the same kernel).  From the per-dispatch trace when present,
    restricted like counters() to the largest grid of the family; else the stats summary."""
    for f in glob.glob(os.path.join(d, "prof_kt", "*kernel_trace.csv")):
        rows = [r for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith(kern)]
        if rows:
            def gs(r):
                return int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            g = max(gs(r) for r in rows)
            dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if gs(r) == g]
            return launches * sum(dur) / len(dur) * 1e-6, len(dur)
    for f in glob.glob(os.path.join(d, "prof_kt", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            if r["Name"].startswith(kern):
                return launches * float(r["AverageNs"]) * 1e-6, int(r["Calls"])
    return None, 0


def sweep(a):
    """The Jacobian sweep's fields (tools/gpu_sweep_prof.sh: bench.jacobian_sweep alone, no bench.json): HBM bound,
    algorithmic bytes = bytes_per_instance x B (bench.py's formula), kernel-trace mean duration, PMC traffic."""
    kname = a.sweep
    kern = "void alip::" + kname.replace(",", ", ")[:-1]
    c, meta = counters(a.dir, kern)
    ms, calls = kernel_ms(a.dir, kern)
    out = {"kernel": kname, "B": a.batch, "bytes_per_instance": a.bytes, "kernel_ms_trace": ms, "trace_calls": calls,
           "build_id": a.build_id, "profile_dir": a.dir}
    if ms:
        ach = a.batch * a.bytes / (ms * 1e-3) / 1e9
        out.update(achieved=ach, peak=8000.0, unit="GB/s", frac=ach / 8000.0)
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        out["hbm_bytes_per_launch"] = 1024.0 * (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"])
        out["algorithmic_bytes_per_launch"] = a.batch * a.bytes
        out["fetch_kib"], out["write_kib"] = c["FETCH_SIZE"], c["WRITE_SIZE"]
    if "GRBM_GUI_ACTIVE" in c and "SQ_INSTS_VALU" in c:
        out["valu_issue_frac"] = 4.0 * c["SQ_INSTS_VALU"] / (SIMDS * c["GRBM_GUI_ACTIVE"] / XCDS)
    if "SQ_ACTIVE_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
        out["active_issue_frac"] = c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"]
    out["vgpr"] = meta.get("VGPR_Count") if meta else None
    print(json.dumps(out, indent=1))
    if a.write:
        db = json.load(open(a.write)) if os.path.exists(a.write) else {}
        db[f"{kname}|B={a.batch}"] = out
        with open(a.write, "w") as fh:
            json.dump(db, fh, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--write", default=None, help="merge the counter fields into this JSON (bench.py reads it)")
    ap.add_argument("--sweep", default=None, help="Jacobian-sweep kernel name, e.g. 'sweep_kernel<5,true,32,2>'")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--bytes", type=int, default=4272)
    ap.add_argument("--build-id", default=None, help="--sweep: alipmpc_build_id of the profiled library "
                    "(default: <dir>/build_id.txt)")
    a = ap.parse_args()
    if a.sweep:
        if a.build_id is None and os.path.exists(os.path.join(a.dir, "build_id.txt")):
            a.build_id = open(os.path.join(a.dir, "build_id.txt")).read().strip()
        return sweep(a)
    bench = json.load(open(os.path.join(a.dir, "bench.json")))
    rl = bench["roofline"]
    kname = rl["kernel"]
    kern = "void alip::" + kname.replace(",", ", ") if not kname.startswith("void") else kname
    kern = kern[:-1] if kern.endswith(">") else kern   # the family: solve_kernel<..., true/false> (launch form)
    # per-solve figures: counters of the launches of one solve summed (first solve = warmup, skipped)
    launches = int(bench["config"].get("launches_per_solve", 1))
    c, meta = counters(a.dir, kern, skip=launches)
    c = {k: v * launches for k, v in c.items()}
    ms, calls = kernel_ms(a.dir, kern, launches)
    its = rl["iters_per_launch"]
    out = {"kernel": kname, "B": bench["config"]["batch_per_gpu"], "N": bench["config"]["horizon"],
           "launches_per_solve": launches,
           "dtype": bench["dtype"], "build_id": bench["config"].get("build_id"), "profile_dir": a.dir,
           "kernel_ms_trace": ms, "trace_calls": calls, "kernel_ms_bench": rl["kernel_ms"]}
    if ms:
        ach = rl["flops_per_iter"] * its / (ms * 1e-3) / 1e12
        out.update(achieved=ach, peak=rl["peak"], frac=ach / rl["peak"])
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        out["hbm_bytes_per_launch"] = 1024.0 * (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"])
        out["fetch_kib"], out["write_kib"] = c["FETCH_SIZE"], c["WRITE_SIZE"]
    if "GRBM_GUI_ACTIVE" in c:
        simd_cycles = SIMDS * c["GRBM_GUI_ACTIVE"] / XCDS
        out["simd_cycles"] = simd_cycles
        if "SQ_INSTS_VALU" in c:
            out["valu_issue_frac"] = 4.0 * c["SQ_INSTS_VALU"] / simd_cycles
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            out["mfma_busy_share"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles
        if ms:
            out["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / XCDS / (ms * 1e-3) / 1e9
    if "SQ_ACTIVE_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
        out["active_issue_frac"] = c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"]
    if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
        out["wait_inst_frac"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
    for k in ("SQ_INSTS", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_MFMA"):
        if k in c:
            out[k.lower().replace("sq_", "") + "_per_iter"] = c[k] / its
    if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_conflict_share"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
    out["scratch_bytes_per_lane"] = int(meta.get("Scratch_Size", -1)) if meta else None
    out["counters"] = c
    print(json.dumps(out, indent=1))
    # the bench line's own fields, for comparison
    print("bench roofline:", json.dumps({k: rl[k] for k in ("achieved", "peak", "frac", "traffic", "kernel_ms")}),
          file=sys.stderr)
    if a.write:
        db = json.load(open(a.write)) if os.path.exists(a.write) else {}
        db[f"{kname}|B={out['B']}"] = {k: v for k, v in out.items() if k != "counters"}
        with open(a.write, "w") as fh:
            json.dump(db, fh, indent=1)


if __name__ == "__main__":
    main()
