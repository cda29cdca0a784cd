"""Copy the rocprofv3 summaries of a GPU round from gpurun_out/ into profiles/<tag>/ and derive the
per-launch HBM traffic of solve_kernel from the PMC passes (FETCH_SIZE / WRITE_SIZE are in KiB; the
gfx950 'x2 for wide coalesced streaming reads' correction does not apply to this kernel's narrow
scalar/scratch/LDS-staging loads, so FETCH_SIZE is taken as reported — see DESIGN.md)."""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pmc(path, kernel):
    vals, names = [], set()
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if kernel in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
                names.add(r["Kernel_Name"])
    return vals, names


def main(tag, B=4096, N=3):
    src = os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    for sub, name in [(f"prof_kt_{tag}/kt_kernel_stats.csv", "kernel_stats.csv"),
                      (f"prof_kt_{tag}/kt_domain_stats.csv", "domain_stats.csv"),
                      (f"prof_pmc_fetch_{tag}/pmc_counter_collection.csv", "pmc_fetch_size.csv"),
                      (f"prof_pmc_write_{tag}/pmc_counter_collection.csv", "pmc_write_size.csv"),
                      (f"bench_{tag}.json", "bench.json"), (f"pytest_gpu_{tag}.log", "pytest_gpu.log")]:
        p = os.path.join(src, sub)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, name))
    f, names = pmc(os.path.join(dst, "pmc_fetch_size.csv"), "solve_kernel")
    w, _ = pmc(os.path.join(dst, "pmc_write_size.csv"), "solve_kernel")
    if f and w:
        fetch = sum(f) / len(f) * 1024
        write = sum(w) / len(w) * 1024
        out = {"B": B, "N": N, "kernel": sorted(names)[0], "fetch_bytes_per_launch": fetch,
               "write_bytes_per_launch": write, "hbm_bytes_per_launch": fetch + write,
               "source": f"profiles/{tag}/pmc_*_size.csv (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)"}
        with open(os.path.join(dst, "solve_kernel_traffic.json"), "w") as fh:
            json.dump(out, fh, indent=1)
        with open(os.path.join(ROOT, "profiles", "solve_kernel_traffic.json"), "w") as fh:
            json.dump(out, fh, indent=1)
        print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
