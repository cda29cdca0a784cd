#!/bin/bash
# PMC passes (instruction mix / issue, then LDS / memory) of the eval kernel over the Jacobian sweep
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
TAG=${1:-sw}
timeout -k 10 120 python3 $R/tools/sweep_only.py > $OUT/sweep_${TAG}.json 2>&1 || { tail -5 $OUT/sweep_${TAG}.json; exit 1; }
cat $OUT/sweep_${TAG}.json
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES --output-format csv -d $OUT/pmcsw_${TAG}_1 -o pmc -- python3 $R/tools/sweep_only.py 65536 3 > $OUT/pmcsw_${TAG}_1.txt 2>&1 || { tail -5 $OUT/pmcsw_${TAG}_1.txt; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcsw_${TAG}_2 -o pmc -- python3 $R/tools/sweep_only.py 65536 3 > $OUT/pmcsw_${TAG}_2.txt 2>&1 || { tail -5 $OUT/pmcsw_${TAG}_2.txt; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY --output-format csv -d $OUT/pmcsw_${TAG}_3 -o pmc -- python3 $R/tools/sweep_only.py 65536 3 > $OUT/pmcsw_${TAG}_3.txt 2>&1 || { tail -5 $OUT/pmcsw_${TAG}_3.txt; exit 1; }
python3 - <<PY
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob("$OUT/pmcsw_${TAG}_*/pmc_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "eval_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k, sum(v) / len(v))
PY
