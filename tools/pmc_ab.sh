#!/bin/bash
# one PMC pass (instruction mix + issue waits) of the solve kernel for several library variants
#   tools/pmc_ab.sh <tag> default|<lib.so>...      (B=<batch> env, default 4096)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B=${B:-4096}
TAG=$1; shift
for lib in "$@"; do
  if [ "$lib" = default ]; then unset ALIPMPC_LIB; else export ALIPMPC_LIB=$R/$lib; fi
  nm=$(basename $lib .so)
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_BRANCH --output-format csv -d $OUT/pmcab_${TAG}_$nm -o pmc -- python3 $R/bench.py --batch $B --steps 2 --warmup 1 --no-cpu-baseline --sweep-batch 0 > $OUT/pmcab_${TAG}_$nm.txt 2>&1 || { tail -5 $OUT/pmcab_${TAG}_$nm.txt; exit 1; }
done
echo done
