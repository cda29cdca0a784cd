#!/bin/bash
# Instruction-cache PMC pass of the cfg2 bench solve, per restoration mode (r6: the restoration-capable build's code
# size): rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS SQ_WAIT_INST_ANY, one run per mode, plus a kernel
# trace of the same command.   tools/pmc_icache.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for mode in ipopt substitute; do
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS SQ_WAIT_INST_ANY --output-format csv -d $OUT/ic_$mode -o pmc -- python3 $R/bench.py --config cfg2 --steps 10 --warmup 2 --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --restoration $mode > $OUT/ic_$mode.txt 2>&1 || { tail -5 $OUT/ic_$mode.txt; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$mode -o kt -- python3 $R/bench.py --config cfg2 --steps 10 --warmup 2 --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --restoration $mode > $OUT/kt_$mode.txt 2>&1 || { tail -5 $OUT/kt_$mode.txt; exit 1; }
done
echo pmc-done
