#!/bin/bash
# PMC passes of the solve kernel at two batch sizes (1 vs 4 waves per SIMD), one rocprofv3 run per group.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for B in 1024 4096; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_LDS SQ_IFETCH SQ_INST_CYCLES_SALU" \
             "SQC_ICACHE_HITS SQC_ICACHE_MISSES" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_VALU2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmcb${B}_p$i -o pmc -- python3 $R/bench.py --batch $B --steps 2 --warmup 1 --no-cpu-baseline --sweep-batch 0 > $OUT/pmcb${B}_p$i.txt 2>&1 || { tail -5 $OUT/pmcb${B}_p$i.txt; exit 1; }
  done
done
echo pmc-done
