#!/bin/bash
# A/B kernel-variant timing on the GPU box: tools/ab.sh <tag> <lib-or-"default">... (CONFIGS env, default "cfg2 cfg4")
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
TAG=$1; shift
for rep in 1 2; do
  for lib in "$@"; do
    for c in ${CONFIGS:-cfg2 cfg4}; do
      if [ "$lib" = default ]; then unset ALIPMPC_LIB; else export ALIPMPC_LIB=$R/$lib; fi
      timeout -k 10 120 python -u $R/bench.py --config $c --no-cpu-baseline --sweep-batch 0 --steps 20 > $OUT/ab_${TAG}.tmp 2>>$OUT/ab_${TAG}.err || exit 1
      python -c "import json,sys;d=json.load(open('$OUT/ab_${TAG}.tmp'));print('$lib', '$c', round(d['value']), round(d['roofline']['kernel_ms'],4), d['config']['mean_iters'])" | tee -a $OUT/ab_${TAG}.log
    done
  done
done
