#!/bin/bash
# quick GPU iteration: gpu tests + perf sweep
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
TAG=${1:-q}
timeout -k 10 900 python -u -m pytest $R/tests -x -v --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_$TAG.log 2>&1; rc=$?; tail -4 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python $R/tools/perf_sweep.py > $OUT/sweep_$TAG.log 2>&1 || { tail $OUT/sweep_$TAG.log; exit 1; }
grep '^{' $OUT/sweep_$TAG.log
