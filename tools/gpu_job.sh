#!/bin/bash
# One parameterised GPU-box job (replaces the per-run tools/_r5*.sh scripts): tools/gpu_job.sh TAG STEP...
#   check            tools/resto_gpu_check.py (wave program vs the C oracle, both restoration modes, cfg2 timing)
#   pytest:EXPR      pytest -m gpu -k EXPR (EXPR "all": the whole GPU suite), stop at the first failure
#   survey:EXPR      the same, up to 40 failures (a survey of what a change broke)
#   smoke            __graft_entry__.smoke()
#   bench[:ARGS]     bench.py ARGS (default line with no args)
#   gpurun:...       any tools/gpu_run.sh step list (tests bench configs prof wst), comma-separated
# Every GPU step has its own time limit; the chain stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export ALIPMPC_TEST_ARTIFACTS=$OUT/art
n=0
for step in "$@"; do
  n=$((n + 1))
  case $step in
  check)
    timeout -k 10 600 python -u $R/tools/resto_gpu_check.py > $OUT/check.log 2>&1 || { tail -30 $OUT/check.log; exit 1; }
    grep -v amdgpu.ids $OUT/check.log ;;
  pytest:*|survey:*)
    k=${step#*:}
    sel=(); [ "$k" = all ] || sel=(-k "$k")
    stop=-x; case $step in survey:*) stop="--maxfail=40";; esac
    timeout -k 10 1100 python -u -m pytest $R/tests $stop -v --timeout 120 --timeout-method thread -m gpu "${sel[@]}" > $OUT/pytest_$n.log 2>&1; rc=$?
    tail -4 $OUT/pytest_$n.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $OUT/pytest_$n.log | head -90; exit $rc; } ;;
  smoke)
    timeout -k 10 300 python -c "import sys; sys.path.insert(0,'$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
    cat $OUT/smoke.log ;;
  bench*)
    a=${step#bench}; a=${a#:}
    timeout -k 10 400 python $R/bench.py $a > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { tail -20 $OUT/bench_$n.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_$n.json'));print('bench $a', round(d['value']), d['ms_per_step'], d['config'].get('mean_iters'), d['config'].get('status_counts'), d['roofline'].get('kernel_ms'))" ;;
  gpurun:*)
    bash $R/tools/gpu_run.sh $TAG $(echo ${step#gpurun:} | tr , ' ') || exit 1 ;;
  esac
done
echo "=== job done"
