#!/bin/bash
# GPU-box script: tests, bench, rocprofv3 kernel trace + PMC passes.  Every GPU step has its own time
# limit and the chain stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r1}
step() { echo "=== $*" ; }
step pytest && timeout -k 10 900 python -u -m pytest $R/tests -x -v --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_gpu_$TAG.log 2>&1; rc=$?; tail -5 $OUT/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
step smoke && timeout -k 10 300 python -c "import sys; sys.path.insert(0,'$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { cat $OUT/smoke_$TAG.log; exit 1; }
cat $OUT/smoke_$TAG.log
step bench && timeout -k 10 300 python $R/bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
cd /tmp
step rocprof-kt && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_kt_$TAG -o kt -- python3 $R/bench.py --steps 10 --no-cpu-baseline > $OUT/prof_kt_$TAG.log 2>&1 || { tail -20 $OUT/prof_kt_$TAG.log; exit 1; }
step rocprof-pmc-fetch && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_pmc_fetch_$TAG -o pmc -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof_pmc_fetch_$TAG.log 2>&1 || { tail -20 $OUT/prof_pmc_fetch_$TAG.log; exit 1; }
step rocprof-pmc-write && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_pmc_write_$TAG -o pmc -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof_pmc_write_$TAG.log 2>&1 || { tail -20 $OUT/prof_pmc_write_$TAG.log; exit 1; }
step done
find $OUT -name "*stats*" -o -name "*counter_collection*" | head
