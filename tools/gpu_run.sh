#!/bin/bash
# GPU-box driver for one iteration: `tools/gpu_run.sh TAG [tests] [bench] [configs] [prof] [wst]`.
# Every GPU step has its own time limit; the chain stops at the first failure.
#   tests    pytest -m gpu + smoke
#   bench    the default bench line (cfg2, with CPU baselines, closed loop, Jacobian sweep)
#   configs  cfg3 cfg4 cfg5 cfg1 bench lines, each with a bounded CPU baseline (5 s 1 thread + 2.5 s all threads)
#   prof     per config in PROF_CONFIGS (default cfg2 cfg3; "sweep" = the Jacobian sweep): the bench line, a rocprofv3
#            kernel trace and one PMC pass per counter group (tools/roofline.py recomputes the roofline fields)
#   wst      the per-instance diagnostic build (tools/cl_wstamps.py: devlib/libalipmpc_wstamp.so)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
export TMPDIR=/tmp
export ALIPMPC_SCENE_CACHE=/tmp/alipmpc_scenes
PMCS=(FETCH_SIZE WRITE_SIZE "SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE")
for what in "$@"; do
  case $what in
  tests)
    echo "=== pytest -m gpu"
    timeout -k 10 900 python -u -m pytest $R/tests -x -v --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1; rc=$?
    tail -4 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $OUT/pytest_gpu.log | head -80; exit $rc; }
    echo "=== smoke"
    timeout -k 10 300 python -c "import sys; sys.path.insert(0,'$R'); import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
    cat $OUT/smoke.log ;;
  bench)
    echo "=== bench (default = cfg2)"
    timeout -k 10 300 python $R/bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
    cat $OUT/bench.json ;;
  configs)
    for c in ${CONFIGS:-cfg3 cfg4 cfg5 cfg1}; do
      echo "=== bench $c"
      timeout -k 10 400 python $R/bench.py --config $c --steps 5 --cpu-seconds 5 --sweep-batch 0 > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -20 $OUT/bench_$c.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/bench_$c.json'));print('$c', round(d['value']), d['ms_per_step'], d['config']['mean_iters'], d.get('feasible'), d['cpu_baseline']['value'])"
    done ;;
  prof)
    cd /tmp
    for c in ${PROF_CONFIGS:-cfg2 cfg3}; do
      D=$OUT/$c
      mkdir -p $D
      if [ $c = sweep ]; then
        python3 -c "import sys; sys.path.insert(0,'$R/mujoco-lip-mpc-simulation_amd'); import alipmpc; print(alipmpc.build_id())" > $D/build_id.txt
        echo "=== rocprofv3 kernel trace sweep"
        timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_kt -o kt -- python3 $R/tools/sweep_only.py > $D/prof_kt.log 2>&1 || { tail -20 $D/prof_kt.log; exit 1; }
        for pmc in "${PMCS[@]}"; do
          tag=$(echo $pmc | cut -d' ' -f1)
          echo "=== rocprofv3 --pmc $tag (sweep)"
          timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $D/pmc_$tag -o pmc -- python3 $R/tools/sweep_only.py > $D/pmc_$tag.log 2>&1 || { tail -20 $D/pmc_$tag.log; exit 1; }
        done
        continue
      fi
      flags="--config $c --no-cpu-baseline --closed-loop-steps 0 --sweep-batch 0"
      echo "=== bench $c"
      timeout -k 10 300 python3 $R/bench.py $flags --steps 10 > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
      echo "=== rocprofv3 kernel trace $c"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_kt -o kt -- python3 $R/bench.py $flags --steps 10 > $D/prof_kt.log 2>&1 || { tail -20 $D/prof_kt.log; exit 1; }
      for pmc in "${PMCS[@]}"; do
        tag=$(echo $pmc | cut -d' ' -f1)
        echo "=== rocprofv3 --pmc $tag ($c)"
        timeout -s KILL 150 rocprofv3 --pmc $pmc --output-format csv -d $D/pmc_$tag -o pmc -- python3 $R/bench.py $flags --steps 3 --warmup 1 > $D/pmc_$tag.log 2>&1 || { tail -20 $D/pmc_$tag.log; exit 1; }
      done
    done
    cd $R ;;
  wst)
    echo "=== per-instance records (diagnostic build)"
    timeout -k 10 300 python $R/tools/cl_wstamps.py run --out $OUT/wst > $OUT/wst.log 2>&1 || { tail -30 $OUT/wst.log; exit 1; }
    tail -30 $OUT/wst.log ;;
  esac
done
echo "=== done"
