# GPU-box dev script: sweep-kernel GPU tests, then tools/sweep_ab.py timings (sweep kernel at B = 64K/256K/1M, eval_kernel at 256K)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sw3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -v --timeout 120 --timeout-method thread -m gpu -k "sweep_kernel or eval" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for B in 65536 262144 1048576; do
  timeout -k 10 120 python tools/sweep_ab.py sweep $B > $O/ab_sweep_$B.log 2>&1 || exit 1
  echo "=== sweep $B"; cat $O/ab_sweep_$B.log
done
timeout -k 10 120 python tools/sweep_ab.py group 262144 > $O/ab_group_262144.log 2>&1; echo "=== group 262144"; cat $O/ab_group_262144.log
