set -o pipefail
O=$PWD/gpurun_out/r5q; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu -k "test_solve_variants_vs_oracle" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest.log | head -60; exit 1; }
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ceiling_kt -o kt -- python3 $GRAFT_REPO_ROOT/tools/sweep_ceiling.py 65536 20 > $O/ceiling.json 2> $O/ceiling.err || { tail $O/ceiling.err; exit 1; }
cat $O/ceiling.json; cat $O/ceiling_kt/kt_kernel_stats.csv | cut -c1-200
