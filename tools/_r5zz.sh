set -o pipefail
O=$PWD/gpurun_out/r5zz; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu -k "test_solve_variants_vs_oracle" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest.log | head -60; exit 1; }
