mkdir -p gpurun_out/r5g
export ALIPMPC_TEST_ARTIFACTS=$PWD/gpurun_out/r5g/art
timeout -k 10 1000 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r5g/pytest_gpu.log 2>&1
tail -3 gpurun_out/r5g/pytest_gpu.log; grep -E "FAILED|^E  " gpurun_out/r5g/pytest_gpu.log | cut -c1-300 | head -30
cat gpurun_out/r5g/art/closed_loop_m3_*.json | tr -d '\n '; echo
