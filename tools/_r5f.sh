mkdir -p gpurun_out/r5f
export ALIPMPC_TEST_ARTIFACTS=$PWD/gpurun_out/r5f/art
timeout -k 10 300 python -u tools/cl_m3.py --test-episodes --out gpurun_out/r5f/m3 > gpurun_out/r5f/m3.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu -k "closed_loop or fp32_all or goal" > gpurun_out/r5f/pytest_gpu.log 2>&1
tail -3 gpurun_out/r5f/pytest_gpu.log; grep -E "FAILED|^E  " gpurun_out/r5f/pytest_gpu.log | cut -c1-300 | head -30; tail -5 gpurun_out/r5f/m3.log | cut -c1-1500
for f in gpurun_out/r5f/art/closed_loop_same_inputs_*.json; do echo $f; cat $f | tr -d '\n'; echo; done
