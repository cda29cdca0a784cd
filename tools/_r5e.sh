mkdir -p gpurun_out/r5e
export ALIPMPC_TEST_ARTIFACTS=$PWD/gpurun_out/r5e/art
ALIPMPC_LIB=devlib/libalipmpc_dbg.so timeout -k 10 300 python -u tools/cl_fp32_study.py --out gpurun_out/r5e --tag dbg --no-oracle > gpurun_out/r5e/study_dbg.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/cl_fp32_study.py --out gpurun_out/r5e --tag floor > gpurun_out/r5e/study_floor.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/cl_same_inputs.py --out gpurun_out/r5e > gpurun_out/r5e/same_0.log 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r5e/pytest_gpu.log 2>&1
tail -3 gpurun_out/r5e/pytest_gpu.log; grep -E "FAILED|^E  " gpurun_out/r5e/pytest_gpu.log | cut -c1-300 | head -30; cat gpurun_out/r5e/study_floor.log gpurun_out/r5e/same_0.log
