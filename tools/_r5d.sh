mkdir -p gpurun_out/r5d
timeout -k 10 300 python -u tools/cl_fp32_study.py --out gpurun_out/r5d --tag scal > gpurun_out/r5d/study_scal.log 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r5d/pytest_gpu.log 2>&1
tail -3 gpurun_out/r5d/pytest_gpu.log; grep -E "FAILED|^E  " gpurun_out/r5d/pytest_gpu.log | head -30; cat gpurun_out/r5d/study_scal.log
