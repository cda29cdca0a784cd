mkdir -p gpurun_out/r5a
timeout -k 10 300 python -u tools/cl_fp32_study.py --out gpurun_out/r5a --tag hd64 > gpurun_out/r5a/study.log 2>&1
timeout -k 10 120 python tools/sweep_ceiling.py 65536 > gpurun_out/r5a/ceiling.json 2>gpurun_out/r5a/ceiling.err
timeout -k 10 120 python tools/sweep_ceiling.py 1048576 > gpurun_out/r5a/ceiling_1m.json 2>>gpurun_out/r5a/ceiling.err
timeout -k 10 1000 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r5a/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --cpu-seconds 3 > gpurun_out/r5a/bench.json 2> gpurun_out/r5a/bench.err
tail -5 gpurun_out/r5a/pytest_gpu.log; grep -E "FAILED|Error" gpurun_out/r5a/pytest_gpu.log | head -20; cat gpurun_out/r5a/study.log gpurun_out/r5a/ceiling*.json gpurun_out/r5a/bench.json; tail -3 gpurun_out/r5a/ceiling.err gpurun_out/r5a/bench.err
