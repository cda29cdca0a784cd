mkdir -p gpurun_out/r5c
ALIPMPC_LIB=devlib/libalipmpc_dbg.so timeout -k 10 300 python -u tools/cl_fp32_study.py --out gpurun_out/r5c --tag dbg3 --no-oracle > gpurun_out/r5c/study_dbg3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/cl_fp32_study.py --out gpurun_out/r5c --tag m64 > gpurun_out/r5c/study_m64.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --steps 5 > gpurun_out/r5c/bench_cfg5.json 2>> gpurun_out/r5c/bench.err || exit 1
timeout -k 10 800 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu -k "closed_loop or lane or fp32 or goal" > gpurun_out/r5c/pytest_gpu.log 2>&1
tail -3 gpurun_out/r5c/pytest_gpu.log; grep -E "FAILED|^E  " gpurun_out/r5c/pytest_gpu.log | head -20; cat gpurun_out/r5c/study_m64.log
python -c "import json; d=json.load(open('gpurun_out/r5c/bench_cfg5.json')); print('cfg5', d['value'], d['ms_per_step'])"
