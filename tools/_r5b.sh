mkdir -p gpurun_out/r5b
ALIPMPC_LIB=devlib/libalipmpc_dbg.so timeout -k 10 300 python -u tools/cl_fp32_study.py --out gpurun_out/r5b --tag dbg2 --no-oracle > gpurun_out/r5b/study_dbg2.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/cl_fp32_study.py --out gpurun_out/r5b --tag rp64 > gpurun_out/r5b/study_rp64.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --sweep-batch 0 --steps 5 > gpurun_out/r5b/bench_cl_t8.json 2>> gpurun_out/r5b/bench.err || exit 1
ALIPMPC_LIB=devlib/libalipmpc_team4.so timeout -k 10 300 python bench.py --no-cpu-baseline --sweep-batch 0 --steps 5 > gpurun_out/r5b/bench_cl_t4.json 2>> gpurun_out/r5b/bench.err || exit 1
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --steps 5 > gpurun_out/r5b/bench_cfg5.json 2>> gpurun_out/r5b/bench.err || exit 1
timeout -k 10 800 python -u -m pytest tests -v --timeout 120 --timeout-method thread -m gpu -k "variants_vs_oracle or all_horizons or split or team or groups or closed_loop or lane or fp32 or goal" > gpurun_out/r5b/pytest_gpu.log 2>&1
tail -3 gpurun_out/r5b/pytest_gpu.log; grep -E "FAILED" gpurun_out/r5b/pytest_gpu.log | head; cat gpurun_out/r5b/study_rp64.log
for f in gpurun_out/r5b/bench_cl_*.json gpurun_out/r5b/bench_cfg5.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d.get('closed_loop',{}).get('ms'), d.get('closed_loop',{}).get('solves_per_s'), d['ms_per_step'])"; done
