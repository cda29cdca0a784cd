# Dev (GPU box): cfg2 bench with and without the cold-solve launch order, then the GPU suite
set -u
mkdir -p gpurun_out/so
ALIPMPC_SOLVE_ORDER=0 timeout -k 10 200 python bench.py --no-cpu-baseline --closed-loop-steps 0 --sweep-batch 0 > gpurun_out/so/bench_id.json 2>/dev/null || exit 1
ALIPMPC_SOLVE_ORDER=1 timeout -k 10 200 python bench.py --no-cpu-baseline --closed-loop-steps 0 --sweep-batch 0 > gpurun_out/so/bench_ord.json 2>/dev/null || exit 1
python -c "
import json
for f in ('bench_id', 'bench_ord'):
    d = json.load(open('gpurun_out/so/%s.json' % f)); print(f, round(d['value']), round(d['roofline']['kernel_ms'], 4), d['config']['status_counts'])
"
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/so/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/so/pytest.log; grep -B3 -A30 "FAILED\|Error" gpurun_out/so/pytest.log | head -40
exit $rc
