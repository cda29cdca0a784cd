# Dev (GPU box): the sweep kernel per launch shape (time + output hash), then the eval / sweep GPU tests.
set -e
mkdir -p gpurun_out/sw
for B in 65536 262144; do for sh in ${SHAPES:-641 322}; do
 ALIPMPC_SWEEP_SHAPE=$sh timeout -k 10 120 python tools/sweep_shapes.py $B >> gpurun_out/sw/shapes.txt 2>/dev/null
done; done
cat gpurun_out/sw/shapes.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "sweep or eval" > gpurun_out/sw/pytest.log 2>&1; tail -3 gpurun_out/sw/pytest.log
