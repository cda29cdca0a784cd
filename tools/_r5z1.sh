set -o pipefail
export ALIPMPC_TEST_ARTIFACTS=$PWD/gpurun_out/r5z/art
mkdir -p gpurun_out/r5z
bash tools/gpu_run.sh r5z tests || exit 1
PROF_CONFIGS="cfg2 cfg3 sweep" bash tools/gpu_run.sh r5z prof || exit 1
for c in cfg2 cfg3; do python tools/roofline.py gpurun_out/r5z/$c --write profiles/solve_kernel_counters.json > gpurun_out/r5z/$c/roofline.json 2>&1 || exit 1; done
python tools/roofline.py gpurun_out/r5z/sweep --sweep 'sweep_kernel<5,true,32,2>' --write profiles/solve_kernel_counters.json > gpurun_out/r5z/sweep/roofline.json 2>&1 || exit 1
cp profiles/solve_kernel_counters.json gpurun_out/r5z/solve_kernel_counters_a.json
echo ok
