set -o pipefail
PROF_CONFIGS="cfg4 cfg5" bash tools/gpu_run.sh r5z prof || exit 1
for c in cfg4 cfg5; do python tools/roofline.py gpurun_out/r5z/$c --write profiles/solve_kernel_counters.json > gpurun_out/r5z/$c/roofline.json 2>&1 || exit 1; done
cp profiles/solve_kernel_counters.json gpurun_out/r5z/solve_kernel_counters_b.json
CONFIGS="cfg1 cfg3 cfg4 cfg5" bash tools/gpu_run.sh r5z configs bench || exit 1
echo ok
