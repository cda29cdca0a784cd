set -o pipefail
PROF_CONFIGS="${PC:-cfg2 cfg3 sweep}" bash tools/gpu_run.sh r5p prof || exit 1
for c in ${PC:-cfg2 cfg3 sweep}; do
  if [ $c = sweep ]; then
    python tools/roofline.py gpurun_out/r5p/sweep --sweep 'sweep_kernel<5,true,32,2>' --write profiles/solve_kernel_counters.json > gpurun_out/r5p/sweep/roofline.json 2>&1 || exit 1
  else
    python tools/roofline.py gpurun_out/r5p/$c --write profiles/solve_kernel_counters.json > gpurun_out/r5p/$c/roofline.json 2>&1 || exit 1
  fi
done
cp profiles/solve_kernel_counters.json gpurun_out/r5p/solve_kernel_counters_${TAGX:-a}.json
if [ -n "${CF:-}" ]; then CONFIGS="$CF" bash tools/gpu_run.sh r5p configs bench || exit 1; fi
echo ok
