set -o pipefail
export ALIPMPC_TEST_ARTIFACTS=$PWD/gpurun_out/r5n/art
mkdir -p gpurun_out/r5n
bash tools/gpu_run.sh r5n tests bench || exit 1
cat gpurun_out/r5n/art/closed_loop_m3_*.json | tr -d '\n '; echo
