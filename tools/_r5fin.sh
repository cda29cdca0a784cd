set -o pipefail
export ALIPMPC_TEST_ARTIFACTS=$PWD/gpurun_out/r5fin/art
mkdir -p gpurun_out/r5fin
bash tools/gpu_run.sh r5fin tests bench || exit 1
