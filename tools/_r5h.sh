set -o pipefail
mkdir -p gpurun_out/r5h
timeout -k 10 300 python -u tools/stamps.py devlib/libalipmpc_stamps.so > gpurun_out/r5h/stamps.log 2>&1 || { tail -20 gpurun_out/r5h/stamps.log; exit 1; }
cat gpurun_out/r5h/stamps.log
CONFIGS=cfg1 bash tools/gpu_run.sh r5h configs || exit 1
PROF_CONFIGS=cfg2 bash tools/gpu_run.sh r5h prof || exit 1
python tools/roofline.py gpurun_out/r5h/cfg2 2>&1 | tail -30
