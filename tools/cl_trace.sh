#!/bin/bash
# GPU box: rocprofv3 kernel trace of the bench's closed loop (tools/cl_params.py SETTING, default 16,40,2) into
# gpurun_out/TAG; summarise with `python tools/cl_trace_summary.py gpurun_out/TAG` (profiles/r4/closed_loop).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=$R/gpurun_out/${1:-clkt}
mkdir -p $D
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D -o kt -- python3 $R/tools/cl_params.py ${2:-16,40,2} > $D/log.txt 2>&1 || { tail -20 $D/log.txt; exit 1; }
grep "ms " $D/log.txt
