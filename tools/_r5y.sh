set -o pipefail
O=gpurun_out/r5y; mkdir -p $O
for rep in 1 2 3; do for lib in default k4; do
  if [ $lib = default ]; then unset ALIPMPC_LIB; else export ALIPMPC_LIB=$PWD/devlib/libalipmpc_$lib.so; fi
  timeout -k 10 120 python -u bench.py --config cfg1 --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --steps 200 > $O/t.tmp 2>>$O/t.err || exit 1
  python -c "import json;d=json.load(open('$O/t.tmp'));r=d['roofline'];print('$lib', 'cfg1', round(d['value']), round(d['ms_per_step'],4), round(r['kernel_ms'],4), d['roofline'].get('kernel'))" | tee -a $O/t.log
done; done
export ALIPMPC_LIB=$PWD/devlib/libalipmpc_k4.so
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest_k4.log 2>&1; rc=$?; tail -3 $O/pytest_k4.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_k4.log | head -60; exit 1; }
