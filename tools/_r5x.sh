set -o pipefail
O=gpurun_out/r5x; mkdir -p $O
for rep in 1 2; do for lib in rf8_8 rf8_4 rf8_16 rf8_32; do
  ALIPMPC_LIB=$PWD/devlib/libalipmpc_$lib.so timeout -k 10 120 python -u bench.py --config cfg5 --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --steps 10 > $O/t.tmp 2>>$O/t.err || exit 1
  python -c "import json;d=json.load(open('$O/t.tmp'));r=d['roofline'];print('$lib', 'cfg5', round(d['value']), round(r['kernel_ms'],4))" | tee -a $O/t.log
done; for lib in rf7_8 rf7_4 rf7_16; do
  ALIPMPC_LIB=$PWD/devlib/libalipmpc_$lib.so timeout -k 10 120 python -u bench.py --config cfg4 --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --steps 10 > $O/t.tmp 2>>$O/t.err || exit 1
  python -c "import json;d=json.load(open('$O/t.tmp'));r=d['roofline'];print('$lib', 'cfg4', round(d['value']), round(r['kernel_ms'],4))" | tee -a $O/t.log
done; done
unset ALIPMPC_LIB
for rep in 1 2; do for g in 1 2 3 4; do
  ALIPMPC_CL_GROUPS=$g timeout -k 10 200 python -u bench.py --config cfg2 --no-cpu-baseline --sweep-batch 0 --steps 3 > $O/c.tmp 2>>$O/c.err || exit 1
  python -c "import json;d=json.load(open('$O/c.tmp'));c=d['closed_loop'];print('cl_groups', $g, c['ms'], round(c['solves_per_s']))" | tee -a $O/t.log
done; done
