set -o pipefail
O=gpurun_out/r5s; mkdir -p $O
for rep in 1 2; do for lib in tw4 tw2; do for tr in 0 16 32 64; do
  ALIPMPC_LIB=$PWD/devlib/libalipmpc_$lib.so ALIPMPC_SPLIT_TR=$tr timeout -k 10 120 python -u bench.py --config cfg2 --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --steps 20 > $O/t.tmp 2>>$O/t.err || exit 1
  python -c "import json;d=json.load(open('$O/t.tmp'));r=d['roofline'];print('$lib', 'split_tr', $tr, round(d['value']), round(r['kernel_ms'],4), d['config']['mean_iters'], d['config']['status_counts'])" | tee -a $O/t.log
done; done; done
