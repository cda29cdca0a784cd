set -o pipefail
O=gpurun_out/r5ab; mkdir -p $O
for rep in 1 2 3; do for lib in at0 at1; do
  export ALIPMPC_LIB=$PWD/devlib/libalipmpc_$lib.so
  timeout -k 10 120 python -u bench.py --config cfg2 --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --steps 20 > $O/t.tmp 2>>$O/t.err || exit 1
  python -c "import json;d=json.load(open('$O/t.tmp'));r=d['roofline'];print('$lib', 'cfg2', round(d['value']), round(r['kernel_ms'],4), d['config']['mean_iters'], (r.get('latency') or {}).get('cycles_per_iter'))" | tee -a $O/t.log
done; done
