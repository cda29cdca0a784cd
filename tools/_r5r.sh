set -o pipefail
O=gpurun_out/r5r; mkdir -p $O
ab() {   # ab TAG CONFIG LIB...
  local tag=$1 c=$2; shift 2
  for rep in 1 2 3; do for lib in "$@"; do
    export ALIPMPC_LIB=$PWD/devlib/libalipmpc_$lib.so
    timeout -k 10 120 python -u bench.py --config $c --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --steps 20 > $O/$tag.tmp 2>>$O/$tag.err || return 1
    python -c "import json;d=json.load(open('$O/$tag.tmp'));r=d['roofline'];print('$lib', '$c', round(d['value']), round(r['kernel_ms'],4), d['config']['mean_iters'], (r.get('latency') or {}).get('cycles_per_iter'))" | tee -a $O/$tag.log
  done; done
}
ab cfg2 cfg2 w_old w_new || exit 1
ab cfg4 cfg4 l7_old l7_new || exit 1
ab cfg5 cfg5 l8_old l8_new || exit 1
