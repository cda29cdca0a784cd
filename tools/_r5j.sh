set -o pipefail
O=gpurun_out/r5j; mkdir -p $O
ab() {   # ab TAG CONFIG LIB...
  local tag=$1 c=$2; shift 2
  for rep in 1 2; do for lib in "$@"; do
    if [ "$lib" = default ]; then unset ALIPMPC_LIB; else export ALIPMPC_LIB=$PWD/devlib/libalipmpc_$lib.so; fi
    timeout -k 10 120 python -u bench.py --config $c --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --steps 20 > $O/$tag.tmp 2>>$O/$tag.err || return 1
    python -c "import json;d=json.load(open('$O/$tag.tmp'));r=d['roofline'];print('$lib', '$c', round(d['value']), round(r['kernel_ms'],4), d['config']['mean_iters'], (r.get('latency') or {}).get('cycles_per_iter'))" | tee -a $O/$tag.log
  done; done
}
ab cfg2 cfg2 ser hl hl_dense hl_noscal || exit 1
ab cfg1 cfg1 ser hl || exit 1
ab cfg5 cfg5 gd gm || exit 1
for v in gd gm; do
  ALIPMPC_LIB=$PWD/devlib/libalipmpc_$v.so timeout -k 10 300 python -u tools/cl_fp32_study.py --out $O --tag $v > $O/study_$v.log 2>&1 || { tail $O/study_$v.log; exit 1; }
  grep -E "^lane_fp32|^host" $O/study_$v.log
done
