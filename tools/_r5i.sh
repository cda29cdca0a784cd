set -o pipefail
O=gpurun_out/r5i; mkdir -p $O
ab() {   # ab TAG CONFIG LIB...
  local tag=$1 c=$2; shift 2
  for rep in 1 2; do for lib in "$@"; do
    if [ "$lib" = default ]; then unset ALIPMPC_LIB; else export ALIPMPC_LIB=$PWD/devlib/libalipmpc_$lib.so; fi
    timeout -k 10 120 python -u bench.py --config $c --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --steps 20 > $O/$tag.tmp 2>>$O/$tag.err || return 1
    python -c "import json;d=json.load(open('$O/$tag.tmp'));print('$lib', '$c', round(d['value']), round(d['roofline']['kernel_ms'],4), d['config']['mean_iters'])" | tee -a $O/$tag.log
  done; done
}
ab cfg2 cfg2 default bis_cur bis_5e3a500 bis_c5cb82f bis_90b7298 bis_793a0c8 || exit 1
unset ALIPMPC_LIB
ab cfg5 cfg5 default m32 fl0 m32fl0 || exit 1
for v in m32 m32fl0; do
  ALIPMPC_LIB=$PWD/devlib/libalipmpc_$v.so timeout -k 10 300 python -u tools/cl_fp32_study.py --out $O --tag $v > $O/study_$v.log 2>&1 || { tail $O/study_$v.log; exit 1; }
  grep -E "^lane_fp32|^host" $O/study_$v.log
done
