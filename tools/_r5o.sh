set -o pipefail
O=gpurun_out/r5o; mkdir -p $O
for rep in 1 2; do for tr in 0 24 48 96 160; do
  ALIPMPC_SPLIT_TR=$tr timeout -k 10 120 python -u bench.py --config cfg2 --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --steps 20 > $O/tr.tmp 2>>$O/tr.err || exit 1
  python -c "import json;d=json.load(open('$O/tr.tmp'));r=d['roofline'];print('split_tr', $tr, round(d['value']), round(r['kernel_ms'],4), d['config']['launch'][:40])" | tee -a $O/tr.log
done; done
