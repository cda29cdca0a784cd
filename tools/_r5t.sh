set -o pipefail
O=gpurun_out/r5t; mkdir -p $O
for rep in 1 2; do for it in 12 14 16 18 20 22; do
  ALIPMPC_SPLIT_IT=$it timeout -k 10 120 python -u bench.py --config cfg2 --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --steps 20 > $O/t.tmp 2>>$O/t.err || exit 1
  python -c "import json;d=json.load(open('$O/t.tmp'));r=d['roofline'];print('split_it', $it, round(d['value']), round(r['kernel_ms'],4))" | tee -a $O/t.log
done; done
for rep in 1 2; do for it in 12 16 20; do
  ALIPMPC_CL_SPLIT_IT=$it timeout -k 10 200 python -u bench.py --config cfg2 --no-cpu-baseline --sweep-batch 0 --steps 3 > $O/c.tmp 2>>$O/c.err || exit 1
  python -c "import json;d=json.load(open('$O/c.tmp'));c=d['closed_loop'];print('cl_split_it', $it, c['ms'], round(c['solves_per_s']))" | tee -a $O/t.log
done; done
