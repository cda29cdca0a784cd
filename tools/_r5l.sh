set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5l; mkdir -p $O; cd /tmp
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1; grep -i "icache\|SQC_" $O/counters.txt | head -40
for v in hl hl_noscal hl_s1; do
  ALIPMPC_LIB=$GRAFT_REPO_ROOT/devlib/libalipmpc_$v.so timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS SQ_WAIT_INST_ANY --output-format csv -d $O/pmc_$v -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg2 --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --steps 3 --warmup 1 > $O/pmc_$v.log 2>&1 || { tail -20 $O/pmc_$v.log; exit 1; }
  python3 - <<PY
import csv,glob,collections
f=glob.glob('$O/pmc_$v/*counter_collection.csv')[0]
rows=[r for r in csv.DictReader(open(f)) if 'solve_kernel' in r['Kernel_Name'] and r['Grid_Size']=='262144']
byd=collections.defaultdict(dict)
for r in rows: byd[int(r['Dispatch_Id'])][r['Counter_Name']]=float(r['Counter_Value'])
ds=sorted(byd)
for i,d in enumerate(ds): print('$v', 'phase', 1+i%2, byd[d])
PY
done
