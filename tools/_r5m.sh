set -o pipefail
O=gpurun_out/r5m; mkdir -p $O; cd /tmp
for rep in 1 2; do for v in hl2 p2l81 p2l81ns hl_noscal; do
  ALIPMPC_LIB=$GRAFT_REPO_ROOT/devlib/libalipmpc_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_${v}_$rep -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg2 --no-cpu-baseline --sweep-batch 0 --closed-loop-steps 0 --steps 10 > $GRAFT_REPO_ROOT/$O/kt_$v.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/kt_$v.log; exit 1; }
  python3 - <<PY
import csv,glob
f=glob.glob('$GRAFT_REPO_ROOT/$O/kt_${v}_$rep/*kernel_trace.csv')[0]
rows=[r for r in csv.DictReader(open(f)) if 'solve_kernel' in r['Kernel_Name'] and r['Grid_Size_X']=='262144']
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000 for r in rows]
p1=d[2::2]; p2=d[3::2]
print('$v', 'phase1', round(sum(p1)/len(p1),1), 'phase2', round(sum(p2)/len(p2),1), 'p2 min/max', min(p2), max(p2), rows[3]['LDS_Block_Size'])
PY
done; done
