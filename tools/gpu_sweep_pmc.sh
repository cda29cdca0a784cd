# GPU-box dev script: sweep vs group eval kernel timings (twice each) and one rocprofv3 PMC pass per counter group for each
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sw2
mkdir -p $O
cd /tmp
for k in sweep group sweep group; do
  ALIPMPC_EVAL_KERNEL=$k timeout -k 10 120 python $R/tools/sweep_ab.py $k >> $O/ab.log 2>&1 || exit 1
  echo "--- $k" >> $O/ab.log
done
for k in sweep group; do
  for pmc in "SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM" "SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
    tag=$(echo $pmc | cut -d' ' -f1)
    ALIPMPC_EVAL_KERNEL=$k timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $O/pmc_${k}_$tag -o pmc -- python3 $R/tools/sweep_only.py > $O/pmc_${k}_$tag.log 2>&1 || { tail $O/pmc_${k}_$tag.log; exit 1; }
  done
done
cat $O/ab.log
