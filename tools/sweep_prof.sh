set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sw
mkdir -p $OUT
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/tools/sweep_only.py > $OUT/kt.log 2>&1 || { tail $OUT/kt.log; exit 1; }
for pmc in FETCH_SIZE WRITE_SIZE "SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM" "SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
  tag=$(echo $pmc | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc_$tag -o pmc -- python3 $R/tools/sweep_only.py > $OUT/pmc_$tag.log 2>&1 || { tail $OUT/pmc_$tag.log; exit 1; }
done
echo done
