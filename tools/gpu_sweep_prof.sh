# GPU-box dev script: the Jacobian sweep alone (bench.jacobian_sweep, B = 65536): kernel trace + one rocprofv3 PMC pass
# per counter group (HBM bytes, instruction mix, issue / wait), into gpurun_out/$1
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-swp}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o kt -- python3 $R/tools/sweep_only.py > $O/prof_kt.log 2>&1 || { tail $O/prof_kt.log; exit 1; }
for pmc in FETCH_SIZE WRITE_SIZE "SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM" "SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
  tag=$(echo $pmc | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $O/pmc_$tag -o pmc -- python3 $R/tools/sweep_only.py > $O/pmc_$tag.log 2>&1 || { tail $O/pmc_$tag.log; exit 1; }
done
tail -2 $O/prof_kt.log
