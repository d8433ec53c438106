# PMC passes (one rocprofv3 run per counter set, kernel trace only besides the counters) over
# tools/prof_kernels.py in three modes, plus a kernel-trace stats run of each mode.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_r02j
mkdir -p $OUT
cd /tmp
for mode in ntt50 ntt60 c3; do
  MODE=$mode timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$mode/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py > $OUT/log_${mode}_trace.txt 2>&1 || { echo "trace $mode failed"; tail -5 $OUT/log_${mode}_trace.txt; exit 1; }
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM" \
             "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr"; do
    i=$((i+1))
    MODE=$mode timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/$mode/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py > $OUT/log_${mode}_$i.txt 2>&1 || { echo "pass $mode $i failed"; tail -5 $OUT/log_${mode}_$i.txt; exit 1; }
  done
done
cd $GRAFT_REPO_ROOT
for mode in ntt50 ntt60 c3; do echo "== $mode"; python3 tools/pmc_summary.py $OUT/$mode; done > $OUT/summary.txt
cat $OUT/summary.txt | head -150
