# PMC passes over the NTT profiling driver (separate rocprofv3 runs, counters only with kernel trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $OUT
cd /tmp
run() { timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/p$1 -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_ntt.py > $OUT/log_$1.txt 2>&1; }
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_ntt.py > $OUT/log_$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $OUT/log_$i.txt; exit 1; }
done
ls -R $OUT | head -40
