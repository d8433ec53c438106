# PMC passes over the C3 relinearize driver (separate rocprofv3 runs, counters only with kernel trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_c3${TAG}
mkdir -p $OUT
cd /tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  MODE=c3 ITERS=5 timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py > $OUT/log_$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $OUT/log_$i.txt; exit 1; }
done
