# Micro-benchmarks + rocprofv3 kernel stats (csv) + PMC passes for the NTT.  Each GPU step has
# its own time limit; the chain stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r01}
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench_isa > gpurun_out/ubench_isa.txt 2>&1 || exit 1
timeout -k 10 120 ./tools/ubench_mem > gpurun_out/ubench_mem.txt 2>&1 || exit 1
cat gpurun_out/ubench_isa.txt gpurun_out/ubench_mem.txt
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/stats_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/stats_$TAG.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/stats_$TAG.log; exit 1; }
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_ntt.py > $OUT/log_$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $OUT/log_$i.txt; exit 1; }
done
find $GRAFT_REPO_ROOT/gpurun_out/stats_$TAG $OUT -name "*.csv" | head -20
