# HBM traffic of the NTT passes from PMC counters: FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 passes (they cannot share one), over tools/prof_ntt.py (15-buffer ring, 346 MB,
# larger than the 256 MiB Infinity Cache).  Summary: tools/pmc_traffic.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_traffic_r02
mkdir -p $OUT
cd /tmp
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_ntt.py > $OUT/log_$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $OUT/log_$i.txt; exit 1; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_traffic.py $OUT > $OUT/ntt_pmc_traffic.json && cat $OUT/ntt_pmc_traffic.json
