set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_r02q
mkdir -p $OUT
cd /tmp
for f in 1 0; do
  PHX_FUSED_BCONV=$f MODE=c3 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/f$f/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py > $OUT/log_f${f}_trace.txt 2>&1 || { echo "trace $f failed"; tail -5 $OUT/log_f${f}_trace.txt; exit 1; }
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    PHX_FUSED_BCONV=$f MODE=c3 timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/f$f/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py > $OUT/log_f${f}_$i.txt 2>&1 || { echo "pass $f $i failed"; tail -5 $OUT/log_f${f}_$i.txt; exit 1; }
  done
done
cd $GRAFT_REPO_ROOT
for f in 1 0; do echo "== fused=$f"; python3 tools/pmc_summary.py $OUT/f$f; done > $OUT/summary.txt
python3 - <<'PY'
import csv
for f in ["1","0"]:
    print("== fused", f)
    for r in csv.DictReader(open(f"gpurun_out/pmc_r02q/f{f}/trace/run_kernel_stats.csv")):
        n=r["Name"]; n=n[n.find("phx::"):][:70] if "phx::" in n else n[:70]
        print(f'{n:72s} calls={r["Calls"]:>5} avg={float(r["AverageNs"])/1000:8.2f}us tot={float(r["TotalDurationNs"])/1e6:7.3f}ms')
PY
