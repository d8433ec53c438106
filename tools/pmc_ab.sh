# PMC passes of the forward + inverse NTT under two settings of a run-time knob (tools/prof_ntt.py):
#   KNOB=PHX_NTT_COL_DMA BITS=c4 REP=1 bash tools/pmc_ab.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-pmcab}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
SETS=${PMC_SETS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES;FETCH_SIZE;WRITE_SIZE"}
IFS=';' read -ra sets <<< "$SETS"
for v in 0 1; do
  i=0
  for set in "${sets[@]}"; do
    i=$((i+1))
    (cd /tmp && env $KNOB=$v ITERS=20 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv \
       -d "$OUT/k$v/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/tools/prof_ntt.py" > "$OUT/k$v.p$i.log" 2>&1) \
       || { echo "pmc $v/$i failed"; tail -5 "$OUT/k$v.p$i.log"; exit 1; }
  done
  python3 tools/pmc_summary.py "$OUT/k$v" > "$OUT/summary_$KNOB=$v.txt"
  echo "== $KNOB=$v"; cat "$OUT/summary_$KNOB=$v.txt"
done
