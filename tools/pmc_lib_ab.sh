# PMC passes (SQ set; FETCH_SIZE; WRITE_SIZE) of the forward + inverse NTT (tools/prof_ntt.py,
# BITS / REP as there) for tools/variants/$VARS and the in-tree build, summarised per kernel
#   gpurun -- 'TAG=... VARS="base" BITS=c4 REP=3 bash tools/pmc_lib_ab.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmclib}; mkdir -p "$OUT"
SETS=${PMC_SETS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES;FETCH_SIZE;WRITE_SIZE"}
IFS=';' read -ra sets <<< "$SETS"
for v in ${VARS:-} cur; do
  if [ $v = cur ]; then PYD=$GRAFT_REPO_ROOT/phantom-fhe-boot_amd/py; else PYD=$GRAFT_REPO_ROOT/tools/variants/$v/py; fi
  i=0
  for set in "${sets[@]}"; do
    i=$((i+1))
    (cd /tmp && ITERS=20 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv \
       -d "$OUT/$v/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/tools/prof_ntt.py" "$PYD" > "$OUT/$v.p$i.log" 2>&1) \
       || { echo "pmc $v/$i failed"; tail -5 "$OUT/$v.p$i.log"; exit 1; }
  done
  python3 tools/pmc_summary.py "$OUT/$v" > "$OUT/summary_$v.txt"
  echo "== $v"; cat "$OUT/summary_$v.txt"
done
