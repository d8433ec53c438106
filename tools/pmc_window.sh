# PMC passes ($PMC_SETS, ';'-separated; default FETCH_SIZE; WRITE_SIZE; TCC_HIT_sum + TCC_MISS_sum) over bootstrapping_example prof 16 8
# (one warm bootstrap, then one lockstep group of 8) for the in-tree build and tools/variants/$VARS,
# summarised per kernel instantiation over the group window by tools/window_pmc.py.
#   gpurun -- 'TAG=... VARS="base" bash tools/pmc_window.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmcwin}; mkdir -p $OUT
for v in ${VARS:-} cur; do
  if [ $v = cur ]; then LIB=$GRAFT_REPO_ROOT/phantom-fhe-boot_amd/lib; else LIB=$GRAFT_REPO_ROOT/tools/variants/$v/lib; fi
  i=0
  IFS=';' read -ra SETS <<< "${PMC_SETS:-FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum}"
  for set in "${SETS[@]}"; do
    i=$((i+1))
    (cd /tmp && LD_LIBRARY_PATH=$LIB timeout -s KILL ${T_PMC:-240} rocprofv3 --kernel-trace --pmc $set --output-format csv \
       -d "$OUT/${v}_p$i" -o run -- "$GRAFT_REPO_ROOT/phantom-fhe-boot_amd/bin/bootstrapping_example" prof 16 8 \
       > "$OUT/${v}_p$i.log" 2>&1) || { echo "pass $v $i failed"; tail -5 "$OUT/${v}_p$i.log"; exit 1; }
  done
  python3 tools/window_pmc.py $(for k in $(seq 1 $i); do echo "$OUT/${v}_p$k"; done) > "$OUT/${v}_window.json" || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/${v}_window.json'))['kernels']
for k, e in list(d.items())[:12]: print('$v', k[:60], e.get('calls'), e.get('ms_per_bootstrap'), e.get('read_GB'), e.get('write_GB'), e.get('tcc_hit_rate'))"
done
