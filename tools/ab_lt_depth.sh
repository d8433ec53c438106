# A/B of the inner-product kernels' plaintext prefetch depth (PHX_LT_DEPTH 2 in-tree, 3, 4 in
# tools/variants/d3, d4): kernel traces of one bootstrap and one lockstep group of 4 per build,
# twice, alternating, on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-ltdepth}
mkdir -p $OUT
for rep in 1 2; do for v in main d3 d4; do
  if [ $v = main ]; then LIB=$PWD/phantom-fhe-boot_amd/lib; else LIB=$PWD/tools/variants/$v/lib; fi
  (cd /tmp && LD_LIBRARY_PATH=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/${v}_$rep" -o run \
     -- "$GRAFT_REPO_ROOT/phantom-fhe-boot_amd/bin/bootstrapping_example" prof 16 4 > "$OUT/${v}_$rep.log" 2>&1) || exit 1
  python3 tools/prof_windows.py "$(find "$OUT/${v}_$rep" -name '*kernel_trace.csv' | head -1)" "$OUT/${v}_${rep}" > /dev/null || exit 1
  n=$(ls $OUT/${v}_${rep}_w*.csv | wc -l)
  s=$OUT/${v}_${rep}_w$((n-2)).csv; g=$OUT/${v}_${rep}_w$((n-1)).csv
  echo "$v rep $rep single: $(python3 tools/kernel_families.py $s | grep lt_bsgs | tr -s ' ') | group: $(python3 tools/kernel_families.py $g | grep lt_bsgs | tr -s ' ')"
done; done
