# Rescale / moddown finish: the in-tree build (row-pass finish at 3 waves per SIMD) against a variant
# (tools/variants/$VAR, e.g. PHX_EPI_WAVES=2): parity tests, C3 per-op times and the C4 bootstrap,
# alternating builds on one box; then a kernel trace of C3 on the in-tree build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abepi}
VAR=${VAR:-epi2}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_ckks.py tests/test_gpu_ntt.py tests/test_gpu_bootk.py tests/test_gpu_bootstrap.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in main $VAR; do
    if [ $v = main ]; then P=phantom-fhe-boot_amd/py; LIB=phantom-fhe-boot_amd/lib; else P=tools/variants/$v/py; LIB=tools/variants/$v/lib; fi
    timeout -k 10 200 python3 -u tools/time_c3.py $P >> $OUT/c3_ab.txt 2>&1 || { tail -5 $OUT/c3_ab.txt; exit 1; }
    LD_LIBRARY_PATH=$LIB timeout -k 10 200 phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 3 > $OUT/boot_${v}_$rep.txt 2>&1 || { tail -5 $OUT/boot_${v}_$rep.txt; exit 1; }
    echo "$v $(grep '"stage": "bootstrap"' $OUT/boot_${v}_$rep.txt | cut -c1-120)" >> $OUT/c3_ab.txt
  done
done
cat $OUT/c3_ab.txt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/c3trace" -o run \
   -- python3 "$GRAFT_REPO_ROOT/tools/prof_c3.py" > "$GRAFT_REPO_ROOT/$OUT/c3trace.log" 2>&1) || { tail -5 $OUT/c3trace.log; exit 1; }
python3 tools/c3_steps.py "$(find $OUT/c3trace -name '*kernel_trace.csv' | head -1)"
