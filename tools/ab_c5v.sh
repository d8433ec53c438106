# C5 A/B between the in-tree build and tools/variants/$VARS at $C5_TOTAL (alternating, $REPS rounds)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-abc5v}; mkdir -p $OUT
for i in $(seq 1 ${REPS:-3}); do for v in ${VARS:-base} cur; do
  if [ $v = cur ]; then P=phantom-fhe-boot_amd/py; else P=tools/variants/$v/py; fi
  C5_TOTAL=${C5_TOTAL:-768} timeout -k 10 300 python3 tools/time_c5.py $P 2>&1 | grep -v amdgpu.ids | tee -a $OUT/c5.txt || exit 1
done; done
