set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r06m; mkdir -p $OUT
for i in 1 2; do
  C5_TOTAL=768 C5_LANES=3 timeout -k 10 300 python3 tools/time_c5.py phantom-fhe-boot_amd/py 2>&1 | grep -v amdgpu.ids | tee -a $OUT/c5.txt || exit 1
  C5_TOTAL=768 C5_LANES=3 C5_GROUP=16 timeout -k 10 300 python3 tools/time_c5.py tools/variants/g16/py 2>&1 | grep -v amdgpu.ids | tee -a $OUT/c5.txt || exit 1
  C5_TOTAL=768 C5_LANES=2 C5_GROUP=16 timeout -k 10 300 python3 tools/time_c5.py tools/variants/g16/py 2>&1 | grep -v amdgpu.ids | tee -a $OUT/c5.txt || exit 1
done
