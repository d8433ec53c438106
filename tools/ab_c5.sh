# A/B of C5 throughput between library builds (alternating, 3 rounds).  Arguments: the py/ dirs to
# compare (default: tools/variants/base and the in-tree build).
set -o pipefail
OUT=gpurun_out/abc5; rm -rf $OUT; mkdir -p $OUT
V=${*:-tools/variants/base/py phantom-fhe-boot_amd/py}
for i in 1 2 3; do for v in $V; do
  timeout -k 10 200 python3 tools/time_c5.py $v >> $OUT/c5.txt 2>&1 || exit 1
done; done
grep -v amdgpu.ids $OUT/c5.txt
