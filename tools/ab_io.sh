# A/B of a library change against tools/variants/base on one box (alternating builds):
# NTT forward / inverse at the C4 chain (40 limbs, and 3 x 40), C2 batch, bootstrap latency, C5
#   gpurun -- 'TAG=... bash tools/ab_io.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-abio}; mkdir -p $OUT
B=tools/variants/${VAR:-base}/py; C=phantom-fhe-boot_amd/py
NTT_BITS=60 timeout -k 10 300 python3 tools/ntt_ab.py $B $C > $OUT/ntt60.txt 2>&1 || { tail $OUT/ntt60.txt; exit 1; }
cat $OUT/ntt60.txt
NTT_BITS=60 NTT_REP=3 timeout -k 10 300 python3 tools/ntt_ab.py $B $C > $OUT/ntt60x3.txt 2>&1 || { tail $OUT/ntt60x3.txt; exit 1; }
cat $OUT/ntt60x3.txt
NTT_BITS=50 timeout -k 10 300 python3 tools/ntt_ab.py $B $C > $OUT/ntt50.txt 2>&1 || { tail $OUT/ntt50.txt; exit 1; }
cat $OUT/ntt50.txt
[ -n "$NO_BOOT" ] && exit 0
for i in 1 2; do for v in base cur; do
  if [ $v = base ]; then LIB=$PWD/tools/variants/${VAR:-base}/lib; else LIB=$PWD/phantom-fhe-boot_amd/lib; fi
  LD_LIBRARY_PATH=$LIB timeout -k 10 200 phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 5 > $OUT/boot_${v}_${i}.txt 2>&1 || exit 1
  echo "$v $(grep '"stage": "bootstrap"' $OUT/boot_${v}_${i}.txt | cut -c1-110)" | tee -a $OUT/boot.txt
done; done
for i in 1 2; do for v in $B $C; do
  C5_TOTAL=${C5_TOTAL:-384} timeout -k 10 200 python3 tools/time_c5.py $v 2>&1 | grep -v amdgpu.ids | tee -a $OUT/c5.txt || exit 1
done; done
