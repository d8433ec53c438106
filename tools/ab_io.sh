# A/B of library builds on one box (alternating): the in-tree build against tools/variants/$VARS
# (default base).  NTT forward / inverse at the C4 chain (40 limbs, and 3 x 40) and the C2 batch,
# C3 chain (NO_C3=1 skips), bootstrap latency (NO_BOOT=1 skips), C5 at $C5_TOTAL bootstraps (NO_C5=1 skips).
#   gpurun -- 'TAG=... VARS="base v2" bash tools/ab_io.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-abio}; mkdir -p $OUT
VARS=${VARS:-base}
PYS=""; for v in $VARS; do PYS="$PYS tools/variants/$v/py"; done; PYS="$PYS phantom-fhe-boot_amd/py"
IFS=';' read -ra CFGS <<< "${NTT_CFGS:-60 1;60 3;50 1}"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  NTT_BITS=$1 NTT_REP=$2 timeout -k 10 400 python3 tools/ntt_ab.py $PYS > $OUT/ntt$1x$2.txt 2>&1 || { tail $OUT/ntt$1x$2.txt; exit 1; }
  tail -1 $OUT/ntt$1x$2.txt
done
[ -n "$NO_C3" ] || for i in $(seq 1 ${C3_REPS:-2}); do for v in $PYS; do
  timeout -k 10 200 python3 tools/time_c3.py $v 2>&1 | grep -v amdgpu.ids | tail -1 | tee -a $OUT/c3.txt || exit 1
done; done
[ -n "$NO_BOOT" ] || for i in 1 2; do for v in $VARS cur; do
  if [ $v = cur ]; then LIB=$PWD/phantom-fhe-boot_amd/lib; else LIB=$PWD/tools/variants/$v/lib; fi
  LD_LIBRARY_PATH=$LIB timeout -k 10 200 phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 5 > $OUT/boot_${v}_${i}.txt 2>&1 || exit 1
  echo "$v $(grep '"stage": "bootstrap"' $OUT/boot_${v}_${i}.txt | cut -c1-110)" | tee -a $OUT/boot.txt
done; done
[ -n "$NO_C5" ] || for i in 1 2; do for v in $PYS; do
  C5_TOTAL=${C5_TOTAL:-384} timeout -k 10 200 python3 tools/time_c5.py $v 2>&1 | grep -v amdgpu.ids | tee -a $OUT/c5.txt || exit 1
done; done
