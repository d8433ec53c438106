set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-abrow}
mkdir -p $OUT
timeout -k 10 120 python3 -u tools/host_c3.py > $OUT/host_c3.txt 2>&1; cat $OUT/host_c3.txt
P=phantom-fhe-boot_amd/py; V=tools/variants/${VAR:-row4}/py
NTT_BITS=60 REPS=3 timeout -k 10 300 python3 -u tools/ntt_ab.py $P $V > $OUT/ab_60.txt 2>&1 || exit 1; tail -1 $OUT/ab_60.txt
NTT_BITS=60 NTT_REP=3 REPS=2 timeout -k 10 300 python3 -u tools/ntt_ab.py $P $V > $OUT/ab_60x3.txt 2>&1 || exit 1; tail -1 $OUT/ab_60x3.txt
NTT_BITS=50 REPS=3 timeout -k 10 300 python3 -u tools/ntt_ab.py $P $V > $OUT/ab_50.txt 2>&1 || exit 1; tail -1 $OUT/ab_50.txt
for rep in 1 2; do for v in main ${VAR:-row4}; do
  if [ $v = main ]; then LIB=phantom-fhe-boot_amd/lib; else LIB=tools/variants/$v/lib; fi
  LD_LIBRARY_PATH=$LIB timeout -k 10 200 phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 3 > $OUT/boot_${v}_$rep.txt 2>&1 || { tail -3 $OUT/boot_${v}_$rep.txt; exit 1; }
  echo "$v $(grep '"stage": "bootstrap"' $OUT/boot_${v}_$rep.txt | cut -c1-100)"
done; done
