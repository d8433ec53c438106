# A/B of the bootstrap latency between the in-tree build and tools/variants/$VAR (default base; alternating,
# one process per run): bootstrapping_example boot 16 5 with each library, 3 rounds.
#   gpurun -- 'bash tools/ab_boot.sh'   -> gpurun_out/abboot/boot.txt
set -o pipefail
OUT=gpurun_out/abboot
rm -rf $OUT; mkdir -p $OUT
for i in 1 2 3; do for v in base cur; do
  if [ $v = base ]; then LIB=$PWD/tools/variants/${VAR:-base}/lib; else LIB=$PWD/phantom-fhe-boot_amd/lib; fi
  LD_LIBRARY_PATH=$LIB timeout -k 10 200 phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 5 > $OUT/boot_${v}_${i}.txt 2>&1 || exit 1
  echo "$v $(grep '"stage": "bootstrap"' $OUT/boot_${v}_${i}.txt | cut -c1-110)" >> $OUT/boot.txt
done; done
cat $OUT/boot.txt
