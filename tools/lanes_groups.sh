# C5 on one GPU through the bootstrap example: (lanes, lockstep group) pairs, 256 bootstraps each, 2 rounds
set -o pipefail
OUT=gpurun_out/lg; mkdir -p $OUT
for rep in 1 2; do for lg in "4 4" "2 8" "3 8" "2 6" "3 4" "4 2"; do set -- $lg
  timeout -k 10 200 phantom-fhe-boot_amd/bin/bootstrapping_example batch 16 256 $1 $2 > $OUT/b_$1_$2_$rep.txt 2>&1 || exit 1
  grep '"stage": "batch"' $OUT/b_$1_$2_$rep.txt
done; done
