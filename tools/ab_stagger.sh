# NTT stagger experiment: C4-chain forward / inverse A/B of the in-tree build against
# tools/variants/{c24,c48,c96,r48} (PHX_NTT_STAGGER / PHX_NTT_STAGGER_ROW), 40 and 120 limbs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-stagger}
mkdir -p $OUT
P=phantom-fhe-boot_amd/py; V=tools/variants
NTT_BITS=60 REPS=3 timeout -k 10 400 python3 -u tools/ntt_ab.py $P $V/c24/py $V/c48/py $V/c96/py $V/r48/py > $OUT/ab_60.txt 2>&1 || exit 1; tail -6 $OUT/ab_60.txt
NTT_BITS=60 NTT_REP=3 REPS=2 timeout -k 10 400 python3 -u tools/ntt_ab.py $P $V/c24/py $V/c48/py $V/c96/py $V/r48/py > $OUT/ab_60x3.txt 2>&1 || exit 1; tail -6 $OUT/ab_60x3.txt
