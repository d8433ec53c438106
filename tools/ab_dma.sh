# NTT column-pass forms (PHX_NTT_COL_DMA = 0 / 1 / 2) on one box: NTT + bootstrap-kernel parity tests,
# then alternating A/B timings (tools/ntt_ab.py) at the C4 chain (40 limbs, x3) and the C2 batch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-dma}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ntt.py tests/test_gpu_bootk.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
P=phantom-fhe-boot_amd/py
V="$P@PHX_NTT_COL_DMA=0 $P@PHX_NTT_COL_DMA=1 $P@PHX_NTT_COL_DMA=2"
NTT_BITS=60 REPS=3 timeout -k 10 300 python3 -u tools/ntt_ab.py $V > $OUT/ab_60.txt 2>&1 || exit 1; tail -1 $OUT/ab_60.txt
NTT_BITS=60 NTT_REP=3 REPS=2 timeout -k 10 300 python3 -u tools/ntt_ab.py $V > $OUT/ab_60x3.txt 2>&1 || exit 1; tail -1 $OUT/ab_60x3.txt
NTT_BITS=50 REPS=3 timeout -k 10 300 python3 -u tools/ntt_ab.py $V > $OUT/ab_50.txt 2>&1 || exit 1; tail -1 $OUT/ab_50.txt
