# Carry-free integer butterflies (PHX_INT_NOCARRY): GPU parity tests, then integer-path (C4 chain)
# and FP64-path forward NTT timings of the new build against the old-arithmetic variant
# (tools/variants/old, -DPHX_INT_NOCARRY=0), interleaved, then the bootstrap example.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/int
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export PHX_PY=$GRAFT_REPO_ROOT/tools/variants/old/py; else unset PHX_PY; fi
    for mode in ntt60 ntt50; do
      MODE=$mode ITERS=600 timeout -k 10 120 python -u tools/prof_kernels.py > $OUT/t_${v}_${mode}_$rep.txt 2>&1
      rc=$?; echo "$v $(tail -1 $OUT/t_${v}_${mode}_$rep.txt)"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
unset PHX_PY
timeout -k 10 300 phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 5 > $OUT/boot.txt 2>&1
rc=$?; tail -6 $OUT/boot.txt; exit $rc
