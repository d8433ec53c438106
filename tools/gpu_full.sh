# Full round-end rehearsal: pytest -m gpu, smoke(), bench.py defaults
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-full}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -5 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 600 python3 -u bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.log || { tail -20 $OUT/bench.log; exit 1; }
tail -c 2500 $OUT/bench.json
