# Quick GPU iteration: NTT parity tests, a short bench, rocprofv3 kernel stats (csv).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-quick}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ntt.py ${EXTRA_TESTS} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/bench_$TAG.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/stats_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/stats_$TAG.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/stats_$TAG.log; exit $rc; }
python3 $GRAFT_REPO_ROOT/tools/stats_short.py $GRAFT_REPO_ROOT/gpurun_out/stats_$TAG/run_kernel_stats.csv
