# One GPU round: parity tests, bench, rocprofv3 kernel-trace summary.  Every GPU step has its
# own time limit and the chain stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; cat gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 --no-c4 --no-c5 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
rc=$?; tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log; find $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -name "*stats*"; exit $rc
