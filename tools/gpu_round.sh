set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -20 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench.log 2>&1
rc=$?; cat gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
rc=$?; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof.log; find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*stats*" | head; exit $rc
