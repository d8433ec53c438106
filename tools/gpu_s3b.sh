# MFMA base conversion: parity, C3/C4 bench, C3 kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/s3b
timeout -k 10 300 python -u -m pytest tests/test_gpu_ckks.py tests/test_gpu_bootk.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s3b/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/s3b/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c5 > gpurun_out/s3b/bench.log 2>&1
rc=$?; tail -2 gpurun_out/s3b/bench.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && MODE=c3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s3b/c3 -o c3 -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py > $GRAFT_REPO_ROOT/gpurun_out/s3b/c3.log 2>&1
rc=$?; tail -3 $GRAFT_REPO_ROOT/gpurun_out/s3b/c3.log; exit $rc
