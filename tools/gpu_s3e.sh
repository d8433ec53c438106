# MFMA base conversion: parity (CKKS + bootstrap kernels) and C3 kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/s3e
timeout -k 10 300 python -u -m pytest tests/test_gpu_ckks.py tests/test_gpu_bootk.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3e/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/s3e/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
MODE=c3 timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/s3e/main -o c3 -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py > $GRAFT_REPO_ROOT/gpurun_out/s3e/main.log 2>&1
