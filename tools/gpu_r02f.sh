set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ntt.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r02f.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu_r02f.log
exit $rc
