set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r02a.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_r02a.log
exit $rc
