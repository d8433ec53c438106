set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bootk.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r02d.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu_r02d.log
exit $rc
