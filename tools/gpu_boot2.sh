# Bootstrap: parity subset, the bootstrap example (RUNS), and a kernel trace (rocpd db) of 2 runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-boot2}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_bconv.py tests/test_gpu_bootk.py tests/test_gpu_ckks.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 ${RUNS:-3} > gpurun_out/$TAG/boot.txt 2>&1
rc=$?; tail -4 gpurun_out/$TAG/boot.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run -- $GRAFT_REPO_ROOT/phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 2 > $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof.log 2>&1
