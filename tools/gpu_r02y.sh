# parity of the CKKS / bootstrap kernels + bootstrap timing + C3 relinearize kernel split
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02y
timeout -k 10 600 python -u -m pytest tests/test_gpu_ckks.py tests/test_gpu_bootk.py tests/test_gpu_bootstrap.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02y/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r02y/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 5 > gpurun_out/r02y/boot.log 2>&1 || { tail -5 gpurun_out/r02y/boot.log; exit 1; }
grep ms_median gpurun_out/r02y/boot.log | cut -c1-130
cd /tmp
MODE=c3 timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r02y/c3 -o c3 -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py > $GRAFT_REPO_ROOT/gpurun_out/r02y/c3.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r02y/c3.log; exit 1; }
