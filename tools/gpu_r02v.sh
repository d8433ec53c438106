# batched baby steps (keyswitch_rotate_batch): parity at C4 size, the bootstrap tests, timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02v
timeout -k 10 600 python -u -m pytest tests/test_gpu_bootk.py tests/test_gpu_ckks.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02v/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r02v/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 5 > gpurun_out/r02v/boot.log 2>&1 || { tail -5 gpurun_out/r02v/boot.log; exit 1; }
tail -4 gpurun_out/r02v/boot.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02v/boot -o boot -- ./phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 2 > gpurun_out/r02v/boot_prof.log 2>&1 || { tail -5 gpurun_out/r02v/boot_prof.log; exit 1; }
python3 tools/prof_last_window.py gpurun_out/r02v/boot > gpurun_out/r02v/boot_warm_kernel_stats.csv
head -12 gpurun_out/r02v/boot_warm_kernel_stats.csv | cut -c1-160
