# full validation of the current build: GPU tests, smoke, the default bench line, and a kernel
# trace of a warm bootstrap
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02t
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02t/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r02t/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02t/smoke.log 2>&1 || { tail -5 gpurun_out/r02t/smoke.log; exit 1; }
cat gpurun_out/r02t/smoke.log | tail -2
timeout -k 10 600 python -u bench.py > gpurun_out/r02t/bench.json 2> gpurun_out/r02t/bench.err || { tail -20 gpurun_out/r02t/bench.err; exit 1; }
cat gpurun_out/r02t/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02t/boot -o boot -- ./phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 2 > gpurun_out/r02t/boot_prof.log 2>&1 || { tail -5 gpurun_out/r02t/boot_prof.log; exit 1; }
python3 tools/prof_last_window.py gpurun_out/r02t/boot > gpurun_out/r02t/boot_warm_kernel_stats.csv
head -3 gpurun_out/r02t/boot_warm_kernel_stats.csv | cut -c1-200
