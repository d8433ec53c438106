# round-2 profiles of the current build: NTT-only bench under rocprofv3 kernel trace (stats), and a
# kernel trace of two bootstraps (the last, warm one is cut out by tools/prof_last_window.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r02o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r02o/bench -o bench -- python3 bench.py --no-c3 --no-c4 --no-c5 --no-cpu-baseline > gpurun_out/prof_r02o/bench_ntt.json 2> gpurun_out/prof_r02o/bench_ntt.err || { tail -5 gpurun_out/prof_r02o/bench_ntt.err; exit 1; }
cat gpurun_out/prof_r02o/bench_ntt.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02o/boot -o boot -- ./phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 2 > gpurun_out/prof_r02o/boot.log 2>&1 || { tail -5 gpurun_out/prof_r02o/boot.log; exit 1; }
python3 tools/prof_last_window.py gpurun_out/prof_r02o/boot > gpurun_out/prof_r02o/boot_warm_kernel_stats.csv
head -12 gpurun_out/prof_r02o/boot_warm_kernel_stats.csv | cut -c1-150
find gpurun_out/prof_r02o -name "*stats*"
