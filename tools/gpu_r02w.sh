# timing only: bootstrap example x2 + warm kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02w
timeout -k 10 300 ./phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 5 > gpurun_out/r02w/boot.log 2>&1 || { tail -5 gpurun_out/r02w/boot.log; exit 1; }
grep ms_median gpurun_out/r02w/boot.log | cut -c1-130
timeout -k 10 300 ./phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 5 > gpurun_out/r02w/boot2.log 2>&1 || { tail -5 gpurun_out/r02w/boot2.log; exit 1; }
grep ms_median gpurun_out/r02w/boot2.log | cut -c1-130
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02w/boot -o boot -- ./phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 2 > gpurun_out/r02w/boot_prof.log 2>&1 || { tail -5 gpurun_out/r02w/boot_prof.log; exit 1; }
python3 tools/prof_last_window.py gpurun_out/r02w/boot > gpurun_out/r02w/boot_warm_kernel_stats.csv
grep -E "window|lt_bsgs|batch_full" gpurun_out/r02w/boot_warm_kernel_stats.csv | cut -c1-150
