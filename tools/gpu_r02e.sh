set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_boot
export TMPDIR=/tmp
timeout -k 10 200 ./phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 3 > gpurun_out/boot_r02e.txt 2>&1 || exit 1
grep bootstrap gpurun_out/boot_r02e.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_boot -o boot -- ./phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 2 > gpurun_out/prof_boot.log 2>&1 || { tail -5 gpurun_out/prof_boot.log; exit 1; }
find gpurun_out/prof_boot -name "*stats*" | head
