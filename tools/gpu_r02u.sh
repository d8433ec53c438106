set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02u
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d gpurun_out/r02u/boot -o boot -- ./phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 2 > gpurun_out/r02u/boot_prof.log 2>&1 || { tail -5 gpurun_out/r02u/boot_prof.log; exit 1; }
ls -R gpurun_out/r02u | head
