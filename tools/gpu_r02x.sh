# C3 relinearize kernel split (rocprofv3 kernel trace over tools/prof_kernels.py MODE=c3)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02x
cd /tmp
MODE=c3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r02x/c3 -o c3 -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py > $GRAFT_REPO_ROOT/gpurun_out/r02x/c3.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r02x/c3.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/r02x/c3 -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | head -16
