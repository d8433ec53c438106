# MFMA base conversion: C3 kernel traces of the main build and the tools/variants builds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/s3d
cd /tmp
MODE=c3 timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/s3d/main -o c3 -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py > $GRAFT_REPO_ROOT/gpurun_out/s3d/main.log 2>&1 || exit 1
for v in $(ls $GRAFT_REPO_ROOT/tools/variants); do
  PHX_PY=$GRAFT_REPO_ROOT/tools/variants/$v/py MODE=c3 timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/s3d/$v -o c3 -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py > $GRAFT_REPO_ROOT/gpurun_out/s3d/$v.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/s3d/$v.log; exit 1; }
done
