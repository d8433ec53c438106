# NTT (C2 shape, 44 x 50-bit limbs) kernel traces of the main build and the tools/variants builds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/s3g
cd /tmp
MODE=${MODE:-ntt50} timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/s3g/main -o n -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py > $GRAFT_REPO_ROOT/gpurun_out/s3g/main.log 2>&1 || exit 1
for v in $(ls $GRAFT_REPO_ROOT/tools/variants); do
  PHX_PY=$GRAFT_REPO_ROOT/tools/variants/$v/py MODE=${MODE:-ntt50} timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/s3g/$v -o n -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py > $GRAFT_REPO_ROOT/gpurun_out/s3g/$v.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/s3g/$v.log; exit 1; }
done
