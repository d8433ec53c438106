# C3 relinearize kernel trace for each library variant under tools/variants/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02z
cd /tmp
for v in $(ls $GRAFT_REPO_ROOT/tools/variants); do
  PHX_PY=$GRAFT_REPO_ROOT/tools/variants/$v/py MODE=c3 timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r02z/$v -o c3 -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py > $GRAFT_REPO_ROOT/gpurun_out/r02z/$v.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r02z/$v.log; exit 1; }
done
