# Bootstrap iteration on the GPU box: all GPU parity tests, the bootstrap example, and a
# rocprofv3 kernel trace of it (per-kernel stats + per-dispatch trace, csv).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-boot}
RUNS=${RUNS:-3}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 $RUNS > gpurun_out/boot_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/boot_$TAG.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- $GRAFT_REPO_ROOT/phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log; exit $rc; }
echo profiled
