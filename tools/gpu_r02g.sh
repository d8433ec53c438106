set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r02g.log 2>&1
rc=$?
tail -8 gpurun_out/pytest_gpu_r02g.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r02g.json 2> gpurun_out/bench_r02g.err || { tail -20 gpurun_out/bench_r02g.err; exit 1; }
cat gpurun_out/bench_r02g.json
