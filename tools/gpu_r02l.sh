set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r02l.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_r02l.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-c5 --no-cpu-baseline > gpurun_out/bench_r02l.json 2> gpurun_out/bench_r02l.err || { tail -20 gpurun_out/bench_r02l.err; exit 1; }
cat gpurun_out/bench_r02l.json
