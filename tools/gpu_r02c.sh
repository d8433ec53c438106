set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r02c.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r02c.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r02c.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench_r02c.json 2> gpurun_out/bench_r02c.err || { tail -20 gpurun_out/bench_r02c.err; exit 1; }
cat gpurun_out/bench_r02c.json
