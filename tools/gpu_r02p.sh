set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r02p.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_r02p.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-c5 --no-cpu-baseline --steps 50 > gpurun_out/bench_r02p.json 2> gpurun_out/bench_r02p.err || { tail -20 gpurun_out/bench_r02p.err; exit 1; }
cat gpurun_out/bench_r02p.json
PHX_FUSED_BCONV=0 timeout -k 10 300 python -u bench.py --no-c5 --no-cpu-baseline --steps 50 > gpurun_out/bench_r02p_unfused.json 2> gpurun_out/bench_r02p_unfused.err || { tail -20 gpurun_out/bench_r02p_unfused.err; exit 1; }
cat gpurun_out/bench_r02p_unfused.json
