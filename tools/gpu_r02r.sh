set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r02r.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_r02r.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-c5 --no-cpu-baseline --steps 50 > gpurun_out/bench_r02r.json 2> gpurun_out/bench_r02r.err || { tail -20 gpurun_out/bench_r02r.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r02r.json')); print(d['roofline']['fwd_ms'], d['c3']['ms'], d['c4']['ms_median'])"
