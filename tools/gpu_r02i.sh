set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
NTT_BITS=60 timeout -k 10 300 python -u tools/time_variants.py > gpurun_out/variants60_r02i.log 2>&1 || { tail -20 gpurun_out/variants60_r02i.log; exit 1; }
cat gpurun_out/variants60_r02i.log
NTT_BITS=50 timeout -k 10 300 python -u tools/time_variants.py > gpurun_out/variants50_r02i.log 2>&1 || { tail -20 gpurun_out/variants50_r02i.log; exit 1; }
cat gpurun_out/variants50_r02i.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r02i.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_r02i.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-c5 --no-cpu-baseline > gpurun_out/bench_r02i.json 2> gpurun_out/bench_r02i.err || { tail -20 gpurun_out/bench_r02i.err; exit 1; }
cat gpurun_out/bench_r02i.json
