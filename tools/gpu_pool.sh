# Full GPU tests, then C5 at lockstep groups of 4 and 8 (pool footprint in the c5 entry)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-pool}
mkdir -p $OUT
if [ "${RUN_TESTS:-1}" = 1 ]; then timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc; fi
for g in 4 8; do
  timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-c4 --c5-group $g > $OUT/c5_g$g.json 2> $OUT/c5_g$g.log || { tail -20 $OUT/c5_g$g.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/c5_g$g.json').read().splitlines()[-1])['c5']; print({k: d[k] for k in ('bootstraps_per_s','lockstep_group','min_avg_bits','rank0_pool_GiB','roofline')})"
done
