# C5 lanes x lockstep-group sweep: throughput and the engine pool's footprint per configuration
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-c5sweep}
mkdir -p $OUT
CFGS=${CFGS:-"2x4 3x4 4x4 2x8 3x8 4x8"}
for cfg in $CFGS; do
  l=${cfg%x*}; g=${cfg#*x}
  timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c3 --no-c4 --c5-batch ${BATCH:-512} \
    --c5-lanes $l --c5-group $g > $OUT/c5_${cfg}.json 2> $OUT/c5_${cfg}.log || { tail -20 $OUT/c5_${cfg}.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c5_${cfg}.json').read().splitlines()[-1])['c5']; print('$cfg', d['bootstraps_per_s'], d['rank0_pool_GiB'], d['min_avg_bits'])"
done
