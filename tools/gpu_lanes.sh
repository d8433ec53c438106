# C5 throughput per GPU against the number of concurrent bootstrap lanes, with HIP's default 4
# hardware queues and with 16 (every lane runs 3 streams, so 4 lanes oversubscribe 4 queues).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/lanes
mkdir -p $OUT
run() {  # $1 = lanes, $2 = hardware queues
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 150 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-c4 \
    --c5-batch 240 --c5-lanes $1 --c5-verify 8 > $OUT/l$1_q$2.json 2> $OUT/l$1_q$2.err || { tail -5 $OUT/l$1_q$2.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/l$1_q$2.json').read().strip().splitlines()[-1]); print('lanes', $1, 'queues', $2, d['c5']['bootstraps_per_s'])"
}
for q in 4 16; do
  for l in 1 2 4 6; do run $l $q; done
done
