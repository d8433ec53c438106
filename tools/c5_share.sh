# C5 at the 8-GPU job's per-rank count (128) and at the 1-GPU count (1024) on one box, alternating,
# with bench.py's default lanes x group (c5_shape): the per-rank share against the full batch
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-c5share}; mkdir -p $OUT
for i in 1 2; do for b in 128 1024; do
  timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c3 --no-c4 --c5-batch $b \
    > $OUT/c5_${b}_$i.json 2> $OUT/c5_${b}_$i.log || { tail -20 $OUT/c5_${b}_$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c5_${b}_$i.json').read().splitlines()[-1])['c5']; print($b, d['lanes_per_rank'], d['lockstep_group'], d['bootstraps_per_s'], d['max_rank_s'], d['rank0_pool_GiB'])" | tee -a $OUT/summary.txt
done; done
