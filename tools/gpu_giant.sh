# Bootstrap latency against the number of concurrent giant-step chains (PHX_BOOT_GIANT_STREAMS)
# and hardware queues; bootstrapping_example boot, 5 timed runs each.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/giant
mkdir -p $OUT
for q in 4 8; do
  for g in 1 2 3 4; do
    GPU_MAX_HW_QUEUES=$q PHX_BOOT_GIANT_STREAMS=$g timeout -k 10 120 phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 5 > $OUT/g${g}_q$q.txt 2>&1 || { tail -5 $OUT/g${g}_q$q.txt; exit 1; }
    echo "giant $g queues $q $(grep '"stage": "bootstrap"' $OUT/g${g}_q$q.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_median"], d["ms_min"], d["avg_bits"])')"
  done
done
