# C3 leg of bench.py for each library variant under tools/variants/ (tools only)
cd $GRAFT_REPO_ROOT
for v in $(ls tools/variants); do
  PHANTOM_AMD_LIB=$GRAFT_REPO_ROOT/tools/variants/$v/lib/libphantom_amd.so timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', d['roofline']['fwd_ms'], d['c3']['ms'], d['c3']['total_ms'])" || exit 1
done
