# One parametrised GPU-box launcher (replaces the per-experiment gpu_*.sh scripts).
#
#   gpurun -- 'bash tools/gpu.sh STEP [STEP ...]'
#
# Steps run in order; the chain stops at the first failure (every GPU step has its own time
# limit).  Output lands under gpurun_out/$TAG/.  Steps:
#   tests        pytest -m gpu (TESTS=... selects files/-k, default the whole suite)
#   bench        python bench.py $BENCH_ARGS          -> bench.json / bench.log
#   stats        rocprofv3 --kernel-trace --stats of $PROF_CMD (default: bench.py C2 only)
#   boot         the bootstrap example ($RUNS runs) -> boot.txt
#   bootstats    rocprofv3 kernel stats of the bootstrap example (warm runs)
#   pmc          PMC passes ($PMC_SETS, ';'-separated counter sets) over $PMC_CMD
#   traffic      FETCH_SIZE / WRITE_SIZE passes over $PMC_CMD, summarised by tools/pmc_traffic.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-run}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
PY=python3
DEFAULT_PROF="$PY $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 --no-c4 --no-c5"

step_tests() {
  timeout -k 10 ${T_TESTS:-900} $PY -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
  local rc=$?; tail -4 "$OUT/pytest_gpu.log"; return $rc
}
step_bench() {
  timeout -k 10 ${T_BENCH:-600} $PY -u bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.log"
  local rc=$?; tail -c 3000 "$OUT/bench.json"; [ $rc -eq 0 ] || tail -20 "$OUT/bench.log"; return $rc
}
step_stats() {
  (cd /tmp && timeout -k 10 ${T_STATS:-300} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run \
     -- ${PROF_CMD:-$DEFAULT_PROF} > "$OUT/stats.log" 2>&1)
  local rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/stats.log"; return $rc; }
  $PY tools/stats_short.py "$(find "$OUT/stats" -name '*kernel_stats.csv' | head -1)"
}
step_boot() {
  timeout -k 10 ${T_BOOT:-300} phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 ${RUNS:-3} > "$OUT/boot.txt" 2>&1
  local rc=$?; tail -4 "$OUT/boot.txt"; return $rc
}
step_bootstats() {
  PROF_CMD="$GRAFT_REPO_ROOT/phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 ${RUNS:-2}" step_stats
}
step_pmc() {
  local i=0 set
  IFS=';' read -ra sets <<< "${PMC_SETS:?PMC_SETS unset}"
  for set in "${sets[@]}"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL ${T_PMC:-90} rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/pmc$i" -o run \
       -- ${PMC_CMD:?PMC_CMD unset} > "$OUT/pmc$i.log" 2>&1) || { echo "pmc pass $i failed"; tail -5 "$OUT/pmc$i.log"; return 1; }
  done
}
step_profboot() {  # kernel trace of ONE warm bootstrap and ONE lockstep group of $GROUP, one CSV per window
  (cd /tmp && timeout -k 10 ${T_STATS:-300} rocprofv3 --kernel-trace --output-format csv -d "$OUT/profboot" -o run \
     -- "$GRAFT_REPO_ROOT/phantom-fhe-boot_amd/bin/bootstrapping_example" prof 16 ${GROUP:-4} > "$OUT/profboot.log" 2>&1)
  local rc=$?; tail -2 "$OUT/profboot.log"; [ $rc -eq 0 ] || return $rc
  $PY tools/prof_windows.py "$(find "$OUT/profboot" -name '*kernel_trace.csv' | head -1)" "$OUT/boot_window"
}
step_proftrace() {  # kernel + HIP runtime trace of ONE warm bootstrap and ONE lockstep group of $GROUP
  (cd /tmp && timeout -k 10 ${T_STATS:-300} rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv \
     -d "$OUT/proftrace" -o run -- "$GRAFT_REPO_ROOT/phantom-fhe-boot_amd/bin/bootstrapping_example" prof 16 ${GROUP:-4} \
     > "$OUT/proftrace.log" 2>&1)
  local rc=$?; tail -2 "$OUT/proftrace.log"; return $rc
}
step_gaps() {  # idle gaps between kernels of the one-bootstrap window and of the group window of profboot
  local t; t=$(find "$OUT/profboot" -name '*kernel_trace.csv' | head -1)
  echo "single: $($PY tools/kernel_gaps.py "$t" -2)" | tee "$OUT/gaps.txt"
  echo "group:  $($PY tools/kernel_gaps.py "$t" -1)" | tee -a "$OUT/gaps.txt"
}
step_profpmc() {  # FETCH_SIZE per dispatch over the same run (lt_bsgs_wide vs lt_bsgs_group)
  (cd /tmp && timeout -s KILL ${T_PMC:-240} rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv \
     -d "$OUT/profpmc" -o run -- "$GRAFT_REPO_ROOT/phantom-fhe-boot_amd/bin/bootstrapping_example" prof 16 ${GROUP:-4} \
     > "$OUT/profpmc.log" 2>&1) || { tail -5 "$OUT/profpmc.log"; return 1; }
  $PY tools/lt_fetch.py "$OUT/profpmc" > "$OUT/lt_fetch.json" && cat "$OUT/lt_fetch.json"
}
step_traffic() {
  PMC_SETS="FETCH_SIZE;WRITE_SIZE" step_pmc || return 1
  mkdir -p "$OUT/traffic" && mv "$OUT/pmc1" "$OUT/traffic/p1" && mv "$OUT/pmc2" "$OUT/traffic/p2"
  $PY tools/pmc_traffic.py "$OUT/traffic" > "$OUT/traffic.json" && cat "$OUT/traffic.json"
}

for s in "$@"; do
  echo "== step $s"
  "step_$s" || { echo "step $s failed"; exit 1; }
done
