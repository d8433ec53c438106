# rocprofv3 kernel stats of each NTT library variant under tools/variants/ (tools only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in $(ls tools/variants); do
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/var_$v -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_ntt.py $GRAFT_REPO_ROOT/tools/variants/$v/py > /dev/null 2>&1) || { echo "variant $v failed"; exit 1; }
  echo "== $v"; python3 tools/stats_short.py gpurun_out/var_$v/run_kernel_stats.csv
done
