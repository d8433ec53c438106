set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bootk.py -x -q --timeout 200 --timeout-method thread -k lt_bsgs > gpurun_out/pytest_ltb.log 2>&1 || { tail -20 gpurun_out/pytest_ltb.log; exit 1; }
tail -2 gpurun_out/pytest_ltb.log
for k in 1 2; do
  PHX_LT_BABY=$k PHX_BOOT_TRACE=1 timeout -k 10 200 ./phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 2 > gpurun_out/boot_trace_s$k.txt 2>&1 || { tail -5 gpurun_out/boot_trace_s$k.txt; exit 1; }
  echo "== baby x$k"; grep -E "^\[boot\]" gpurun_out/boot_trace_s$k.txt | tail -6
  PHX_LT_BABY=$k timeout -k 10 200 ./phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 5 > gpurun_out/boot_s$k.txt 2>&1 || { tail -5 gpurun_out/boot_s$k.txt; exit 1; }
  grep '"stage": "bootstrap"' gpurun_out/boot_s$k.txt | cut -c1-160
done
