set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for k in 1 2; do
  PHX_LT_BABY=$k PHX_BOOT_TRACE=1 timeout -k 10 200 ./phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 2 > gpurun_out/boot_trace_k$k.txt 2>&1 || { tail -5 gpurun_out/boot_trace_k$k.txt; exit 1; }
  echo "== baby x$k"; grep -E "^\[boot\]" gpurun_out/boot_trace_k$k.txt | tail -7
  PHX_LT_BABY=$k timeout -k 10 200 ./phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 5 > gpurun_out/boot_k$k.txt 2>&1 || { tail -5 gpurun_out/boot_k$k.txt; exit 1; }
  grep '"stage": "bootstrap"' gpurun_out/boot_k$k.txt | cut -c1-200
done
