set -o pipefail
rm -rf gpurun_out/abks; mkdir -p gpurun_out/abks
for i in 1 2 3; do for v in ${VARS:-base kc2w3 kc1w3}; do
  timeout -k 10 200 python3 tools/time_c3.py tools/variants/$v/py >> gpurun_out/abks/c3.txt 2>&1 || exit 1
  LD_LIBRARY_PATH=$PWD/tools/variants/$v/lib timeout -k 10 200 phantom-fhe-boot_amd/bin/bootstrapping_example boot 16 3 > gpurun_out/abks/boot_${v}_${i}.txt 2>&1 || exit 1
  echo "$v $(grep '"stage": "bootstrap"' gpurun_out/abks/boot_${v}_${i}.txt | cut -c1-120)" >> gpurun_out/abks/boot.txt
done; done
cat gpurun_out/abks/c3.txt | grep -v amdgpu.ids; cat gpurun_out/abks/boot.txt
