set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
NTT_BITS=50 timeout -k 10 300 python -u tools/time_variants.py > gpurun_out/variants50_r02n.log 2>&1 || { tail -20 gpurun_out/variants50_r02n.log; exit 1; }
cat gpurun_out/variants50_r02n.log
NTT_BITS=60 timeout -k 10 300 python -u tools/time_variants.py > gpurun_out/variants60_r02n.log 2>&1 || { tail -20 gpurun_out/variants60_r02n.log; exit 1; }
cat gpurun_out/variants60_r02n.log
