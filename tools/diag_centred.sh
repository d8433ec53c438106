# does mean-unbiased division (tools/variants/diag, -DPHX_DIAG_CENTRED=1; see
# host/rns_tool.cpp) remove the slot-0 offset?  Same seeded keys and ciphertexts through the
# product library and the diagnostic one, both with the unfused key switch (PHX_KS_EPI=0, which the
# diagnostic needs).  TAIL_ONLY_I0=1 keeps only ciphertexts with overflow I = 0 in coefficient 0 or
# N/2, where the offset shows.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-diag}
mkdir -p $OUT
B=phantom-fhe-boot_amd/bin/bootstrapping_example
export PHX_KS_EPI=0 TAIL_KEY_SEED=${SEED:-0x7A11}
# VARS: builds to compare (diag = every division, diagr = the standalone rescales only, diagm = the
# moddowns and the fused moddown + rescale only)
for v in ${VARS:-main diag}; do
  if [ $v = main ]; then LIB=$PWD/phantom-fhe-boot_amd/lib; else LIB=$PWD/tools/variants/$v/lib; fi
  LD_LIBRARY_PATH=$LIB TAIL_ONLY_I0=1 timeout -k 10 400 $B tail 16 ${EVENTS:-6} ${KEYS:-3} > $OUT/i0_$v.txt 2>&1 || { tail -5 $OUT/i0_$v.txt; exit 1; }
  echo "$v $(tail -1 $OUT/i0_$v.txt)"
  [ "${PLAIN:-12}" = 0 ] && continue
  LD_LIBRARY_PATH=$LIB timeout -k 10 300 $B tail 16 ${PLAIN:-12} 1 > $OUT/all_$v.txt 2>&1 || { tail -5 $OUT/all_$v.txt; exit 1; }
  echo "$v $(tail -1 $OUT/all_$v.txt)"
done
