# The opt-in unbiased moddown (PHX_UNBIASED_MODDOWN=1) against the default on the same seeded keys
# and ciphertexts: the slot-0 events (TAIL_ONLY_I0=1, overflow I = 0 in coefficient 0 or N/2, where
# the moddowns' bias shows; tools/diag_centred.sh is the round-5 diagnostic build's version) and
# plain fresh ciphertexts.  Default fused key switch (no PHX_KS_EPI=0 needed).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-unbiased}
mkdir -p $OUT
B=phantom-fhe-boot_amd/bin/bootstrapping_example
export TAIL_KEY_SEED=${SEED:-0x7A11}
for v in off on; do
  U=0; [ $v = on ] && U=1
  PHX_UNBIASED_MODDOWN=$U TAIL_ONLY_I0=1 timeout -k 10 400 $B tail 16 ${EVENTS:-6} ${KEYS:-3} > $OUT/i0_$v.txt 2>&1 || { tail -5 $OUT/i0_$v.txt; exit 1; }
  echo "$v $(tail -1 $OUT/i0_$v.txt)"
  PHX_UNBIASED_MODDOWN=$U timeout -k 10 300 $B tail 16 ${PLAIN:-24} 1 > $OUT/all_$v.txt 2>&1 || { tail -5 $OUT/all_$v.txt; exit 1; }
  echo "$v $(tail -1 $OUT/all_$v.txt)"
done
for v in off on; do
  PHX_UNBIASED_MODDOWN=$([ $v = on ] && echo 1 || echo 0) timeout -k 10 200 $B boot 16 5 > $OUT/boot_$v.txt 2>&1 || exit 1
  echo "$v $(grep '"stage": "bootstrap"' $OUT/boot_$v.txt | cut -c1-160)"
done
