// evaluate.h — CKKS evaluator API with the reference's names and semantics
// (include/evaluate.cuh:31-260; CKKS branches of src/evaluate.cu).  All functions enqueue on
// the context's stream; errors are std::invalid_argument as in the reference.
#pragma once

#include "ciphertext.h"
#include "context.h"
#include "keys.h"

namespace phantom {

// keyswitch_inplace (src/eval_key_switch.cu:112-212): (c0, c1) += KeySwitch(c2) under `evk`
// (device array of dnum digit pointers).
void keyswitch_inplace(const PhantomContext& ctx, PhantomCiphertext& encrypted, const uint64_t* c2,
                       const uint64_t* const* evk);
// the same on raw device buffers: ct is [2][size_Ql][n] at `chain_index`, c2 [size_Ql][n]
void keyswitch_raw(const PhantomContext& ctx, size_t chain_index, uint64_t* ct, const uint64_t* c2,
                   const uint64_t* const* evk, hipStream_t s);

void add_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b);
void sub_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b, bool negate = false);
void negate_inplace(const PhantomContext& ctx, PhantomCiphertext& a);
void add_plain_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomPlaintext& p);
void multiply_plain_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomPlaintext& p);

// multiply_inplace (src/evaluate.cu:1183-1216 -> bgv_ckks_multiply :415-473)
void multiply_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b);
PhantomCiphertext multiply(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomCiphertext& b);

// relinearize_inplace (src/evaluate.cu:1552-1589)
void relinearize_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomRelinKey& rlk);
inline PhantomCiphertext relinearize(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomRelinKey& rlk) {
  PhantomCiphertext d = a;
  relinearize_inplace(ctx, d, rlk);
  return d;
}

// rescale_to_next (src/evaluate.cu:1779-1801 -> mod_switch_scale_to_next :1591-1647)
PhantomCiphertext rescale_to_next(const PhantomContext& ctx, const PhantomCiphertext& a);
inline void rescale_to_next_inplace(const PhantomContext& ctx, PhantomCiphertext& a) { a = rescale_to_next(ctx, a); }

// mod_switch_to_next (src/evaluate.cu:1650-1777, CKKS in NTT form: drop the last limb)
PhantomCiphertext mod_switch_to_next(const PhantomContext& ctx, const PhantomCiphertext& a);
inline void mod_switch_to_next_inplace(const PhantomContext& ctx, PhantomCiphertext& a) {
  a = mod_switch_to_next(ctx, a);
}
void mod_switch_to_inplace(const PhantomContext& ctx, PhantomCiphertext& a, size_t chain_index);
// a copy of `a` at `chain_index` (its leading limbs), one strided device copy
PhantomCiphertext mod_switch_to(const PhantomContext& ctx, const PhantomCiphertext& a, size_t chain_index);

// apply_galois_inplace / rotate_inplace (src/evaluate.cu:1830-1900, NTT-domain path)
void apply_galois_inplace(const PhantomContext& ctx, PhantomCiphertext& a, uint32_t galois_elt,
                          const PhantomGaloisKey& keys);
void rotate_inplace(const PhantomContext& ctx, PhantomCiphertext& a, int step, const PhantomGaloisKey& keys);

}  // namespace phantom
