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
// whether key switches form the Ql half of their inner product inside the moddown finish (the NTT
// epilogue, ntt.h NttEpilogue::ks_beta); PHX_KS_EPI=0 turns it off (the separate kernel)
bool ks_epilogue_enabled();
void keyswitch_raw(const PhantomContext& ctx, size_t chain_index, uint64_t* ct, const uint64_t* c2,
                   const uint64_t* const* evk, hipStream_t s);

// add_inplace / sub_inplace (src/evaluate.cu:127-229, 308-413): same chain index, NTT form, size
// and noise-scale degree, else std::invalid_argument (as the reference, a scale mismatch is not
// an error here)
void add_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b);
void sub_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b, bool negate = false);
void negate_inplace(const PhantomContext& ctx, PhantomCiphertext& a);
inline PhantomCiphertext negate(const PhantomContext& ctx, const PhantomCiphertext& a) {
  PhantomCiphertext d = a;
  negate_inplace(ctx, d);
  return d;
}
inline PhantomCiphertext add(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomCiphertext& b) {
  PhantomCiphertext d = a;
  add_inplace(ctx, d, b);
  return d;
}
inline PhantomCiphertext sub(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomCiphertext& b,
                             bool negate = false) {
  PhantomCiphertext d = a;
  sub_inplace(ctx, d, b, negate);
  return d;
}
// add_many (src/evaluate.cu:232-306): destination = sum of `encrypteds`, one kernel per polynomial
// reading every operand once (add_many_rns_poly); the operands must share chain index, NTT form,
// scale and size, and destination must not be one of them
void add_many(const PhantomContext& ctx, const std::vector<PhantomCiphertext>& encrypteds,
              PhantomCiphertext& destination);
// add_plain_inplace / sub_plain_inplace (src/evaluate.cu:1281-1420): c0 +-= plain; the plaintext
// must be at the ciphertext's chain index with the same scale
void add_plain_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomPlaintext& p);
void sub_plain_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomPlaintext& p);
inline PhantomCiphertext add_plain(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomPlaintext& p) {
  PhantomCiphertext d = a;
  add_plain_inplace(ctx, d, p);
  return d;
}
inline PhantomCiphertext sub_plain(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomPlaintext& p) {
  PhantomCiphertext d = a;
  sub_plain_inplace(ctx, d, p);
  return d;
}
void multiply_plain_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomPlaintext& p);
inline PhantomCiphertext multiply_plain(const PhantomContext& ctx, const PhantomCiphertext& a,
                                        const PhantomPlaintext& p) {
  PhantomCiphertext d = a;
  multiply_plain_inplace(ctx, d, p);
  return d;
}

// multiply_inplace (src/evaluate.cu:1183-1216 -> bgv_ckks_multiply :415-473): when both operands
// are the same object the squaring kernel runs (tensor_square_2x2_rns_poly, :443-450)
void multiply_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b);
PhantomCiphertext multiply(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomCiphertext& b);
// multiply_and_relin_inplace (src/evaluate.cu:1220-1279): tensor product then relinearization
void multiply_and_relin_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b,
                                const PhantomRelinKey& rlk);
inline PhantomCiphertext multiply_and_relin(const PhantomContext& ctx, const PhantomCiphertext& a,
                                            const PhantomCiphertext& b, const PhantomRelinKey& rlk) {
  PhantomCiphertext d = a;
  multiply_and_relin_inplace(ctx, d, &a == &b ? d : b, rlk);
  return d;
}

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

// plaintext modulus switching (src/evaluate.cu:1700-1731, include/evaluate.cuh:199-239): drop the
// last limb(s); "end of modulus switching chain reached" / "cannot switch to higher level modulus"
void mod_switch_to_next_inplace(const PhantomContext& ctx, PhantomPlaintext& plain);
inline PhantomPlaintext mod_switch_to_next(const PhantomContext& ctx, const PhantomPlaintext& plain) {
  PhantomPlaintext d = plain;
  mod_switch_to_next_inplace(ctx, d);
  return d;
}
void mod_switch_to_inplace(const PhantomContext& ctx, PhantomPlaintext& plain, size_t chain_index);
inline PhantomPlaintext mod_switch_to(const PhantomContext& ctx, const PhantomPlaintext& plain, size_t chain_index) {
  PhantomPlaintext d = plain;
  mod_switch_to_inplace(ctx, d, chain_index);
  return d;
}

// apply_galois_inplace / rotate_inplace (src/evaluate.cu:1803-1920, NTT-domain path).  A rotation
// whose key is absent is composed from the keys of its non-adjacent form (rotate_internal,
// :1877-1914), and throws "Galois key not present" when the step is itself a power of two.
void apply_galois_inplace(const PhantomContext& ctx, PhantomCiphertext& a, uint32_t galois_elt,
                          const PhantomGaloisKey& keys);
inline PhantomCiphertext apply_galois(const PhantomContext& ctx, const PhantomCiphertext& a, uint32_t galois_elt,
                                      const PhantomGaloisKey& keys) {
  PhantomCiphertext d = a;
  apply_galois_inplace(ctx, d, galois_elt, keys);
  return d;
}
void rotate_inplace(const PhantomContext& ctx, PhantomCiphertext& a, int step, const PhantomGaloisKey& keys);
inline PhantomCiphertext rotate(const PhantomContext& ctx, const PhantomCiphertext& a, int step,
                                const PhantomGaloisKey& keys) {
  PhantomCiphertext d = a;
  rotate_inplace(ctx, d, step, keys);
  return d;
}
// hoisting_inplace (src/evaluate.cu:1922-2149): ct <- sum over `steps` of rotate(ct, step), with
// one modup of c1 shared by every rotation (standard, non-fused Galois keys: each step permutes
// the shared digits and takes one inner product; the sums are moved down once)
void hoisting_inplace(const PhantomContext& ctx, PhantomCiphertext& ct, const PhantomGaloisKey& keys,
                      const std::vector<int>& steps);
inline PhantomCiphertext hoisting(const PhantomContext& ctx, const PhantomCiphertext& ct, const PhantomGaloisKey& keys,
                                  const std::vector<int>& steps) {
  PhantomCiphertext d = ct;
  hoisting_inplace(ctx, d, keys, steps);
  return d;
}

}  // namespace phantom
