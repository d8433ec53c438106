// ckks.h — CKKS kernels beside the hot path: device-side sampling for key generation and
// encryption (the reference samples on the GPU too, src/prng.cu + sample_* in src/secretkey.cu),
// and the small bootstrap helpers of src/evaluate.cu (monomial multiply, extended-basis glue).
#pragma once

#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

#include "chacha.h"
#include "salsa.h"

namespace phx {

// Sampling from draw `nonce` of the ChaCha20 stream `key` (chacha.h), output [L][n] residues:
// uniform: 128-bit keystream values reduced mod q[l] (one independent value per element)
hipError_t sample_uniform(uint64_t* out, const uint64_t* q, const uint64_t* barrett, size_t n, size_t L,
                          const ChaChaKey& key, uint64_t nonce, hipStream_t s);
// the reference's expansion of a public 64-byte seed into a uniform [L][n] polynomial
// (sample_uniform_poly, src/prng.cu:164-197; salsa.h), bit for bit
hipError_t sample_uniform_seeded(uint64_t* out, const uint64_t* q, const uint64_t* barrett, size_t n, size_t L,
                                 const SalsaSeed& seed, hipStream_t s);
// centered binomial e_k (21 + 21 bits, sigma ~3.24), the same e_k in every limb (coefficient form)
hipError_t sample_cbd(uint64_t* out, const uint64_t* q, size_t n, size_t L, const ChaChaKey& key, uint64_t nonce,
                      hipStream_t s);
// ternary u_k in {-1, 0, 1}, the same u_k in every limb (coefficient form)
hipError_t sample_ternary(uint64_t* out, const uint64_t* q, size_t n, size_t L, const ChaChaKey& key, uint64_t nonce,
                          hipStream_t s);

// out[l][k] = in[l][k] * c[l] mod q[l] + (acc ? acc[l][k] : 0), Shoup constants c/c_shoup per limb
hipError_t mul_scalar_add(const uint64_t* in, const uint64_t* c, const uint64_t* c_shoup, const uint64_t* acc,
                          uint64_t* out, const uint64_t* q, size_t n, size_t L, hipStream_t s);
// out[p][l][k] += in[l][k] * c[l] mod q[l] for p < polys (out[p] at p poly_stride), one launch
hipError_t mul_scalar_accumulate(const uint64_t* in, const uint64_t* c, const uint64_t* c_shoup, uint64_t* out,
                                 size_t poly_stride, size_t polys, const uint64_t* q, size_t n, size_t L, hipStream_t s);

}  // namespace phx

namespace phx {

// ---- hoisted baby-step / giant-step linear transform (bootstrap CoeffToSlot / SlotToCoeff) ----
// For every giant step i < b:
//   out[i][t] = sum_{j < g} baby[j][t] * pts[g i + j]   (t = 0, 1)
// over the extended basis Ql u P ([2][Ql + P][n] ciphertexts, [Ql + P][n] plaintexts).  One
// launch reads every baby and every plaintext once (the reference multiplies and adds one
// (baby, plaintext) pair per launch: EvalMultExt + EvalAddExtInPlace, bootstrap.cu:1322-1332).
// pts is a device array of b * g non-null pointers (absent diagonals point at a zero
// plaintext); every out[i] is non-null.
constexpr int kLtMaxG = 32, kLtMaxB = 64;
struct LtArgs {
  const uint64_t* baby[kLtMaxG];
  uint64_t* out[kLtMaxB];
  const uint64_t* const* pts;  // device array [b][g]
  const uint64_t* q;           // full QP chain
  const uint64_t* barrett;     // [QP][2]
  int g = 0, b = 0, Ql = 0, P = 0, size_Q = 0;
  // every modulus of the chain below 2^60 (phantom::below_2_60): the 30-bit split partial sums
  // may then take 8 (tile kernels) or 16 (lt_bsgs_kernel) products before folding; otherwise a
  // high-half product reaches 2^62 and the sums fold every 4 products (0 is always safe)
  uint32_t q60 = 0;
};
hipError_t lt_bsgs(const LtArgs& a, size_t n, hipStream_t s);
// lt_bsgs of `count` (2..kLtGroupMax) ciphertexts at one level through the same plaintexts
// (bootstraps in lockstep) in one launch, the ciphertexts' blocks for the same elements on one XCD
// so that the plaintexts are read from HBM about once for all.  Each ciphertext's babies are
// contiguous (baby j at baby0[c] + j baby_stride words), its inner sum 0 goes to acc[c] and inner
// sum i >= 1 to giant1[c] + (i - 1) giant_stride; g == 32, b <= 8 (the bootstrap's levels).  Each
// result equals its own lt_bsgs, bit for bit.
#ifndef PHX_GROUP_MAX
#define PHX_GROUP_MAX 8  // ciphertexts of one lockstep group (the grouped kernels' argument arrays)
#endif
constexpr int kLtGroupMax = PHX_GROUP_MAX;
struct LtGroupArgs {
  const uint64_t* const* pts = nullptr;
  const uint64_t* q = nullptr;
  const uint64_t* barrett = nullptr;
  int g = 0, b = 0, Ql = 0, P = 0, size_Q = 0, count = 0;
  uint32_t q60 = 0;  // as LtArgs::q60
  uint64_t baby_stride = 0, giant_stride = 0;
  const uint64_t* baby0[kLtGroupMax] = {};
  uint64_t* acc[kLtGroupMax] = {};
  uint64_t* giant1[kLtGroupMax] = {};
};
hipError_t lt_bsgs_group(const LtGroupArgs& ga, size_t n, hipStream_t s);

// ---- Chebyshev leaves: M linear combinations of the same K ciphertexts in one pass ----------
//   out[m][t][l] = sum_k in[k][t][l] * coef[m][k][l] + (t == 0 ? cadd[m][l] : 0)   (mod q_l)
// in[k]: [2][*][n] ciphertexts with at least L limbs (polynomial stride in_stride[k] elements),
// out[m]: [2][L][n]; coef: device [2][M][K][L] (values, then Shoup quotients), cadd: [M][L].
// Every input is read once for all M outputs (the reference evaluates each leaf by separate
// EvalMult/EvalAdd passes: bootstrap.cu EvalChebyshevSeriesPS).
constexpr int kLeafMaxK = 16, kLeafMaxM = 8;
struct LeafArgs {
  const uint64_t* in[kLeafMaxK];
  size_t in_stride[kLeafMaxK];
  uint64_t* out[kLeafMaxM];
  const uint64_t* coef;
  const uint64_t* cadd;
  const uint64_t* q;
  const uint64_t* barrett;  // [L][2]
  int K = 0, M = 0, L = 0;
};
hipError_t leaf_combine(const LeafArgs& a, size_t n, hipStream_t s);

// out[l] = in[l] * c[l] (+ acc[l]) with per-limb constants passed by value (no device upload);
// L <= kMaxScalarLimbs
constexpr int kMaxScalarLimbs = 64;
struct LimbScalars {
  uint64_t v[kMaxScalarLimbs];
  uint64_t vs[kMaxScalarLimbs];  // Shoup quotients (mul) / unused (add)
};
// mul_scalar_v over `polys` polynomials with the same constants: input p at in + p * in_stride
// (0: L n; a larger stride reads the first L limbs of longer polynomials, i.e. drops limbs),
// out and acc contiguous [polys][L][n]: out = in * c (+ acc)
hipError_t mul_scalar_v(const uint64_t* in, const LimbScalars& c, uint64_t* out, const uint64_t* q, size_t n,
                        size_t L, hipStream_t s, size_t polys = 1, size_t in_stride = 0,
                        const uint64_t* acc = nullptr);
// Tensor product of two [2][L][n] ciphertexts into out [3][L][n] with MulAddRescale's linear
// epilogue fused: d = f (ct1 x ct2) (if scale) and, for t, d[p] += t[p] c for p < 2
// (t[p] at t + p * t_stride, its first L limbs).  out must not alias the inputs.
struct TensorLinArgs {
  const uint64_t* ct1;
  const uint64_t* ct2;
  uint64_t* out;
  const uint64_t* t = nullptr;
  size_t t_stride = 0;
  const uint64_t* q;
  const uint64_t* barrett;
  bool scale = false;
  LimbScalars f;
  LimbScalars c;
};
hipError_t tensor_lin(const TensorLinArgs& a, size_t n, size_t L, hipStream_t s);

// tensor_lin of up to kTensorBatchMax independent products at one level in one launch (one grid
// row per product), with the product's constant folded in as well: for product k,
// out[k] = factor ct1 x ct2 (+ t c in polys 0, 1) (+ cadd in poly 0), every per-limb constant a
// residue (c, cadd) in `limb` [count][2][L] by value.  The values are those of tensor_lin followed
// by add_scalar_v, bit for bit.
constexpr int kTensorBatchMax = 8, kTensorBatchLimbWords = 384;
struct TensorLinJob {
  const uint64_t* ct1;
  const uint64_t* ct2;
  uint64_t* out;
  const uint64_t* t;  // null: no term
  uint64_t t_stride;
  uint64_t factor;    // 1: unscaled
  uint32_t has_const;
};
struct TensorLinBatchArgs {
  const uint64_t* q;
  const uint64_t* barrett;
  uint32_t L = 0, count = 0;
  TensorLinJob job[kTensorBatchMax];
  uint64_t limb[kTensorBatchLimbWords];
};
hipError_t tensor_lin_batch(const TensorLinBatchArgs& a, size_t n, hipStream_t s);

// d[p] = d[p] * ca (ca may be null: unscaled) + (p < t_polys ? t[p] * cb : 0) for p < d_polys;
// d contiguous [d_polys][L][n], t[p] at t + p * t_stride (its first L limbs)
hipError_t lin_comb_v(uint64_t* d, size_t d_polys, const LimbScalars* ca, const uint64_t* t, size_t t_polys,
                      size_t t_stride, const LimbScalars& cb, const uint64_t* q, size_t n, size_t L, hipStream_t s);
hipError_t add_scalar_v(const uint64_t* in, const LimbScalars& c, uint64_t* out, const uint64_t* q, size_t n,
                        size_t L, hipStream_t s);

}  // namespace phx
