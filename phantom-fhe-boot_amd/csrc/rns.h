// rns.h — RNS polynomial kernels on gfx950: elementwise arithmetic (src/polymath.cu), fast
// base conversion (src/rns_bconv.cu), hybrid key-switch pieces (src/rns_bconv.cu:530-843,
// src/eval_key_switch.cu; the moddown and rescale finishes run as forward-NTT epilogues, ntt.h),
// NTT-domain automorphism (src/galois.cu:104-119) and the bootstrap helpers
// (src/evaluate.cu:2414-2554).
//
// Every launcher enqueues on `stream` and returns hipGetLastError().  Modulus arrays are
// device arrays indexed by limb; `barrett` is [limb][2] = floor(2^128/q) {lo, hi}.
#pragma once

#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace phx {

// Per-limb modulus view (device pointers).
struct ModView {
  const uint64_t* q = nullptr;
  const uint64_t* barrett = nullptr;  // [L][2]
};

// ---- elementwise, all [L][n] limb-major, one modulus per limb -------------------------
// `polys` polynomials per launch: a and out contiguous [polys][L][n]; b at b + p * b_stride
// (kContiguous: [polys][L][n] too; 0: the same b for every polynomial, e.g. a plaintext)
constexpr size_t kContiguous = ~size_t(0);
hipError_t poly_add(const uint64_t* a, const uint64_t* b, uint64_t* out, ModView m, size_t n, size_t L,
                    hipStream_t s, size_t polys = 1, size_t b_stride = kContiguous);
hipError_t poly_sub(const uint64_t* a, const uint64_t* b, uint64_t* out, ModView m, size_t n, size_t L,
                    hipStream_t s, size_t polys = 1, size_t b_stride = kContiguous);
hipError_t poly_negate(const uint64_t* a, uint64_t* out, ModView m, size_t n, size_t L, hipStream_t s,
                       size_t polys = 1);
hipError_t poly_mul(const uint64_t* a, const uint64_t* b, uint64_t* out, ModView m, size_t n, size_t L,
                    hipStream_t s, size_t polys = 1, size_t b_stride = kContiguous);
// out = sum of the polynomials in[0 .. count) (add_many_rns_poly, src/polymath.cu): each operand
// is read once; `polys` polynomials per operand, operand i's polynomial y at in[i] + y * stride
constexpr int kAddManyMax = 16;
struct AddManyArgs {
  const uint64_t* in[kAddManyMax];
  int count = 0;
  bool accumulate = false;  // out += sum (chunks of more than kAddManyMax operands)
};
hipError_t poly_add_many(const AddManyArgs& a, uint64_t* out, ModView m, size_t n, size_t L, hipStream_t s,
                         size_t polys, size_t stride);
// out = a * b + c
hipError_t poly_mul_add(const uint64_t* a, const uint64_t* b, const uint64_t* c, uint64_t* out, ModView m,
                        size_t n, size_t L, hipStream_t s);
// out[l] = a[l] * scalar[l] (scalar, scalar_shoup: device arrays of L)
hipError_t poly_mul_scalar(const uint64_t* a, const uint64_t* scalar, const uint64_t* scalar_shoup, uint64_t* out,
                           ModView m, size_t n, size_t L, hipStream_t s, size_t polys = 1);
// out[l] = a[l] + scalar[l]
hipError_t poly_add_scalar(const uint64_t* a, const uint64_t* scalar, uint64_t* out, ModView m, size_t n,
                           size_t L, hipStream_t s);
// (c0, c1) x (d0, d1) -> (c0 d0, c0 d1 + c1 d0, c1 d1); ct1/ct2 are [2][L][n], out [3][L][n]
// (tensor_prod_2x2_rns_poly, src/polymath.cu:501-536).  out may alias ct1.
hipError_t tensor_prod_2x2(const uint64_t* ct1, const uint64_t* ct2, uint64_t* out, ModView m, size_t n, size_t L,
                           hipStream_t s);
// (c0, c1)^2 -> (c0^2, 2 c0 c1, c1^2) (tensor_square_2x2_rns_poly, src/polymath.cu:538-582); ct is
// [2][L][n], out [3][L][n], out may alias ct
hipError_t tensor_square_2x2(const uint64_t* ct, uint64_t* out, ModView m, size_t n, size_t L, hipStream_t s);

// ---- base conversion ------------------------------------------------------------------
// Fast base conversion (bconv_mult + bconv_matmul, src/rns_bconv.cu:40-179, 455-485):
//   t_i = [x_i * qhat_inv_i]_{q_i}            (skipped when qhat_inv == nullptr: x already scaled)
//   y_j = sum_i t_i * qhat_mod_p[i][j] mod p_j
// Output limb j goes to out[(j < skip_at ? j : j + skip_len) * n].
struct BconvArgs {
  const uint64_t* in;            // [ibase][n]
  uint64_t* out;
  const uint64_t* ibase;         // [ibase]
  const uint64_t* qhat_inv;      // [ibase] or nullptr
  const uint64_t* qhat_inv_shoup;
  const uint64_t* qhat_mod_p;    // [ibase][obase]
  const uint64_t* obase;         // [obase]
  const uint64_t* obase_barrett; // [obase][2]
  int ibase_size = 0;
  int obase_size = 0;
  int skip_at = 1 << 30;
  int skip_len = 0;
  // batch: `polys` inputs at in + p * in_stride, outputs at out + p * out_stride (elements)
  int polys = 1;
  size_t in_stride = 0;
  size_t out_stride = 0;
  // digits: with jobs > 1 the `polys` conversions are different converters of one shape (the
  // modup digits): conversion d uses job_qhat_mod_p[d], job_obase[d], job_obase_barrett[d] and
  // skips at skip_at + d * skip_step
  static constexpr int kMaxJobs = 8;
  int jobs = 1;
  int skip_step = 0;
  // several independent batches of the same job set (the giant steps' modups): with period > 0,
  // polynomial z runs job z % period at in + (z / period) in_outer + (z % period) in_stride (out
  // likewise) and skips at skip_at + (z % period) skip_step; polys is a multiple of period
  int period = 0;
  size_t in_outer = 0;
  size_t out_outer = 0;
  const uint64_t* job_qhat_mod_p[kMaxJobs] = {};
  const uint64_t* job_obase[kMaxJobs] = {};
  const uint64_t* job_obase_barrett[kMaxJobs] = {};
  // Matrix-core form (bconv_mfma_tables): with these set, ibase <= 16, obase <= 64 and n a
  // multiple of 16, the conversion runs as int8 MFMA products (rns.hip, bconv_mfma_kernel)
  const void* mfma_frag = nullptr;       // A fragments, bconv_mfma_frag_bytes(ibase, obase) bytes
  const uint64_t* mfma_rows = nullptr;   // [16 * ceil(obase / 16)][2] = {p_j, bits of double(1 / p_j)}
  const void* job_mfma_frag[kMaxJobs] = {};
  const uint64_t* job_mfma_rows[kMaxJobs] = {};
};
hipError_t bconv(const BconvArgs& a, size_t n, hipStream_t s);

// Matrix-core base conversion tables.  The conversion y_j = sum_s t_s c_sj mod p_j runs as int8
// MFMA products: with m_{s,a,j} = c_sj 256^a mod p_j and t_s = sum_a d_{s,a} 256^a (signed base-256
// digits d in [-128, 128)), y_j = sum_b 256^b T_bj (mod p_j) with T_bj = sum_{s,a} d_{s,a} e_b(m_{s,a,j})
// (e_b: signed digit b), 8 int8 GEMMs with K = 8 ibase.  The host precomputes the A fragments of
// v_mfma_i32_16x16x64_i8: [jb][b][kstep][lane][16 bytes], lane (r, g) = (lane & 15, lane >> 4)
// holding row j = 16 jb + r, bytes i <-> (limb s = 8 kstep + 2 g + i / 8, digit a = i % 8).
constexpr int kBconvMfmaMaxIbase = 16;
constexpr int kBconvMfmaMaxObase = 64;
size_t bconv_mfma_frag_bytes(int ibase, int obase);
// fills frag (bconv_mfma_frag_bytes) and rows from qhat_mod_p [ibase][obase] and obase (host arrays)
void bconv_mfma_tables(const uint64_t* qhat_mod_p, const uint64_t* obase, int ibase, int obase_size, uint8_t* frag,
                       uint64_t* rows);

// ---- hybrid key switching -------------------------------------------------------------
// modup_copy_partQl_kernel (src/rns_bconv.cu:522-528): t_mod_up[beta][qlp] gets the digit's own
// NTT-form limbs of c2 for every digit.
hipError_t modup_copy_digits(const uint64_t* c2, uint64_t* t_mod_up, size_t n, size_t size_ql, size_t size_qlp,
                             size_t alpha, hipStream_t s);
// key_switch_inner_prod_c2_and_evk (src/eval_key_switch.cu:26-85).  evk: device array of
// beta pointers to [2][size_QP][n] key digits; modulus/barrett over the full QP chain.
// Optional addend: cx[t][l] += P c[t][l] for the Ql limbs (c [2][size_ql][n], P mod q_l with
// Shoup quotients), i.e. the P-scaled extended form of (c0, c1) + KeySwitch(c2).  first_limb:
// only limbs [first_limb, size_ql + size_p) are formed (first_limb = size_ql: the P half, when the
// moddown's NTT epilogue forms the Ql half itself, ntt.h NttEpilogue::ks_beta).
struct KsAddend {
  const uint64_t* c = nullptr;
  const uint64_t* pmod = nullptr;
  const uint64_t* pmod_shoup = nullptr;
};
hipError_t keyswitch_inner_prod(const uint64_t* t_mod_up, const uint64_t* const* evk, uint64_t* cx,
                                const uint64_t* qp_mod, const uint64_t* qp_barrett, size_t n, size_t size_ql,
                                size_t size_q, size_t size_p, size_t beta, hipStream_t s,
                                const KsAddend& add = KsAddend{}, size_t first_limb = 0);
// Coefficient-domain moddown whose result goes straight into a modup (a giant-step rotation of
// an extended-basis ciphertext): c1 and delta [size_ql][n] coefficient form,
//   y = (c1 - delta) P^-1 mod q_l -> t_mod_up[l / alpha][l]  (the digit's own limb)
//   t_cks[l] = y partQlHatInv_l                                (the digits' base-conversion input)
struct ModdownModupConsts {
  const uint64_t* q;  // Ql
  const uint64_t* pinv;
  const uint64_t* pinv_shoup;
  const uint64_t* hatinv;
  const uint64_t* hatinv_shoup;
  uint64_t bias = 0;  // added to every output coefficient (the opt-in unbiased moddown; 0 = off)
};
// `polys` independent ones per launch: c1 at p c1_stride, t_mod_up at p mod_up_stride, delta and
// t_cks contiguous [polys][size_ql][n]
hipError_t moddown_modup_finish(const uint64_t* c1, const uint64_t* delta, const ModdownModupConsts& k,
                                uint64_t* t_cks, uint64_t* t_mod_up, size_t n, size_t size_ql, size_t size_qlp,
                                size_t alpha, hipStream_t s, size_t polys = 1, size_t c1_stride = 0,
                                size_t mod_up_stride = 0);

// ---- automorphism ---------------------------------------------------------------------
// apply_galois_ntt_permutation_direct (src/galois.cu:104-119): out[l][j] = in[l][perm[j]]
hipError_t galois_ntt(const uint64_t* in, uint64_t* out, const uint32_t* perm, size_t n, size_t L,
                      hipStream_t s);

// Hoisted-rotation epilogue (EvalFastRotationExt, src/evaluate.cu:3770-3860: add P c0, then
// the NTT-domain automorphism), fused with the giant-step accumulation of the linear
// transforms.  cx [2][qlp][n] is the key-switch output before the permutation:
//   mode 0: x = cx
//   mode 1: x = cx + (P c0 on the first ql limbs of polynomial 0)   c0 [ql][n], pmod per limb
//   mode 2: x = cx + (c0 on every limb of polynomial 0)             c0 [qlp][n]
//   out[t][l][j] = (accumulate ? out[t][l][j] : 0) + x[t][l][perm[j]]
// q: the extended-basis moduli in buffer order.  out must not alias cx or c0.
// Key switch fused with its automorphism epilogue (EvalFastRotationExt / the giant-step
// rotate-and-accumulate, src/evaluate.cu:3660-3755): for every limb l of Ql u P and output
// index i with source j = perm[i],
//   v_t[j] = sum_b digits[b][l][j] * evk[b][t][row(l)][j]  mod q_l      (the inner product)
//   mode 1: v_0[j] += P * c0[l][j] for l < Ql;  mode 2: v_0[j] += c0[l][j];  mode 0: nothing
//   out[t][l][i] = v_t[perm[i]] (+ out[t][l][i] when accumulate)
// The inner product of a source block is computed into LDS and written permuted, so the key
// switch's output never makes an HBM round trip before the permutation (galois_finish).
struct KsRotateArgs {
  const uint64_t* digits = nullptr;      // [beta][QlP][n]
  const uint64_t* const* evk = nullptr;  // device array of beta pointers to [2][size_QP][n]
  const uint64_t* qp = nullptr;          // full-chain modulus / Barrett tables (by table row)
  const uint64_t* qp_barrett = nullptr;
  const uint64_t* c0 = nullptr;          // mode 1: [Ql][n]; mode 2: [QlP][n]
  const uint64_t* pmod = nullptr;        // mode 1: P mod q_l, Shoup
  const uint64_t* pmod_shoup = nullptr;
  uint64_t* out = nullptr;               // [2][QlP][n]; must not alias digits / c0
  const uint32_t* perm = nullptr;
  uint32_t ql = 0, qlp = 0, size_q = 0, size_p = 0, beta = 0;
  bool accumulate = false;
};
hipError_t keyswitch_rotate(const KsRotateArgs& a, int mode, size_t n, hipStream_t s);
// keyswitch_rotate of `count` (2..kKsGroupMax) ciphertexts by the same rotation (evk, perm) in one
// launch, their workgroups of an output block on one XCD so that the key is read from HBM about
// once for all; each result equals its own keyswitch_rotate, bit for bit
#ifndef PHX_GROUP_MAX
#define PHX_GROUP_MAX 8  // ciphertexts of one lockstep group (the grouped kernels' argument arrays)
#endif
constexpr int kKsGroupMax = PHX_GROUP_MAX;
struct KsRotateGroupArgs {
  KsRotateArgs a[kKsGroupMax];
  int count = 1;
};
hipError_t keyswitch_rotate_group(const KsRotateGroupArgs& ga, int mode, size_t n, hipStream_t s);

// Batched baby steps: keyswitch_rotate (mode 1) for several rotations of one ciphertext in ONE
// launch.  A workgroup owns a SOURCE block (limb l, kGaloisBlock consecutive indices), reads the
// shared digits and c0 there once from HBM, and for each entry writes the output block that block
// maps to (binv) -- the digits are read once per level instead of once per rotation.
constexpr uint32_t kGaloisBlock = 1024;  // automorphism block (min(n, this) consecutive indices)
struct KsBatchEntry {
  const uint64_t* const* evk = nullptr;  // device array of beta key pointers; nullptr: identity, out = P (c0, c1)
  const uint32_t* perm = nullptr;        // NTT-domain permutation of the rotation
  const uint32_t* binv = nullptr;        // source block -> output block (n / min(n, kGaloisBlock) entries)
  int64_t out_off = 0;                   // output [2][QlP][n] at out + out_off (elements)
};
struct KsRotateBatchArgs {
  const uint64_t* digits = nullptr;        // [beta][QlP][n]
  const KsBatchEntry* entries = nullptr;   // device array of `count` entries
  uint32_t count = 0;
  const uint64_t* qp = nullptr;            // full-chain modulus / Barrett tables (by table row)
  const uint64_t* qp_barrett = nullptr;
  const uint64_t* ct = nullptr;            // [2][Ql][n]: c0 (every entry), c1 (identity entries)
  const uint64_t* pmod = nullptr;          // P mod q_l, Shoup
  const uint64_t* pmod_shoup = nullptr;
  uint64_t* out = nullptr;                 // base of the outputs; must not alias digits / ct
  uint32_t ql = 0, qlp = 0, size_q = 0, size_p = 0, beta = 0;
  // every key modulus is below 2^60 (set from the context): the grouped kernel may then reduce
  // with approximate quotients (lazy sums below 12q); otherwise it takes the exact form
  uint32_t q60 = 0;
};
hipError_t keyswitch_rotate_batch(const KsRotateBatchArgs& a, size_t n, hipStream_t s);
// keyswitch_rotate_batch of `count` (2..kKsGroupMax) ciphertexts at one level through the same entries (keys)
// in one launch, the ciphertexts' workgroups of a (limb, source block) on one XCD so that the keys
// are read from HBM about once for all; a[0..count) differ only in digits / ct / out.  Each result
// equals its own keyswitch_rotate_batch, bit for bit.
struct KsRotateBatchGroupArgs {
  KsRotateBatchArgs a[kKsGroupMax];
  int count = 1;
};
hipError_t keyswitch_rotate_batch_group(const KsRotateBatchGroupArgs& ga, size_t n, hipStream_t s);

struct GaloisFinishArgs {
  const uint64_t* cx;
  const uint64_t* c0;
  const uint64_t* pmod;
  const uint64_t* pmod_shoup;
  uint64_t* out;
  const uint32_t* perm;
  const uint64_t* q;
  uint32_t ql = 0, qlp = 0;
  bool accumulate = false;
};
hipError_t galois_finish(const GaloisFinishArgs& a, int mode, size_t n, hipStream_t s);

// ---- bootstrap helpers ----------------------------------------------------------------
// switchModulusKernel (src/evaluate.cu:2414-2457): lift limb-0 coefficients (mod q0) to L limbs
hipError_t switch_modulus_raise(const uint64_t* in_q0, uint64_t* out, const uint64_t* q, const uint64_t* barrett,
                                size_t n, size_t L, hipStream_t s);

}  // namespace phx
