// ntt.h — negacyclic NTT / INTT over RNS limbs on gfx950.
//
// Replaces the reference's launcher family of include/ntt.cuh:157-226
// (nwt_2d_radix8_forward_inplace, nwt_2d_radix8_backward_inplace, the _scale,
// _include_special_mod, _exclude_range and out-of-place variants).
#pragma once

#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace phx {

// Device-resident NTT tables for a list of moduli (the reference's DNTTTable,
// include/ntt.cuh:36-129).  Layout [num_moduli][n] for every table.
struct NttTables {
  size_t n = 0;
  int log_n = 0;
  size_t num_moduli = 0;
  uint64_t* modulus = nullptr;   // [num_moduli]
  uint64_t* barrett = nullptr;   // [num_moduli][2] floor(2^128/q) {lo, hi}
  uint64_t* tw = nullptr;        // tw[brv(i)] = psi^i
  uint64_t* tw_shoup = nullptr;
  uint64_t* itw = nullptr;       // itw[brv(i)] = psi^-i (n^-1 NOT folded in; applied separately)
  uint64_t* itw_shoup = nullptr;
  uint64_t* n_inv = nullptr;     // [num_moduli]
  uint64_t* n_inv_shoup = nullptr;
  // FP64 path (farith.h), used for q < 2^50.  All twiddles are centered doubles (|w| <= q/2).
  double* modulus_f = nullptr;   // [num_moduli] q
  double* modulus_inv = nullptr; // [num_moduli] fl(1/q)
  double* col_fwd = nullptr;     // [num_moduli][S1] tw[0..S1): the column-pass (first log2 S1) stages
  double* col_inv = nullptr;     // [num_moduli][S1] itw[0..S1) with [1] = itw[1] n^-1 and [0] = n^-1
  // row-pass twiddles factored as tw[(S1 + row) 2^g + iloc] = A_g(row) * B_g(iloc) (see ntt.hip)
  double* row_a_fwd = nullptr;   // [num_moduli][S1][16]: A_g(row) for row-pass stage g
  double* row_b_fwd = nullptr;   // [num_moduli][S2]: B_g(iloc) at index 2^g + iloc
  double* row_a_inv = nullptr;   // the same factors of itw (inverses of the forward ones)
  double* row_b_inv = nullptr;
  bool lazy16 = false;           // every modulus < 2^60: forward integer passes use the 16q lazy range
  bool int_only = false;         // every modulus >= 2^50: no limb takes the FP64 path
};

// log2 of the column-pass size S1 for a given log2(n) (the row pass handles the rest)
inline int ntt_split_log_s1(int log_n) { return log_n / 2; }

// Which table row each buffer limb uses.  Buffer limb i (0 <= i < num_limbs) maps to
// table row (i < split ? first_a + i : first_b + (i - split)); limbs in
// [skip_begin, skip_end) are left untouched (the reference's exclude_range).
//
// Batching: `polys` polynomials of the same shape go through one launch.  Polynomial p starts
// at in + p * in_stride / out + p * out_stride (elements; 0 = num_limbs * n, i.e. contiguous)
// and skips [skip_begin + p * skip_step, skip_end + p * skip_step) — the modup digits.
// Grouped batches (period > 0): polynomial p = g * period + j starts at g * in_outer + j * in_stride
// (out likewise) and skips by j only — the digits of several key switches' modups in one launch.
struct LimbMap {
  int num_limbs = 0;
  int split = 0;
  int first_a = 0;
  int first_b = 0;
  int skip_begin = 0;
  int skip_end = 0;
  int polys = 1;
  int skip_step = 0;
  size_t in_stride = 0;
  size_t out_stride = 0;
  int period = 0;
  size_t in_outer = 0;
  size_t out_outer = 0;
  __host__ __device__ int skip_index(int p) const { return period > 0 ? p % period : p; }
  __host__ __device__ size_t in_off(int p) const {
    return period > 0 ? (size_t)(p / period) * in_outer + (size_t)(p % period) * in_stride : (size_t)p * in_stride;
  }
  __host__ __device__ size_t out_off(int p) const {
    return period > 0 ? (size_t)(p / period) * out_outer + (size_t)(p % period) * out_stride : (size_t)p * out_stride;
  }
  static LimbMap contiguous(int num_limbs, int first) {
    LimbMap m;
    m.num_limbs = num_limbs; m.split = num_limbs; m.first_a = first; m.first_b = 0;
    return m;
  }
  // `polys` polynomials with the given element strides (0: contiguous)
  LimbMap batched(int count, size_t in_s = 0, size_t out_s = 0) const {
    LimbMap m = *this;
    m.polys = count; m.in_stride = in_s; m.out_stride = out_s;
    return m;
  }
  // `count` polynomials in groups of `per` (see above)
  LimbMap grouped(int count, int per, size_t stride, size_t outer) const {
    LimbMap m = *this;
    m.polys = count; m.period = per;
    m.in_stride = m.out_stride = stride;
    m.in_outer = m.out_outer = outer;
    return m;
  }
};

// Forward NTT, out-of-place allowed (out may equal in).  Output fully reduced, bit-reversed
// order (A[i] = a(psi^(2 brv(i) + 1))), identical to nwt_2d_radix8_forward_inplace.
hipError_t ntt_forward(const NttTables& t, const uint64_t* in, uint64_t* out, const LimbMap& map,
                       hipStream_t stream);

// Forward NTT with a fused prologue and epilogue (the rescale and moddown tails):
//  - prologue (bcast != null): buffer limb i of polynomial p is read as bcast[p][k] mod q_row,
//    one coefficient-form limb broadcast over the limbs (`in` is not read): divide_and_round's
//    spread of the last limb (src/rns.cu:1128-1139);
//  - epilogue (epi.out != null): the transform's value y is not stored; instead
//    epi.out[p][i][k] = (epi.c[p][i][k] - y) * w[i] (+ epi.out[p][i][k] when accumulate), mod q:
//    the rescale / moddown finish (src/rns.cu:1141-1158, src/ntt/ntt_moddown.cu:199-214).
// Polynomial p of c / out starts at p * c_stride / p * out_stride (elements).
//  - key-switch form (ks_beta > 0, the moddown of a key switch): c is not read; its value is the
//    key-switch inner product of the Ql limbs formed in the epilogue,
//      c[p][i][k] = sum_{d < ks_beta} tmu[d][i][k] * evk[d][p][i][k]  mod q_i
//    (src/eval_key_switch.cu:26-85 for limbs i < size_Ql), so the inner product's Ql half never
//    makes an HBM round trip (tmu: digit stride tmu_stride; evk: device array of ks_beta digit
//    pointers, polynomial stride evk_poly_stride; the buffer limbs must be the first Ql limbs).
//  - several ciphertexts in one launch (ks_prods > 1, polys = 2 ks_prods): polynomial p is c(p % 2)
//    of ciphertext k = p / 2, written to out_p[k] + (p % 2) out_stride (any epilogue); in the
//    key-switch form its tmu starts at tmu + k tmu_prod_stride and its addend at add_p[k] (+ (p % 2)
//    add_stride), the key shared.  ks_prods <= 1 uses out / add_c.
constexpr int kMaxKsBeta = 3;  // digits of the key-switch form (C3: 3, the C4 chain: <= 3)
constexpr int kMaxKsProds = 16;
struct NttEpilogue {
  const uint64_t* c = nullptr;
  size_t c_stride = 0;
  uint64_t* out = nullptr;
  size_t out_stride = 0;
  const uint64_t* w = nullptr;   // per buffer limb
  const uint64_t* ws = nullptr;  // Shoup quotients
  bool accumulate = false;
  int ks_beta = 0;
  const uint64_t* tmu = nullptr;
  size_t tmu_stride = 0;
  const uint64_t* const* evk = nullptr;
  size_t evk_poly_stride = 0;
  // optional addend of the key-switch form (rns.h KsAddend): c[p][i][k] += P_i * add_c[p][i][k]
  // (add_c polynomial stride add_stride), the P-scaled (c0, c1) of a relinearize + rescale
  const uint64_t* add_c = nullptr;
  size_t add_stride = 0;
  const uint64_t* pmod = nullptr;
  const uint64_t* pmod_shoup = nullptr;
  // inverse prologue only (ntt_inverse_ks): tmu limb of buffer limb 0, and how many leading buffer
  // limbs take the addend
  size_t tmu_limb0 = 0;
  int add_limbs = 0;
  // batched key switches (see above)
  int ks_prods = 1;
  size_t tmu_prod_stride = 0;
  uint64_t* out_p[kMaxKsProds] = {};
  const uint64_t* add_p[kMaxKsProds] = {};
  __host__ __device__ uint64_t* ks_out(int p) const {
    return (ks_prods > 1 ? out_p[p >> 1] : out) + (size_t)(ks_prods > 1 ? (p & 1) : p) * out_stride;
  }
  __host__ __device__ const uint64_t* ks_add(int p) const {
    return (ks_prods > 1 ? add_p[p >> 1] : add_c) + (size_t)(ks_prods > 1 ? (p & 1) : p) * add_stride;
  }
  __host__ __device__ const uint64_t* ks_tmu(int p) const { return tmu + (size_t)(p >> 1) * tmu_prod_stride; }
};
hipError_t ntt_forward_fused(const NttTables& t, const uint64_t* in, uint64_t* out, const LimbMap& map,
                             const uint64_t* bcast, size_t bcast_stride, const NttEpilogue& epi, hipStream_t stream);

// Forward NTT whose input is a fast base conversion (src/rns_bconv.cu:40-69, 143-179): buffer
// limb i of polynomial p (processed index j = i minus the limbs of p's exclude range below it) is
//   x[k] = sum_{s < ib[p]} in[p][s][k] * mat[p][s * ob + j]  mod q_row,
// computed in the column pass's registers from the ib input limbs (coefficient form, already
// multiplied by qHat_s^-1 — the INTT's scale), so the converted limbs never go to HBM.  It
// replaces bconv + NTT in modup (per digit: the complement limbs), moddown (P -> Ql) and
// moddown-rescale; `epi` is the NttEpilogue above.  Inputs and matrix entries < 2^60, ib <= 15
// (30-bit split sums).  2-D sizes only (n >= 2^10): hipErrorNotSupported below.
constexpr int kMaxBconvPolys = 8;
struct BconvPrologue {
  const uint64_t* in = nullptr;   // polynomial p's input limb s at in + p * in_stride + s * n
  size_t in_stride = 0;
  const uint64_t* mat[kMaxBconvPolys] = {};  // [ib][ob] per polynomial
  int ib[kMaxBconvPolys] = {};
  int ob = 0;
};
hipError_t ntt_forward_bconv(const NttTables& t, uint64_t* out, const LimbMap& map, const BconvPrologue& bcv,
                             const NttEpilogue& epi, hipStream_t stream);

// Inverse NTT.  When scale/scale_shoup are given (one value per buffer limb, indexed by
// buffer limb), the output is additionally multiplied by scale[i] (the reference's
// nwt_2d_radix8_backward_scale used by modup, src/ntt/ntt_modup.cu:356-393).
hipError_t ntt_inverse(const NttTables& t, const uint64_t* in, uint64_t* out, const LimbMap& map,
                       const uint64_t* scale, const uint64_t* scale_shoup, hipStream_t stream);

// Inverse NTT whose input is the key-switch inner product of the moddown's dropped limbs (the P
// limbs, plus q_last for a relinearize + rescale): buffer limb i of polynomial p (table row r) is
//   x[k] = sum_{d < ks_beta} tmu[d][tmu_limb0 + i][k] * evk[d][p][r][k]
//          (+ P_r * add_c[p][tmu_limb0 + i][k] for i < add_limbs)  mod q_r
// (src/eval_key_switch.cu:26-85 for those limbs) formed in the first pass's registers, so the
// inner product's dropped half makes no HBM round trip either.  There is no `in`; `ks` carries
// ks_beta, tmu, tmu_stride, evk, evk_poly_stride, tmu_limb0 and the optional addend (add_c,
// add_stride, pmod / pmod_shoup indexed by tmu_limb0 + i).  2-D sizes (n >= 2^10) only.
hipError_t ntt_inverse_ks(const NttTables& t, uint64_t* out, const LimbMap& map, const uint64_t* scale,
                          const uint64_t* scale_shoup, const NttEpilogue& ks, hipStream_t stream);

// Inverse NTT that also copies its (NTT-form) input: the first pass stores every loaded input
// limb l (buffer limb index) unchanged at copy + (l / alpha) * digit_stride + l * n as well.  This
// is modup's modup_copy_partQl_kernel (src/rns_bconv.cu:522-528) folded into its INTT
// (nwt_2d_radix8_backward_scale): the copy no longer re-reads c2.  2-D sizes (n >= 2^10) only.
struct NttCopy {
  uint64_t* out = nullptr;
  size_t digit_stride = 0;  // elements between digits
  int alpha = 1;            // limbs per digit
  size_t poly_stride = 0;   // batched inverses: polynomial p's digits start at out + p * poly_stride
};
hipError_t ntt_inverse_copy(const NttTables& t, const uint64_t* in, uint64_t* out, const LimbMap& map,
                            const uint64_t* scale, const uint64_t* scale_shoup, const NttCopy& copy,
                            hipStream_t stream);

// The 1-D radix-2 path (fnwt_1d / inwt_1d, include/ntt.cuh:157-169, src/ntt/ntt_1d.cu): one
// workgroup per limb, the limb in LDS; n = 2^3 .. 2^11.  ntt_forward / ntt_inverse use it for
// n < 2^10; these entry points force it (the reference's test_nwt_1d covers n = 2^8 .. 2^11).
hipError_t ntt_1d_forward(const NttTables& t, uint64_t* inout, const LimbMap& map, hipStream_t stream);
hipError_t ntt_1d_inverse(const NttTables& t, uint64_t* inout, const LimbMap& map, const uint64_t* scale,
                          const uint64_t* scale_shoup, hipStream_t stream);

}  // namespace phx
