// arith.h — 64-bit modular arithmetic for gfx950 (CDNA4) device code.
//
// gfx950 has no 64x64-bit multiplier: every 64-bit product is built from
// v_mad_u64_u32 / v_mul_hi_u32 / v_mul_lo_u32, each a half-rate instruction
// (≈4.3 cycles per wave64 instruction per SIMD, measured with tools/ubench_isa.hip),
// so the helpers below are written to minimise those instructions.
//
// Semantics follow the reference's device arithmetic (include/uintmodmath.cuh:18-242,
// include/butterfly.cuh:10-37): Shoup products with precomputed w' = floor(w 2^64 / q)
// and lazy ranges, Barrett reduction of 128-bit values with floor(2^128 / q).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace phx {

struct u128 {
  uint64_t lo, hi;
};

__device__ __forceinline__ uint32_t lo32(uint64_t x) { return static_cast<uint32_t>(x); }
__device__ __forceinline__ uint32_t hi32(uint64_t x) { return static_cast<uint32_t>(x >> 32); }

// full 64x64 -> 128 product from four 32x32 partial products (v_mad_u64_u32 chain)
__device__ __forceinline__ u128 mul_wide(uint64_t a, uint64_t b) {
  const uint64_t ll = static_cast<uint64_t>(lo32(a)) * lo32(b);
  const uint64_t lh = static_cast<uint64_t>(lo32(a)) * hi32(b) + hi32(ll);
  const uint64_t hl = static_cast<uint64_t>(hi32(a)) * lo32(b) + lo32(lh);
  const uint64_t hh = static_cast<uint64_t>(hi32(a)) * hi32(b) + hi32(lh) + hi32(hl);
  u128 r;
  r.lo = (static_cast<uint64_t>(lo32(hl)) << 32) | lo32(ll);
  r.hi = hh;
  return r;
}

// high 64 bits of a 64x64 product
__device__ __forceinline__ uint64_t mulhi(uint64_t a, uint64_t b) { return __umul64hi(a, b); }

__device__ __forceinline__ uint64_t csub(uint64_t x, uint64_t m) {
  const uint64_t t = x - m;
  return static_cast<int64_t>(t) < 0 ? x : t;
}

__device__ __forceinline__ uint64_t add_mod(uint64_t a, uint64_t b, uint64_t q) { return csub(a + b, q); }
__device__ __forceinline__ uint64_t sub_mod(uint64_t a, uint64_t b, uint64_t q) { return csub(a + q - b, q); }
__device__ __forceinline__ uint64_t neg_mod(uint64_t a, uint64_t q) { return a ? q - a : 0; }

// Shoup product, lazy: returns a*w mod q in [0, 2q) for any a < 2^64, w < q.
__device__ __forceinline__ uint64_t mul_shoup_lazy(uint64_t a, uint64_t w, uint64_t ws, uint64_t q) {
  return a * w - mulhi(a, ws) * q;
}

// Shoup product, fully reduced to [0, q).
__device__ __forceinline__ uint64_t mul_shoup(uint64_t a, uint64_t w, uint64_t ws, uint64_t q) {
  return csub(mul_shoup_lazy(a, w, ws, q), q);
}

// Barrett reduction of a 128-bit value x < 2^128 with ratio = floor(2^128 / q) = {r0, r1}.
// The quotient estimate floor(x * ratio / 2^128) is at most one below floor(x / q), so one
// conditional subtraction gives the canonical residue (as include/uintmodmath.cuh:206-246).
__device__ __forceinline__ uint64_t barrett_reduce_128(u128 x, uint64_t q, uint64_t r0, uint64_t r1) {
  // floor((x.hi 2^64 + x.lo)(r1 2^64 + r0) / 2^128) mod 2^64
  const uint64_t p0 = mulhi(x.lo, r0);
  const u128 p1 = mul_wide(x.lo, r1);
  const u128 p2 = mul_wide(x.hi, r0);
  uint64_t mid = p1.lo + p0;
  uint64_t carry = mid < p0;
  uint64_t mid2 = mid + p2.lo;
  carry += mid2 < mid;
  const uint64_t quot = x.hi * r1 + p1.hi + p2.hi + carry;
  return csub(x.lo - quot * q, q);
}

// Barrett reduction of a 64-bit value with r1 = floor(2^64 / q) (uintmodmath.cuh:254-261)
__device__ __forceinline__ uint64_t barrett_reduce_64(uint64_t x, uint64_t q, uint64_t r1) {
  return csub(x - mulhi(x, r1) * q, q);
}

// ---- 30-bit split accumulation: sum_i x_i y_i = LL + MM 2^30 + HH 2^60 with x = xh 2^30 + xl and
// y = yh 2^30 + yl (x, y < 2^60), every partial product below 2^60, reduced once at the end ----
struct SplitRed {
  uint64_t c30, c30s, c60, c60s;  // 2^30 mod q, 2^60 mod q and their Shoup quotients
  uint64_t nq, nq2, nq4;          // -q, -2q, -4q mod 2^64
};
// floor(w 2^64 / q) for w < q from the Barrett ratio floor(2^128 / q) = {r0, r1} (an estimate at
// most 2 low, corrected exactly)
__device__ __forceinline__ uint64_t shoup_from_barrett(uint64_t w, uint64_t q, uint64_t r0, uint64_t r1) {
  uint64_t s = w * r1 + mulhi(w, r0);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    // remainder w 2^64 - s q (< 3q, so its high word is 0 or 1)
    const u128 p = mul_wide(s, q);
    const uint64_t rlo = 0 - p.lo, rhi = w - p.hi - (p.lo != 0);
    if (rhi != 0 || rlo >= q) ++s;
  }
  return s;
}
// a uniform 64-bit value in scalar registers (every lane holds the same value)
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}
// the constants of one modulus, for a workgroup-uniform q (kept in scalar registers)
__device__ __forceinline__ SplitRed split_red(uint64_t q, uint64_t r0, uint64_t r1) {
  SplitRed k;
  k.c30 = uniform_u64((1ull << 30) % q);
  k.c60 = uniform_u64((1ull << 60) % q);
  k.c30s = uniform_u64(shoup_from_barrett(k.c30, q, r0, r1));
  k.c60s = uniform_u64(shoup_from_barrett(k.c60, q, r0, r1));
  k.nq = uniform_u64(0 - q);
  k.nq2 = uniform_u64(0 - (q << 1));
  k.nq4 = uniform_u64(0 - (q << 2));
  return k;
}

// split_reduce (below) with exact high products, for q < 2^61: three lazy residues in [0, 2q), their
// sum below 6q < 2^64, one more Barrett step and one conditional subtraction.  More instructions,
// fewer registers.
__device__ __forceinline__ uint64_t split_reduce_exact(uint64_t ll, uint64_t mm, uint64_t hh, const SplitRed& k,
                                                       uint64_t q, uint64_t r1) {
  const uint64_t a = ll - mulhi(ll, r1) * q;
  const uint64_t b = mm * k.c30 - mulhi(mm, k.c30s) * q;
  const uint64_t c = hh * k.c60 - mulhi(hh, k.c60s) * q;
  const uint64_t s = a + b + c;
  return csub(s - mulhi(s, r1) * q, q);
}

__device__ __forceinline__ uint64_t mul_mod(uint64_t a, uint64_t b, uint64_t q, uint64_t r0, uint64_t r1) {
  return barrett_reduce_128(mul_wide(a, b), q, r0, r1);
}

__device__ __forceinline__ void add128(u128& acc, u128 v) {
  acc.lo += v.lo;
  acc.hi += v.hi + (acc.lo < v.lo);
}

// Cooley-Tukey butterfly (include/butterfly.cuh:10-22): inputs in [0, 4q), outputs in [0, 4q).
__device__ __forceinline__ void ct_bfly(uint64_t& x, uint64_t& y, uint64_t w, uint64_t ws, uint64_t q) {
  const uint64_t q2 = q << 1;
  const uint64_t t = mul_shoup_lazy(y, w, ws, q);
  const uint64_t u = csub(x, q2);
  x = u + t;
  y = u + q2 - t;
}

// Gentleman-Sande butterfly (include/butterfly.cuh:28-37): inputs in [0, 2q), outputs in [0, 2q).
__device__ __forceinline__ void gs_bfly(uint64_t& x, uint64_t& y, uint64_t w, uint64_t ws, uint64_t q) {
  const uint64_t q2 = q << 1;
  const uint64_t d = x + q2 - y;
  x = csub(x + y, q2);
  y = mul_shoup_lazy(d, w, ws, q);
}

// ---------------------------------------------------------------------------------------
// NTT butterflies for the 2-D kernels' integer path (primes q < 2^61; MOD_BIT_COUNT_MAX = 61,
// include/host/defines.h:4), with an approximate Shoup quotient.
//
// a ws = a1 s1 2^64 + (a1 s0 + a0 s1) 2^32 + a0 s0 (32-bit halves), so
//   floor(a ws / 2^64) - [a1 s1 + hi(a1 s0) + hi(a0 s1)]  in {0, 1, 2}:
// dropping a0 s0 and the low halves of the cross products loses less than 3 * 2^32 below 2^64.
// Three multiplies instead of four, and the remainder a w - Q' q lies in [0, 4q) instead of
// [0, 2q).  The butterflies keep the reference's structure (include/butterfly.cuh:10-37) with
// the lazy ranges doubled: CT values in [0, 8q), GS values in [0, 4q); 8q < 2^64.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mulhi_approx(uint64_t a, uint64_t s) {
  const uint32_t a0 = lo32(a), a1 = hi32(a), s0 = lo32(s), s1 = hi32(s);
  const uint64_t h = static_cast<uint64_t>(__umulhi(a1, s0)) + __umulhi(a0, s1);
  return static_cast<uint64_t>(a1) * s1 + h;
}

// Carry-free forms.  A 64-bit subtraction compiles to v_sub_co / v_subb_co with the borrow in
// VCC, and gfx950 needs wait states (s_nop) between the VCC write and the VCC read; a csub adds
// a 64-bit compare and two v_cndmask behind another VCC hazard.  Here every constant subtraction
// is an addition of the negated constant in one v_lshl_add_u64 (shift 0), and csub selects with
// a sign mask (ashr + and) instead of VCC.  Same integers, so bit-identical results.
__device__ __forceinline__ uint64_t add64(uint64_t a, uint64_t b) {
  uint64_t r;
  asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// hides that v is a negation, so x + v is not canonicalised back into a subtraction
__device__ __forceinline__ uint64_t opaque(uint64_t v) {
  asm("" : "+v"(v));
  return v;
}
// x - m if that is >= 0 else x, for x, m < 2^63, given nm = -m mod 2^64.  t = x - m, s = its sign
// as a 32-bit mask, then the select (s & x) | (~s & t) as one v_bfi_b32 per half: 4 instructions
// (the masked add-back form, t + (m & s), takes 5).
__device__ __forceinline__ uint64_t csub_n(uint64_t x, uint64_t m, uint64_t nm) {
  const uint64_t t = add64(x, nm);
  const uint32_t s = static_cast<uint32_t>(static_cast<int32_t>(hi32(t)) >> 31);
  (void)m;
  uint32_t lo, hi;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(lo) : "v"(s), "v"(lo32(x)), "v"(lo32(t)));
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(hi) : "v"(s), "v"(hi32(x)), "v"(hi32(t)));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}
// a w mod q in [0, 4q) (as mul_shoup_lazy4 below), given nq = -q mod 2^64: a w + Q' (-q)
__device__ __forceinline__ uint64_t mul_shoup_lazy4(uint64_t a, uint64_t w, uint64_t ws, uint64_t q) {
  return a * w + mulhi_approx(a, ws) * opaque(0 - q);
}

// (ll + mm 2^30 + hh 2^60) mod q for q < 2^60 (the lazy sum below 12q must fit 64 bits), canonical (SplitRed above; r1 = floor(2^64 / q), the
// high word of the Barrett ratio).  Three lazy residues with the approximate quotient (mulhi_approx,
// at most 2 low): a 64-bit Barrett step on ll and Shoup products for mm 2^30 and hh 2^60, each in
// [0, 4q); their sum below 12q < 2^64; one more Barrett step to [0, 4q) and two carry-free
// conditional subtractions.  No VCC carries and no zero-extended 64-bit high products.
__device__ __forceinline__ uint64_t split_reduce(uint64_t ll, uint64_t mm, uint64_t hh, const SplitRed& k, uint64_t q,
                                                 uint64_t r1) {
  const uint64_t nq = k.nq;
  const uint64_t a = ll + mulhi_approx(ll, r1) * nq;
  const uint64_t b = mm * k.c30 + mulhi_approx(mm, k.c30s) * nq;
  const uint64_t c = hh * k.c60 + mulhi_approx(hh, k.c60s) * nq;
  uint64_t s = add64(add64(a, b), c);
  s = s + mulhi_approx(s, r1) * nq;
  s = csub_n(s, q << 1, k.nq2);
  return csub_n(s, q, nq);
}

// split_reduce with the three partial sums folded into two first: L = ll + (mm mod 2^30) 2^30 and
// H = hh + floor(mm / 2^30), both below 2^63 (ll, hh < 2^62 and mm < 2^63 for BETA <= 4), so the
// value is L + H 2^60.  A 64-bit Barrett step on L and a Shoup product H (2^60 mod q), each in
// [0, 4q) with approximate quotients, their sum below 8q < 2^63 and three carry-free conditional
// subtractions: 15 multiplies instead of 30.  q < 2^60.
__device__ __forceinline__ uint64_t split_reduce2(uint64_t ll, uint64_t mm, uint64_t hh, const SplitRed& k, uint64_t q,
                                                  uint64_t r1) {
  constexpr uint64_t kM30 = (1ull << 30) - 1;
  const uint64_t nq = k.nq;
  const uint64_t L = add64(ll, (mm & kM30) << 30);
  const uint64_t H = add64(hh, mm >> 30);
  const uint64_t a = L + mulhi_approx(L, r1) * nq;
  const uint64_t b = H * k.c60 + mulhi_approx(H, k.c60s) * nq;
  uint64_t s = add64(a, b);
  s = csub_n(s, q << 2, k.nq4);
  s = csub_n(s, q << 1, k.nq2);
  return csub_n(s, q, nq);
}

// forward CT butterfly: x, y in [0, 8q) -> [0, 8q)
__device__ __forceinline__ void ct_bfly8(uint64_t& x, uint64_t& y, uint64_t w, uint64_t ws, uint64_t q) {
  const uint64_t q4 = q << 2;
  const uint64_t t = mul_shoup_lazy4(y, w, ws, q);
  const uint64_t u = csub_n(x, q4, opaque(0 - q4));
  x = add64(u, t);
  y = u + q4 - t;
}

// inverse GS butterfly: x, y in [0, 4q) -> [0, 4q)
__device__ __forceinline__ void gs_bfly4(uint64_t& x, uint64_t& y, uint64_t w, uint64_t ws, uint64_t q) {
  const uint64_t q4 = q << 2;
  const uint64_t d = x + q4 - y;
  x = csub_n(add64(x, y), q4, opaque(0 - q4));
  y = mul_shoup_lazy4(d, w, ws, q);
}

// inverse GS butterfly for q < 2^60 with inputs below 8q: d = x + 8q - y < 16q < 2^64 and
// x' = x + y < 16q, brought below 8q only when RED (ntt.hip lazy_gs decides per element)
template <bool RED>
__device__ __forceinline__ void gs_bfly8(uint64_t& x, uint64_t& y, uint64_t w, uint64_t ws, uint64_t q) {
  const uint64_t q8 = q << 3;
  const uint64_t d = x + q8 - y;
  const uint64_t s = add64(x, y);
  x = RED ? csub_n(s, q8, opaque(0 - q8)) : s;
  y = mul_shoup_lazy4(d, w, ws, q);
}

// [0, 8q) -> [0, q)
__device__ __forceinline__ uint64_t reduce8(uint64_t v, uint64_t q) {
  v = csub_n(v, q << 2, opaque(0 - (q << 2)));
  v = csub_n(v, q << 1, opaque(0 - (q << 1)));
  return csub_n(v, q, opaque(0 - q));
}

// ---- primes q < 2^60: lazy range up to 16q (< 2^64) --------------------------------------
// The forward butterfly reduces x only every other stage (LazyCT below): without the
// reduction x, y < R q -> x + t, x + 4q - t < (R + 4) q; with it (x -= 8q if x >= 8q) the
// outputs are < 12q.  Half the conditional subtractions of ct_bfly8, same integers.
// no reduction of x: x, y < R q with R <= 12 -> outputs < (R + 4) q <= 16 q
__device__ __forceinline__ void ct_bfly_nored(uint64_t& x, uint64_t& y, uint64_t w, uint64_t ws, uint64_t q) {
  const uint64_t t = mul_shoup_lazy4(y, w, ws, q);
  y = x + (q << 2) - t;
  x = add64(x, t);
}
// x < 16q reduced below 8q first: outputs < 12q
__device__ __forceinline__ void ct_bfly_c8(uint64_t& x, uint64_t& y, uint64_t w, uint64_t ws, uint64_t q) {
  const uint64_t q8 = q << 3;
  const uint64_t t = mul_shoup_lazy4(y, w, ws, q);
  const uint64_t u = csub_n(x, q8, opaque(0 - q8));
  x = add64(u, t);
  y = u + (q << 2) - t;
}
// [0, 16q) -> [0, q)
// v < 16q -> v mod q for 2^50 <= q < 2^60 with one conditional subtraction: the quotient
// estimate k = trunc(hi32(v) * rq - 1/4), rq = 2^32 / q in FP32, is floor(v / q) or one less (the
// FP32 error, < 4e-6, and the dropped low word, lo / q < 2^-18, stay inside the 1/4 margin), so
// v - k q lies in [0, 2q).  11 instructions where reduce16's four subtractions take 16.
__device__ __forceinline__ uint64_t reduce16_est(uint64_t v, uint64_t q, float rq) {
  float hf;  // (the compiler would widen a converted high word to a 64-bit conversion)
  asm("v_cvt_f32_u32 %0, %1" : "=v"(hf) : "v"(hi32(v)));
  const uint32_t k = static_cast<uint32_t>(__builtin_fmaxf(__builtin_fmaf(hf, rq, -0.25f), 0.0f));
  const uint64_t nq = opaque(0 - q);
  const uint64_t r = static_cast<uint64_t>(k) * lo32(nq) + v;  // v + k nq (mod 2^64): one v_mad_u64_u32 ...
  uint32_t kh;  // ... and the high word's k nq_hi (a plain multiply: fused into a 64-bit mad, it costs moves)
  asm("v_mul_lo_u32 %0, %1, %2" : "=v"(kh) : "v"(k), "v"(hi32(nq)));
  const uint32_t rh = hi32(r) + kh;
  return csub_n((static_cast<uint64_t>(rh) << 32) | lo32(r), q, nq);
}

__device__ __forceinline__ uint64_t reduce16(uint64_t v, uint64_t q) {
  v = csub_n(v, q << 3, opaque(0 - (q << 3)));
  return reduce8(v, q);
}

}  // namespace phx
