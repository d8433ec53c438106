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

}  // namespace phx
