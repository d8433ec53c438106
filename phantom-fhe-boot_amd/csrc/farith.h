// farith.h — exact modular arithmetic in IEEE double precision for primes q < 2^50.
//
// gfx950 issues v_fma_f64 / v_mul_f64 / v_rndne_f64 at the same half rate as the
// 32-bit integer multiplies (≈4.3 cycles per wave64 instruction per SIMD, measured with
// tools/ubench_isa.hip), but a modular product needs 6 FP64 instructions instead of ~10
// integer multiplies plus carries, so the NTT butterfly costs roughly half as much.
// Results are exact integers: every value is an integer of magnitude < 2^53.
//
// modmul(y, w) for q < 2^50, |y| <= 4q, |w| <= q/2 (the exactness argument):
//   h = fl(y w)                 |y w| <= 2q^2 < 2^101, |h - y w| <= 2q^2 2^-53 < q/4
//   l = fma(y, w, -h)           = y w - h exactly (the error of a product is representable)
//   k = rint(fl(h * qinv))      |fl(h qinv) - y w/q| <= 1/4 + 2q * 2^-52 <= 3/4, |k - y w/q| <= 5/4
//   r = fma(-k, q, h)           = h - k q exactly (|h - k q| <= q/4 + 5q/4 < 2^53)
//   t = r + l                   = y w - k q exactly, |t| <= 1.25 q
// so t ≡ y w (mod q) with |t| <= 1.25q.  A Cooley-Tukey stage grows |x| by at most 1.25q, so
// starting from |x| < q three stages stay within y-inputs <= 3.5q and outputs <= 4.75q;
// ntt.hip reduces every value back to |x| <= q/2 + 1 before every third stage.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace phx {

__device__ __forceinline__ double fmodmul(double y, double w, double q, double qinv) {
  const double h = y * w;
  const double l = __builtin_fma(y, w, -h);
  const double k = __builtin_rint(h * qinv);
  const double r = __builtin_fma(-k, q, h);
  return r + l;
}

// centered reduction: |v| < 2^53 -> v' ≡ v (mod q), |v'| <= q/2 + 1
__device__ __forceinline__ double freduce(double v, double q, double qinv) {
  return __builtin_fma(-__builtin_rint(v * qinv), q, v);
}

// 2^52 magic: for 0 <= x < 2^52, bits(double(2^52) + x) = bits(2^52) + x
constexpr uint64_t kMagicBits = 0x4330000000000000ull;
constexpr double kMagic = 4503599627370496.0;  // 2^52

__device__ __forceinline__ double u64_to_f64(uint64_t x) {  // x < 2^52
  return __longlong_as_double(static_cast<long long>(x + kMagicBits)) - kMagic;
}

// any exact integer |v| < 2^53 -> canonical residue in [0, q)
__device__ __forceinline__ uint64_t f64_to_canonical(double v, double q, double qinv) {
  double r = freduce(v, q, qinv);  // |r| <= q/2 + 1
  r = r < 0.0 ? r + q : r;
  r = r >= q ? r - q : r;
  return static_cast<uint64_t>(__double_as_longlong(r + kMagic)) - kMagicBits;
}

__device__ __forceinline__ uint64_t as_bits(double v) { return static_cast<uint64_t>(__double_as_longlong(v)); }
__device__ __forceinline__ double as_f64(uint64_t b) { return __longlong_as_double(static_cast<long long>(b)); }

}  // namespace phx
