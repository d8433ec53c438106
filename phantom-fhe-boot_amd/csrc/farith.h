// farith.h — exact modular arithmetic in IEEE double precision for primes q < 2^50.
//
// gfx950 issues v_fma_f64 / v_mul_f64 / v_rndne_f64 at the same rate as the 32-bit integer
// multiplies (≈4.3 cycles per wave64 instruction per SIMD, profiles/r01/ubench_isa.txt), but a
// modular product needs 6 FP64 instructions instead of ~10 integer multiplies plus carries, so
// an NTT butterfly costs well under half of the 64-bit integer Shoup butterfly.  All values are
// exact integers of magnitude < 2^53; the results are the same residues the integer path gives.
//
// fmodmul(y, w), q < 2^50 (u = 2^-53, |y| = Y q, |w| = W q):
//   h = fl(y w)                 |h - y w| <= u |y w|
//   l = fma(y, w, -h)           = y w - h exactly (the rounding error of a product is representable)
//   k = rint(fl(h * qinv))      |fl(h qinv) - y w / q| <= 3u |y w| / q  (first order; qinv = fl(1/q))
//   r = fma(-k, q, h)           = h - k q exactly (an integer below 2^53 in magnitude)
//   t = r + l                   = y w - k q exactly
// so t ≡ y w (mod q) and |t| <= q/2 + 3u Y W q^2 <= q (1/2 + (3/8) Y W) because q < 2^50.
// The kernels keep every stored value below 7.75 q < 2^53 and reduce (freduce: |v'| <= q/2 + 1)
// at compile-time-chosen stages; `Bound` below is that bookkeeping (units of q, with margin).
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

__device__ __forceinline__ uint64_t as_bits(double v) { return static_cast<uint64_t>(__double_as_longlong(v)); }
__device__ __forceinline__ double as_f64(uint64_t b) { return __longlong_as_double(static_cast<long long>(b)); }

// x < 2^52 -> double: OR the exponent into the high word (no carry possible), subtract 2^52
__device__ __forceinline__ double u52_to_f64(uint64_t x) {
  const uint32_t lo = static_cast<uint32_t>(x), hi = static_cast<uint32_t>(x >> 32) | 0x43300000u;
  return as_f64((static_cast<uint64_t>(hi) << 32) | lo) - kMagic;
}

// any exact integer |v| < 2^53 -> canonical residue in [0, q)
__device__ __forceinline__ uint64_t f64_to_canonical(double v, double q, double qinv) {
  double r = freduce(v, q, qinv);  // integer in [-q/2 - 1, q/2 + 1]
  r = r < 0.0 ? r + q : r;         // [0, q)
  const uint64_t b = as_bits(r + kMagic);
  return b & 0x000FFFFFFFFFFFFFull;  // mantissa = r (exponent bits of 2^52 masked off)
}

// Compile-time bound model (units of q).  prod(Y, W): bound of fmodmul output for inputs
// bounded by Y and twiddles bounded by W, with a margin for the +-1 terms.
struct Bound {
  static constexpr double kLimit = 7.75;    // every stored value stays below this
  static constexpr double kReduced = 0.51;  // after freduce
  static constexpr double prod(double Y, double W) { return 0.51 + 0.4 * Y * W; }
  // twiddles read from a table are reduced (|w| <= q/2); twiddles computed as an unreduced
  // product of two reduced factors are bounded by prod(0.5, 0.5)
  static constexpr double kTableW = 0.5;
  static constexpr double kGenW = 0.51 + 0.4 * 0.5 * 0.5;
};

}  // namespace phx
