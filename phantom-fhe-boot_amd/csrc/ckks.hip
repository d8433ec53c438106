// ckks.hip — sampling and small CKKS helper kernels (see ckks.h).
#include "ckks.h"

#include <algorithm>

#include "arith.h"

namespace phx {
namespace {

constexpr int kBlock = 256;

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// counter-based generator: word w of element i of stream (seed, sid)
__device__ __forceinline__ uint64_t rand_word(uint64_t seed, uint64_t sid, uint64_t i, uint32_t w) {
  return mix64(mix64(seed ^ (sid * 0x9E3779B97F4A7C15ull)) + (i * 4 + w) * 0xD1B54A32D192ED03ull);
}

__global__ __launch_bounds__(kBlock) void uniform_kernel(uint64_t* out, const uint64_t* q, const uint64_t* barrett,
                                                         uint32_t log_n, size_t total, uint64_t seed, uint64_t sid) {
  for (size_t e = blockIdx.x * (size_t)kBlock + threadIdx.x; e < total; e += (size_t)gridDim.x * kBlock) {
    const uint32_t l = static_cast<uint32_t>(e >> log_n);
    const u128 x{rand_word(seed, sid, e, 0), rand_word(seed, sid, e, 1)};
    out[e] = barrett_reduce_128(x, q[l], barrett[2 * l], barrett[2 * l + 1]);
  }
}

__global__ __launch_bounds__(kBlock) void cbd_kernel(uint64_t* out, const uint64_t* q, uint32_t log_n, size_t total,
                                                     uint64_t seed, uint64_t sid) {
  const size_t n = size_t(1) << log_n;
  for (size_t e = blockIdx.x * (size_t)kBlock + threadIdx.x; e < total; e += (size_t)gridDim.x * kBlock) {
    const uint32_t l = static_cast<uint32_t>(e >> log_n);
    const size_t k = e & (n - 1);
    const uint64_t r = rand_word(seed, sid, k, 0);  // same sample for every limb
    const int v = __popcll(r & 0x1FFFFFull) - __popcll((r >> 21) & 0x1FFFFFull);
    const uint64_t ql = q[l];
    out[e] = v >= 0 ? static_cast<uint64_t>(v) : ql - static_cast<uint64_t>(-v);
  }
}

__global__ __launch_bounds__(kBlock) void mul_scalar_add_kernel(const uint64_t* in, const uint64_t* c,
                                                                const uint64_t* cs, const uint64_t* acc, uint64_t* out,
                                                                const uint64_t* q, uint32_t log_n, size_t total) {
  for (size_t e = blockIdx.x * (size_t)kBlock + threadIdx.x; e < total; e += (size_t)gridDim.x * kBlock) {
    const uint32_t l = static_cast<uint32_t>(e >> log_n);
    const uint64_t ql = q[l];
    uint64_t v = mul_shoup(in[e], c[l], cs[l], ql);
    if (acc) v = add_mod(v, acc[e], ql);
    out[e] = v;
  }
}

template <int G>
__global__ __launch_bounds__(kBlock) void lt_bsgs_kernel(LtArgs a, uint32_t log_n, size_t total) {
  const size_t pstride = total;  // elements per polynomial ([Ql + P][n])
  for (size_t e = blockIdx.x * (size_t)kBlock + threadIdx.x; e < total; e += (size_t)gridDim.x * kBlock) {
    const int l = static_cast<int>(e >> log_n);
    const int row = l < a.Ql ? l : a.size_Q + (l - a.Ql);
    const uint64_t q = a.q[row], r0 = a.barrett[2 * row], r1 = a.barrett[2 * row + 1];
    uint64_t x0[G], x1[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      x0[j] = a.baby[j][e];
      x1[j] = a.baby[j][pstride + e];
    }
    for (int i = 0; i < a.b; ++i) {
      uint64_t* o = a.out[i];
      if (!o) continue;
      u128 acc0{0, 0}, acc1{0, 0};
#pragma unroll
      for (int j = 0; j < G; ++j) {
        const int u = G * i + j;
        if (u >= a.D) break;
        const uint64_t* p = a.pts[u];
        if (!p) continue;
        const uint64_t w = p[e];
        add128(acc0, mul_wide(x0[j], w));  // <= 32 products of 60-bit values: < 2^125
        add128(acc1, mul_wide(x1[j], w));
      }
      o[e] = barrett_reduce_128(acc0, q, r0, r1);
      o[pstride + e] = barrett_reduce_128(acc1, q, r0, r1);
    }
  }
}

template <bool MUL>
__global__ __launch_bounds__(kBlock) void scalar_v_kernel(const uint64_t* in, LimbScalars c, uint64_t* out,
                                                          const uint64_t* q, uint32_t log_n, size_t total) {
  for (size_t e = blockIdx.x * (size_t)kBlock + threadIdx.x; e < total; e += (size_t)gridDim.x * kBlock) {
    const uint32_t l = static_cast<uint32_t>(e >> log_n);
    const uint64_t ql = q[l];
    out[e] = MUL ? mul_shoup(in[e], c.v[l], c.vs[l], ql) : add_mod(in[e], c.v[l], ql);
  }
}

int grid_for(size_t items) {
  const size_t b = (items + kBlock - 1) / kBlock;
  return static_cast<int>(std::max<size_t>(1, std::min<size_t>(b, 2048)));
}

}  // namespace

hipError_t sample_uniform(uint64_t* out, const uint64_t* q, const uint64_t* barrett, size_t n, size_t L, uint64_t seed,
                          uint64_t stream_id, hipStream_t s) {
  const size_t total = n * L;
  uniform_kernel<<<grid_for(total), kBlock, 0, s>>>(out, q, barrett, __builtin_ctzll(n), total, seed, stream_id);
  return hipGetLastError();
}

hipError_t sample_cbd(uint64_t* out, const uint64_t* q, size_t n, size_t L, uint64_t seed, uint64_t stream_id,
                      hipStream_t s) {
  const size_t total = n * L;
  cbd_kernel<<<grid_for(total), kBlock, 0, s>>>(out, q, __builtin_ctzll(n), total, seed, stream_id);
  return hipGetLastError();
}

hipError_t mul_scalar_add(const uint64_t* in, const uint64_t* c, const uint64_t* c_shoup, const uint64_t* acc,
                          uint64_t* out, const uint64_t* q, size_t n, size_t L, hipStream_t s) {
  const size_t total = n * L;
  mul_scalar_add_kernel<<<grid_for(total), kBlock, 0, s>>>(in, c, c_shoup, acc, out, q, __builtin_ctzll(n), total);
  return hipGetLastError();
}

hipError_t lt_bsgs(const LtArgs& a, size_t n, hipStream_t s) {
  if (a.g < 1 || a.g > kLtMaxG || a.b < 1 || a.b > kLtMaxB || a.g * a.b < a.D) return hipErrorInvalidValue;
  const size_t total = n * static_cast<size_t>(a.Ql + a.P);
  const uint32_t log_n = __builtin_ctzll(n);
  const int grid = grid_for(total);
  switch (a.g) {
    case 1: lt_bsgs_kernel<1><<<grid, kBlock, 0, s>>>(a, log_n, total); break;
    case 2: lt_bsgs_kernel<2><<<grid, kBlock, 0, s>>>(a, log_n, total); break;
    case 4: lt_bsgs_kernel<4><<<grid, kBlock, 0, s>>>(a, log_n, total); break;
    case 8: lt_bsgs_kernel<8><<<grid, kBlock, 0, s>>>(a, log_n, total); break;
    case 16: lt_bsgs_kernel<16><<<grid, kBlock, 0, s>>>(a, log_n, total); break;
    case 32: lt_bsgs_kernel<32><<<grid, kBlock, 0, s>>>(a, log_n, total); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t mul_scalar_v(const uint64_t* in, const LimbScalars& c, uint64_t* out, const uint64_t* q, size_t n,
                        size_t L, hipStream_t s) {
  if (L > static_cast<size_t>(kMaxScalarLimbs)) return hipErrorInvalidValue;
  const size_t total = n * L;
  scalar_v_kernel<true><<<grid_for(total), kBlock, 0, s>>>(in, c, out, q, __builtin_ctzll(n), total);
  return hipGetLastError();
}

hipError_t add_scalar_v(const uint64_t* in, const LimbScalars& c, uint64_t* out, const uint64_t* q, size_t n,
                        size_t L, hipStream_t s) {
  if (L > static_cast<size_t>(kMaxScalarLimbs)) return hipErrorInvalidValue;
  const size_t total = n * L;
  scalar_v_kernel<false><<<grid_for(total), kBlock, 0, s>>>(in, c, out, q, __builtin_ctzll(n), total);
  return hipGetLastError();
}

}  // namespace phx
