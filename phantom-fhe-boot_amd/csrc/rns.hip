// rns.hip — elementwise RNS arithmetic, base conversion, key-switch and rescale kernels.
// HBM-bound streaming kernels: 16 B per lane accesses (two coefficients), grid-stride
// loops sized to a few waves per SIMD; per-limb constants come through the scalar cache.
#include "rns.h"

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "arith.h"

namespace phx {
namespace {

constexpr int kBlock = 256;

int num_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipDeviceProp_t p;
    cus = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess) ? p.multiProcessorCount
                                                                                              : 256;
  }
  return cus;
}

int grid_for(size_t work_items) {
  const int cus = num_cus();
  const size_t blocks = (work_items + kBlock - 1) / kBlock;
  return static_cast<int>(std::max<size_t>(1, std::min<size_t>(blocks, static_cast<size_t>(cus) * 8)));
}

// grid of a per-polynomial kernel: x covers one polynomial's work, y = polynomial
dim3 poly_grid(size_t work_items, size_t polys) {
  const int total = grid_for(work_items * polys);
  const int x = std::max(1, (total + static_cast<int>(polys) - 1) / static_cast<int>(polys));
  return dim3(static_cast<unsigned>(x), static_cast<unsigned>(polys));
}

using u64x2 = ulonglong2;

// 16-byte accesses, always to global memory: the explicit address space keeps a pointer the compiler
// cannot trace to a kernel argument (a key digit read from a pointer table) off FLAT instructions,
// which count in lgkmcnt too, so that every LDS wait would also wait for them
typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));
using GV2 = __attribute__((address_space(1))) v2u64;
__device__ __forceinline__ u64x2 ld2(const uint64_t* p) {
  const v2u64 v = *(const GV2*)p;
  return make_ulonglong2(v.x, v.y);
}
// streamed-once operands (keys): nontemporal 16-byte load
__device__ __forceinline__ u64x2 ld2_nt(const uint64_t* p) {
  const v2u64 v = __builtin_nontemporal_load((const GV2*)p);
  return make_ulonglong2(v.x, v.y);
}
__device__ __forceinline__ void st2(uint64_t* p, uint64_t a, uint64_t b) {
  v2u64 v;
  v.x = a;
  v.y = b;
  *(GV2*)p = v;
}

// generic binary elementwise over [L][n] with per-limb modulus
// blockIdx.y: polynomial (a and out contiguous [polys][L][n], b at b + y * b_stride)
template <typename Op>
__global__ __launch_bounds__(kBlock) void ew2_kernel(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b,
                                                     uint64_t* out, ModView m, uint32_t log_n, size_t pairs, Op op,
                                                     size_t b_stride) {
  a += blockIdx.y * 2 * pairs;
  out += blockIdx.y * 2 * pairs;
  b += blockIdx.y * b_stride;
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < pairs; i += (size_t)gridDim.x * kBlock) {
    const size_t e = 2 * i;
    const uint32_t l = static_cast<uint32_t>(e >> log_n);
    const uint64_t q = m.q[l];
    const u64x2 x = ld2(a + e);
    const u64x2 y = ld2(b + e);
    st2(out + e, op(x.x, y.x, q, m, l), op(x.y, y.y, q, m, l));
  }
}

struct AddOp {
  __device__ uint64_t operator()(uint64_t x, uint64_t y, uint64_t q, const ModView&, uint32_t) const {
    return add_mod(x, y, q);
  }
};
struct SubOp {
  __device__ uint64_t operator()(uint64_t x, uint64_t y, uint64_t q, const ModView&, uint32_t) const {
    return sub_mod(x, y, q);
  }
};
struct MulOp {
  __device__ uint64_t operator()(uint64_t x, uint64_t y, uint64_t q, const ModView& m, uint32_t l) const {
    return mul_mod(x, y, q, m.barrett[2 * l], m.barrett[2 * l + 1]);
  }
};

// out (+)= sum_i in[i]; blockIdx.y: polynomial
__global__ __launch_bounds__(kBlock) void add_many_kernel(AddManyArgs a, uint64_t* out, ModView m, uint32_t log_n,
                                                          size_t pairs, size_t stride) {
  const size_t poff = blockIdx.y * stride;
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < pairs; i += (size_t)gridDim.x * kBlock) {
    const size_t e = 2 * i;
    const uint64_t q = m.q[e >> log_n];
    u64x2 acc = a.accumulate ? ld2(out + poff + e) : ld2(a.in[0] + poff + e);
    for (int k = a.accumulate ? 0 : 1; k < a.count; ++k) {
      const u64x2 x = ld2(a.in[k] + poff + e);
      acc.x = add_mod(acc.x, x.x, q);
      acc.y = add_mod(acc.y, x.y, q);
    }
    st2(out + poff + e, acc.x, acc.y);
  }
}

__global__ __launch_bounds__(kBlock) void negate_kernel(const uint64_t* __restrict__ a, uint64_t* out, ModView m,
                                                        uint32_t log_n, size_t pairs) {
  a += blockIdx.y * 2 * pairs;  // blockIdx.y: polynomial
  out += blockIdx.y * 2 * pairs;
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < pairs; i += (size_t)gridDim.x * kBlock) {
    const size_t e = 2 * i;
    const uint64_t q = m.q[e >> log_n];
    const u64x2 x = ld2(a + e);
    st2(out + e, neg_mod(x.x, q), neg_mod(x.y, q));
  }
}

__global__ __launch_bounds__(kBlock) void mul_add_kernel(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b,
                                                         const uint64_t* __restrict__ c, uint64_t* out, ModView m,
                                                         uint32_t log_n, size_t pairs) {
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < pairs; i += (size_t)gridDim.x * kBlock) {
    const size_t e = 2 * i;
    const uint32_t l = static_cast<uint32_t>(e >> log_n);
    const uint64_t q = m.q[l], r0 = m.barrett[2 * l], r1 = m.barrett[2 * l + 1];
    const u64x2 x = ld2(a + e), y = ld2(b + e), z = ld2(c + e);
    u128 p0 = mul_wide(x.x, y.x), p1 = mul_wide(x.y, y.y);
    add128(p0, u128{z.x, 0});
    add128(p1, u128{z.y, 0});
    st2(out + e, barrett_reduce_128(p0, q, r0, r1), barrett_reduce_128(p1, q, r0, r1));
  }
}

__global__ __launch_bounds__(kBlock) void mul_scalar_kernel(const uint64_t* __restrict__ a, const uint64_t* sc,
                                                            const uint64_t* scs, uint64_t* out, ModView m,
                                                            uint32_t log_n, size_t pairs) {
  a += blockIdx.y * 2 * pairs;  // blockIdx.y: polynomial
  out += blockIdx.y * 2 * pairs;
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < pairs; i += (size_t)gridDim.x * kBlock) {
    const size_t e = 2 * i;
    const uint32_t l = static_cast<uint32_t>(e >> log_n);
    const uint64_t q = m.q[l], w = sc[l], ws = scs[l];
    const u64x2 x = ld2(a + e);
    st2(out + e, mul_shoup(x.x, w, ws, q), mul_shoup(x.y, w, ws, q));
  }
}

__global__ __launch_bounds__(kBlock) void add_scalar_kernel(const uint64_t* __restrict__ a, const uint64_t* sc,
                                                            uint64_t* out, ModView m, uint32_t log_n, size_t pairs) {
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < pairs; i += (size_t)gridDim.x * kBlock) {
    const size_t e = 2 * i;
    const uint32_t l = static_cast<uint32_t>(e >> log_n);
    const uint64_t q = m.q[l], w = sc[l];
    const u64x2 x = ld2(a + e);
    st2(out + e, add_mod(x.x, w, q), add_mod(x.y, w, q));
  }
}

// d0 = a0 b0, d1 = a0 b1 + a1 b0 (one Barrett on the 128-bit sum), d2 = a1 b1
__global__ __launch_bounds__(kBlock) void tensor_kernel(const uint64_t* ct1, const uint64_t* ct2, uint64_t* out,
                                                        ModView m, uint32_t log_n, size_t pairs, size_t stride) {
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < pairs; i += (size_t)gridDim.x * kBlock) {
    const size_t e = 2 * i;
    const uint32_t l = static_cast<uint32_t>(e >> log_n);
    const uint64_t q = m.q[l], r0 = m.barrett[2 * l], r1 = m.barrett[2 * l + 1];
    const u64x2 a0 = ld2(ct1 + e), a1 = ld2(ct1 + stride + e);
    const u64x2 b0 = ld2(ct2 + e), b1 = ld2(ct2 + stride + e);
    u128 c1x = mul_wide(a0.x, b1.x), c1y = mul_wide(a0.y, b1.y);
    add128(c1x, mul_wide(a1.x, b0.x));
    add128(c1y, mul_wide(a1.y, b0.y));
    const uint64_t d0x = mul_mod(a0.x, b0.x, q, r0, r1), d0y = mul_mod(a0.y, b0.y, q, r0, r1);
    const uint64_t d2x = mul_mod(a1.x, b1.x, q, r0, r1), d2y = mul_mod(a1.y, b1.y, q, r0, r1);
    st2(out + e, d0x, d0y);
    st2(out + stride + e, barrett_reduce_128(c1x, q, r0, r1), barrett_reduce_128(c1y, q, r0, r1));
    st2(out + 2 * stride + e, d2x, d2y);
  }
}

// squaring (tensor_square_2x2_rns_poly, src/polymath.cu:538-582): d0 = a0^2, d1 = 2 a0 a1,
// d2 = a1^2 — 2 polynomials read instead of 4.  out may alias ct (each lane reads its own
// elements before writing them).
__global__ __launch_bounds__(kBlock) void tensor_square_kernel(const uint64_t* ct, uint64_t* out, ModView m,
                                                               uint32_t log_n, size_t pairs, size_t stride) {
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < pairs; i += (size_t)gridDim.x * kBlock) {
    const size_t e = 2 * i;
    const uint32_t l = static_cast<uint32_t>(e >> log_n);
    const uint64_t q = m.q[l], r0 = m.barrett[2 * l], r1 = m.barrett[2 * l + 1];
    const u64x2 a0 = ld2(ct + e), a1 = ld2(ct + stride + e);
    const uint64_t px = mul_mod(a0.x, a1.x, q, r0, r1), py = mul_mod(a0.y, a1.y, q, r0, r1);
    const uint64_t d0x = mul_mod(a0.x, a0.x, q, r0, r1), d0y = mul_mod(a0.y, a0.y, q, r0, r1);
    const uint64_t d2x = mul_mod(a1.x, a1.x, q, r0, r1), d2y = mul_mod(a1.y, a1.y, q, r0, r1);
    st2(out + e, d0x, d0y);
    st2(out + stride + e, add_mod(px, px, q), add_mod(py, py, q));
    st2(out + 2 * stride + e, d2x, d2y);
  }
}

// ---------------------------------------------------------------------------------------
// fast base conversion.  2-D grid: x = coefficient pairs, y = groups of kBconvJ output limbs, so
// a [15 -> 45] conversion at n = 2^16 runs 1,152 workgroups instead of 128 (one thread per
// coefficient pair looping over all 45 outputs left the chip at half a wave per SIMD: 88 us ->
// 25 us per conversion on MI355X, profiles/r01/c3_*).  Each output group re-reads its ibase
// inputs (L2/MALL hits); J = 3..15 measured within 4% of each other (tools/c3_variants.sh).
// ---------------------------------------------------------------------------------------
constexpr int kMaxIbase = 64;

// Block -> (coefficient chunk, output group).  The groups of one chunk read the same inputs, so
// they are dealt to one XCD back to back (blocks b and b + 8 share an XCD under round-robin
// placement; speed only, any placement is correct): the inputs come from HBM once and the other
// groups hit that XCD's L2, instead of every group re-reading them from the Infinity Cache.
struct BconvBlock {
  uint32_t chunk;
  int group;
};
__device__ __forceinline__ BconvBlock bconv_block(uint32_t chunks, int groups) {
  const uint32_t b = blockIdx.x;
  if (chunks % 8 == 0) {
    const uint32_t x = b % 8, k = b / 8;
    return {x + 8 * (k / groups), static_cast<int>(k % groups)};
  }
  return {b % chunks, static_cast<int>(b / chunks)};
}
constexpr int kBconvJ = 5;

// the job of a multi-converter launch (BconvArgs::jobs): its matrix, output base and skip
__device__ __forceinline__ void bconv_select_job(BconvArgs& a) {
  if (a.jobs > 1) {
    const int d = a.period ? static_cast<int>(blockIdx.z) % a.period : static_cast<int>(blockIdx.z);
    // constant indices only: a dynamic index would copy the kernel arguments to scratch
#pragma unroll
    for (int k = 0; k < BconvArgs::kMaxJobs; ++k)
      if (k == d) {
        a.qhat_mod_p = a.job_qhat_mod_p[k];
        a.obase = a.job_obase[k];
        a.obase_barrett = a.job_obase_barrett[k];
        a.mfma_frag = a.job_mfma_frag[k];
        a.mfma_rows = a.job_mfma_rows[k];
      }
    a.skip_at += d * a.skip_step;
  }
}

// blockIdx.z: polynomial (or digit; with a period, batch z / period of digit z % period)
__device__ __forceinline__ void bconv_offsets(BconvArgs& a) {
  const uint32_t z = blockIdx.z;
  if (a.period) {
    const uint32_t r = z % static_cast<uint32_t>(a.period), o = z / static_cast<uint32_t>(a.period);
    a.in += r * a.in_stride + o * a.in_outer;
    a.out += r * a.out_stride + o * a.out_outer;
  } else {
    a.in += z * a.in_stride;
    a.out += z * a.out_stride;
  }
}

__device__ __forceinline__ void bconv_outputs(const BconvArgs& a, const uint64_t* tx, const uint64_t* ty, int ib,
                                              uint32_t n, uint32_t k, int group) {
  const int j0 = group * kBconvJ, j1 = min(j0 + kBconvJ, a.obase_size);
  for (int j = j0; j < j1; ++j) {
    u128 accx{0, 0}, accy{0, 0};
    const uint64_t p = a.obase[j], r0 = a.obase_barrett[2 * j], r1 = a.obase_barrett[2 * j + 1];
    for (int s = 0; s < ib; ++s) {
      const uint64_t c = a.qhat_mod_p[(size_t)s * a.obase_size + j];
      add128(accx, mul_wide(tx[s], c));
      add128(accy, mul_wide(ty[s], c));
      if (s % 15 == 14 && s + 1 < ib) {  // keep the sum below p * 2^64 for the Barrett quotient
        accx = u128{barrett_reduce_128(accx, p, r0, r1), 0};
        accy = u128{barrett_reduce_128(accy, p, r0, r1), 0};
      }
    }
    const int oj = j < a.skip_at ? j : j + a.skip_len;
    st2(a.out + (size_t)oj * n + k, barrett_reduce_128(accx, p, r0, r1), barrett_reduce_128(accy, p, r0, r1));
  }
}

__device__ __forceinline__ void bconv_inputs(const BconvArgs& a, uint64_t* tx, uint64_t* ty, int ib, uint32_t n,
                                             uint32_t k, bool prescale) {
  for (int s = 0; s < ib; ++s) {
    const u64x2 x = ld2(a.in + (size_t)s * n + k);
    if (prescale) {
      const uint64_t q = a.ibase[s], w = a.qhat_inv[s], ws = a.qhat_inv_shoup[s];
      tx[s] = mul_shoup(x.x, w, ws, q);
      ty[s] = mul_shoup(x.y, w, ws, q);
    } else {
      tx[s] = x.x;
      ty[s] = x.y;
    }
  }
}

__global__ __launch_bounds__(kBlock) void bconv_kernel(BconvArgs a, uint32_t n, uint32_t pairs, bool prescale) {
  bconv_select_job(a);
  bconv_offsets(a);
  const BconvBlock bb = bconv_block((pairs + kBlock - 1) / kBlock, (a.obase_size + kBconvJ - 1) / kBconvJ);
  const uint32_t i = bb.chunk * kBlock + threadIdx.x;
  if (i >= pairs) return;
  uint64_t tx[kMaxIbase], ty[kMaxIbase];
  bconv_inputs(a, tx, ty, a.ibase_size, n, 2 * i, prescale);
  bconv_outputs(a, tx, ty, a.ibase_size, n, 2 * i, bb.group);
}

// Fixed ibase <= 15: 30-bit limb splitting.  With t = th 2^30 + tl and c = ch 2^30 + cl (t, c <
// 2^60), sum_s t_s c_s = HH 2^60 + (M1 + M2) 2^30 + LL where every partial sum of <= 15 products
// of 30-bit halves stays below 2^64: 4 v_mad_u64_u32 per term and no carry chains (the 64x64
// product + 128-bit accumulate form costs ~7 instructions per term plus register shuffles).
template <int IB, bool PRE>
__global__ __launch_bounds__(kBlock) void bconv_fixed_kernel(BconvArgs a, uint32_t n, uint32_t pairs) {
  static_assert(IB <= 15, "partial sums of 30-bit products must stay below 2^64");
  constexpr uint64_t kM30 = (1ull << 30) - 1;
  // this block's [IB][kBconvJ] slice of the matrix (split in 30-bit halves) and output moduli,
  // staged once in LDS: the matrix may alias nothing the kernel writes, but the compiler cannot
  // prove it, so direct reads would be vector loads inside the accumulation loop
  __shared__ uint32_t mlo[IB][kBconvJ], mhi[IB][kBconvJ];
  __shared__ uint64_t mp[kBconvJ][3];
  bconv_select_job(a);
  const BconvBlock bb = bconv_block((pairs + kBlock - 1) / kBlock, (a.obase_size + kBconvJ - 1) / kBconvJ);
  const int j0 = bb.group * kBconvJ;
  for (int e = threadIdx.x; e < IB * kBconvJ; e += kBlock) {
    const int sidx = e / kBconvJ, jj = e % kBconvJ;
    const uint64_t c = j0 + jj < a.obase_size ? a.qhat_mod_p[(size_t)sidx * a.obase_size + j0 + jj] : 0;
    mlo[sidx][jj] = static_cast<uint32_t>(c & kM30);
    mhi[sidx][jj] = static_cast<uint32_t>(c >> 30);
  }
  if (threadIdx.x < kBconvJ && j0 + (int)threadIdx.x < a.obase_size) {
    const int j = j0 + threadIdx.x;
    mp[threadIdx.x][0] = a.obase[j];
    mp[threadIdx.x][1] = a.obase_barrett[2 * j];
    mp[threadIdx.x][2] = a.obase_barrett[2 * j + 1];
  }
  __syncthreads();
  const uint32_t i = bb.chunk * kBlock + threadIdx.x;
  if (i >= pairs) return;
  bconv_offsets(a);
  uint32_t lo[2][IB], hi[2][IB];
  // every input load issued before any use (a branch between them would serialise them)
  u64x2 xin[IB];
#pragma unroll
  for (int s = 0; s < IB; ++s) xin[s] = ld2(a.in + (size_t)s * n + 2 * i);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < IB; ++s) {
    const u64x2 x = xin[s];
    uint64_t tx = x.x, ty = x.y;
    if constexpr (PRE) {
      const uint64_t q = a.ibase[s], w = a.qhat_inv[s], ws = a.qhat_inv_shoup[s];
      tx = mul_shoup(tx, w, ws, q);
      ty = mul_shoup(ty, w, ws, q);
    }
    lo[0][s] = static_cast<uint32_t>(tx & kM30);
    hi[0][s] = static_cast<uint32_t>(tx >> 30);
    lo[1][s] = static_cast<uint32_t>(ty & kM30);
    hi[1][s] = static_cast<uint32_t>(ty >> 30);
  }
#pragma unroll
  for (int jj = 0; jj < kBconvJ; ++jj) {
    const int j = j0 + jj;
    if (j >= a.obase_size) break;
    uint64_t ll[2] = {0, 0}, m1[2] = {0, 0}, m2[2] = {0, 0}, hh[2] = {0, 0};
#pragma unroll
    for (int s = 0; s < IB; ++s) {
      const uint32_t cl = mlo[s][jj], ch = mhi[s][jj];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        ll[e] += static_cast<uint64_t>(lo[e][s]) * cl;
        m1[e] += static_cast<uint64_t>(lo[e][s]) * ch;
        m2[e] += static_cast<uint64_t>(hi[e][s]) * cl;
        hh[e] += static_cast<uint64_t>(hi[e][s]) * ch;
      }
    }
    const uint64_t p = mp[jj][0], r0 = mp[jj][1], r1 = mp[jj][2];
    uint64_t out[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      u128 v{ll[e], 0};
      add128(v, u128{m1[e] << 30, m1[e] >> 34});
      add128(v, u128{m2[e] << 30, m2[e] >> 34});
      add128(v, u128{hh[e] << 60, hh[e] >> 4});
      out[e] = barrett_reduce_128(v, p, r0, r1);
    }
    const int oj = j < a.skip_at ? j : j + a.skip_len;
    st2(a.out + (size_t)oj * n + 2 * i, out[0], out[1]);
  }
}

// ---------------------------------------------------------------------------------------
// Base conversion on the matrix cores (rns.h, bconv_mfma_tables).  Inputs t < 2^61 become signed
// base-256 digits with one add and one xor: (t + 0x80..80) ^ 0x80..80 holds bytes d_a + 128 ^ 128
// = d_a as int8, sum_a d_a 256^a = t.  For a tile of 16 coefficients (the MFMA's columns) and 16
// output limbs (its rows), the 8 products T_b = A_b . D (v_mfma_i32_16x16x64_i8, K = 64 per
// kstep: 8 limbs x 8 digits) are exact int32 sums of at most 128 products of magnitude <= 2^14,
// so |T_b| <= 2^21, and
//   y = sum_b T_b 256^b = sum_{s,a} d_{s,a} m_{s,a}       (|y| <= 2^14 p, congruent to the result)
// is rebuilt from four int32 pairs (T_0 + 256 T_1 ...) as its low 64 bits (wrapping adds) and
// an FP32 estimate of y / p; q = rint(estimate) is the nearest quotient (|error| ~2^-8), so y - q p
// lies in [-p/2, p/2] and one conditional add of p makes it canonical.  Per output element this
// is about 32 VALU instructions instead of the 60 v_mad_u64_u32 of the 30-bit-split form.
//
// The conversion is then bound by its data movement, and what sets that is the reads in flight:
// measured (tools/variants, profiles/r02/bconv_mfma/), the same kernel with its products or its
// reassembly removed ran at the same speed while it kept one tile of loads in flight per wave.
// So: workgroups stage the job's A fragments (<= 64 KB) in LDS once; each wave owns whole
// 16-coefficient tiles (every 16-row block, NJB of them), keeps the inputs of the next TWO tiles
// in flight, and stores through a raw buffer resource (rows past obase are dropped by the range
// check instead of a branch, so the store count is static and the loop's vmcnt waits never wait
// for stores).
// ---------------------------------------------------------------------------------------
typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
// waves per workgroup, two workgroups per CU (4 / 16 measured slower, profiles/r03/ntt_experiments/bconv_c3.txt)
constexpr int kMfmaWaves = 8;
constexpr uint32_t kDropRow = 0x80000000u;  // byte offset of output rows past obase
constexpr int kBufferWord3 = 0x00020000;    // raw buffer resource word 3 (gfx9: 32-bit data format)
constexpr int kStoreSc1 = 16;  // write-through output stores (sc1): 27.3 -> 25.8 us mean, nt 27.6

__device__ __forceinline__ uint64_t signed_digits(uint64_t t) {
  constexpr uint64_t k80 = 0x8080808080808080ull;
  return (t + k80) ^ k80;
}

template <int KT, int NJB, bool PRE>
__global__ __launch_bounds__(kMfmaWaves * 64) __attribute__((amdgpu_waves_per_eu(kMfmaWaves / 2, kMfmaWaves / 2)))
void bconv_mfma_kernel(BconvArgs a, uint32_t n) {
  __shared__ v4i frag[NJB * 8 * KT * 64];
  // per output row j: p_j, quotient factors, {p_j as P0 + 2^32 P1 with P0 a signed 32-bit value,
  // byte offset of the row in a.out}
  __shared__ uint64_t row_p[NJB * 16];
  __shared__ float4 row_f[NJB * 16];  // {2^48, 2^32, 2^16, 1} / p_j
  __shared__ uint4 row_m[NJB * 16];
  __shared__ ulonglong4 pre_c[PRE ? kBconvMfmaMaxIbase : 1];  // {q_s, qHat_s^-1, its Shoup quotient}
  bconv_select_job(a);
  bconv_offsets(a);
  const int ib = a.ibase_size, ob = a.obase_size;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t c = lane & 15, g = lane >> 4;
  const uint32_t tiles = n / 16;
  const uint32_t step = gridDim.x * kMfmaWaves;
  uint32_t tile = blockIdx.x * kMfmaWaves + wave;
  const uint32_t tile_end = tiles;
  // this lane's input limbs: s = 8 t + 2 g + u.  Loads are unconditional: limbs past ib read limb
  // ib - 1 (zeroed when converted) and tiles past the end read the last tile
  auto load = [&](uint64_t (&x)[KT][2], uint32_t tl) {
    const uint64_t* src = a.in + min(tl, tiles - 1) * 16 + c;
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int s = min(8 * t + 2 * static_cast<int>(g) + u, ib - 1);
        x[t][u] = __builtin_nontemporal_load(src + (size_t)s * n);
      }
  };
  uint64_t xa[KT][2], xb[KT][2];
  load(xa, tile);  // in flight while the tables are staged
  load(xb, tile + step);
  {
    const v4i* gf = static_cast<const v4i*>(a.mfma_frag);
    constexpr int kWords = NJB * 8 * KT * 64, kPer = (kWords + kMfmaWaves * 64 - 1) / (kMfmaWaves * 64);
    v4i tmp[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = threadIdx.x + i * kMfmaWaves * 64;
      if (e < kWords) tmp[i] = gf[e];
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = threadIdx.x + i * kMfmaWaves * 64;
      if (e < kWords) frag[e] = tmp[i];
    }
    if constexpr (PRE)
      if (threadIdx.x < static_cast<uint32_t>(ib))
        pre_c[threadIdx.x] = make_ulonglong4(a.ibase[threadIdx.x], a.qhat_inv[threadIdx.x],
                                             a.qhat_inv_shoup[threadIdx.x], 0);
    for (int e = threadIdx.x; e < NJB * 16; e += kMfmaWaves * 64) {
      const uint64_t p = a.mfma_rows[2 * e];
      const double inv = __longlong_as_double(static_cast<long long>(a.mfma_rows[2 * e + 1]));
      row_p[e] = p;
      row_f[e] = make_float4(static_cast<float>(inv * 281474976710656.0), static_cast<float>(inv * 4294967296.0),
                             static_cast<float>(inv * 65536.0), static_cast<float>(inv));
      const int oj = e < a.skip_at ? e : e + a.skip_len;
      const uint32_t p0 = lo32(p), p1 = hi32(p) + (p0 >> 31);  // p = (int32)p0 + 2^32 p1
      row_m[e] = make_uint4(p0, p1, e < ob ? static_cast<uint32_t>(oj) * n * 8u : kDropRow, 0u);
    }
  }
  __syncthreads();
  if (tile >= tile_end) return;  // no barrier below
  // the output rows as a raw buffer (<= kDropRow bytes, checked by the launcher)
  const __amdgpu_buffer_rsrc_t out_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      a.out, 0, static_cast<int>(static_cast<uint32_t>(ob + max(a.skip_len, 0)) * n * 8u), kBufferWord3);

  // convert one tile (its inputs in x, which is then refilled with the tile two steps ahead)
  auto convert = [&](uint64_t (&x)[KT][2], uint32_t tl) {
    v4i bf[KT];
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      uint64_t d[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int s = 8 * t + 2 * static_cast<int>(g) + u;
        uint64_t v = x[t][u];
        if constexpr (PRE) {
          const int sc = min(s, ib - 1);  // per-limb constants from LDS: global loads here would
          v = mul_shoup(v, pre_c[sc].y, pre_c[sc].z, pre_c[sc].x);  // join the loop's vmcnt waits
        }
        d[u] = s < ib ? signed_digits(v) : 0;  // limbs past ib: zero digits (their A bytes are 0 too)
      }
      bf[t] = v4i{(int)lo32(d[0]), (int)hi32(d[0]), (int)lo32(d[1]), (int)hi32(d[1])};
    }
    load(x, tl + 2 * step);
    const uint32_t k = tl * 16 + c;
#pragma unroll
    for (int jb = 0; jb < NJB; ++jb) {
      __builtin_amdgcn_sched_barrier(0);  // one row block at a time (hoisting the next block's LDS reads spills)
      v4i acc[8];
#pragma unroll
      for (int b = 0; b < 8; ++b)  // the first product takes an inline-constant zero accumulator
        acc[b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(frag[(jb * 8 + b) * KT * 64 + lane], bf[0], v4i{0, 0, 0, 0}, 0,
                                                       0, 0);
#pragma unroll
      for (int t = 1; t < KT; ++t)
#pragma unroll
        for (int b = 0; b < 8; ++b)
          acc[b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(frag[((jb * 8 + b) * KT + t) * 64 + lane], bf[t], acc[b], 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = jb * 16 + 4 * static_cast<int>(g) + r;
        const int lo_a = acc[0][r] + acc[1][r] * 256, lo_b = acc[2][r] + acc[3][r] * 256;
        const int hi_a = acc[4][r] + acc[5][r] * 256, hi_b = acc[6][r] + acc[7][r] * 256;
        // low 64 bits of y: (hi_a 2^32 + hi_b 2^48) only touch the high word
        const uint32_t w = static_cast<uint32_t>(hi_a) + (static_cast<uint32_t>(hi_b) << 16);
        const uint64_t L = static_cast<uint64_t>(static_cast<int64_t>(lo_a)) +
                           (static_cast<uint64_t>(static_cast<int64_t>(lo_b)) << 16) + (static_cast<uint64_t>(w) << 32);
        // nearest quotient in FP32 from per-row factors f = {2^48, 2^32, 2^16, 1} / p: the
        // quotient is below 2^15 and every term below ~2^15, so its error is ~2^-8 < 1/2
        const float4 f = row_f[j];
        const uint4 rm = row_m[j];
        const uint64_t p = row_p[j];
        const int qt = static_cast<int>(__builtin_rintf(
            __builtin_fmaf(static_cast<float>(hi_b), f.x,
                           __builtin_fmaf(static_cast<float>(hi_a), f.y,
                                          __builtin_fmaf(static_cast<float>(lo_b), f.z, static_cast<float>(lo_a) * f.w)))));
        // y = L - qt p (mod 2^64) with p = P0 + 2^32 P1: one v_mad_i64_i32 and a high-word
        // subtract; y lies in [-p/2, p/2] (qt is the nearest quotient): one conditional add of p
        const int64_t tq = static_cast<int64_t>(-qt) * static_cast<int64_t>(static_cast<int32_t>(rm.x)) +
                           static_cast<int64_t>(L);
        int64_t y = static_cast<int64_t>(static_cast<uint64_t>(tq) -
                                         (static_cast<uint64_t>(static_cast<uint32_t>(qt) * rm.y) << 32));
        y += static_cast<int64_t>(p) & (y >> 63);
        // rows past ob sit at kDropRow, past the buffer's range: the store is dropped
        const v2u yv = {lo32(static_cast<uint64_t>(y)), hi32(static_cast<uint64_t>(y))};
        __builtin_amdgcn_raw_buffer_store_b64(yv, out_rsrc, rm.z + k * 8u, 0, kStoreSc1);
      }
    }
  };
  for (;;) {  // two tiles per trip: the input buffers alternate without register moves
    convert(xa, tile);
    tile += step;
    if (tile >= tile_end) break;
    convert(xb, tile);
    tile += step;
    if (tile >= tile_end) break;
  }
}

// blockIdx.y = limb l (digit l / alpha: one scalar division per block), blockIdx.x = a chunk of
// kCopyPairs pairs of that limb; every load of a thread issued before its stores
constexpr int kCopyPairs = 4 * kBlock;
__global__ __launch_bounds__(kBlock) void modup_copy_kernel(const uint64_t* c2, uint64_t* tmu, uint32_t log_n,
                                                            size_t size_qlp_n, uint32_t alpha) {
  const uint32_t l = blockIdx.y, digit = l / alpha;
  const size_t base = ((size_t)l << log_n) + (size_t)blockIdx.x * 2 * kCopyPairs;
  const size_t limb_end = (size_t)(l + 1) << log_n;
  const uint64_t* src = c2 + base;
  uint64_t* dst = tmu + digit * size_qlp_n + base;
  u64x2 v[kCopyPairs / kBlock];
#pragma unroll
  for (int r = 0; r < kCopyPairs / kBlock; ++r) {
    const size_t e = 2 * ((size_t)r * kBlock + threadIdx.x);
    if (base + e < limb_end) v[r] = ld2(src + e);
  }
#pragma unroll
  for (int r = 0; r < kCopyPairs / kBlock; ++r) {
    const size_t e = 2 * ((size_t)r * kBlock + threadIdx.x);
    if (base + e < limb_end) *reinterpret_cast<u64x2*>(dst + e) = v[r];
  }
}

__global__ __launch_bounds__(kBlock) void ks_inner_kernel(const uint64_t* __restrict__ tmu,
                                                          const uint64_t* const* __restrict__ evk, uint64_t* cx,
                                                          const uint64_t* qp, const uint64_t* qpb, uint32_t log_n,
                                                          size_t pairs, uint32_t size_ql, uint32_t size_q,
                                                          size_t size_qlp_n, size_t size_qp_n, uint32_t beta,
                                                          KsAddend add, size_t first) {
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < pairs; i += (size_t)gridDim.x * kBlock) {
    const size_t e = first + 2 * i;
    const uint32_t nid = static_cast<uint32_t>(e >> log_n);
    const uint32_t twr = nid >= size_ql ? size_q + (nid - size_ql) : nid;
    const size_t kk = e & ((size_t(1) << log_n) - 1);
    const size_t eidx = ((size_t)twr << log_n) + kk;
    const uint64_t q = qp[twr], r0 = qpb[2 * twr], r1 = qpb[2 * twr + 1];
    u128 a0x{0, 0}, a0y{0, 0}, a1x{0, 0}, a1y{0, 0};
    for (uint32_t b = 0; b < beta; ++b) {
      const u64x2 c = ld2(tmu + b * size_qlp_n + e);
      const uint64_t* key = evk[b];
      const u64x2 k0 = ld2(key + eidx);
      const u64x2 k1 = ld2(key + size_qp_n + eidx);
      add128(a0x, mul_wide(c.x, k0.x));
      add128(a0y, mul_wide(c.y, k0.y));
      add128(a1x, mul_wide(c.x, k1.x));
      add128(a1y, mul_wide(c.y, k1.y));
    }
    uint64_t o0x = barrett_reduce_128(a0x, q, r0, r1), o0y = barrett_reduce_128(a0y, q, r0, r1);
    uint64_t o1x = barrett_reduce_128(a1x, q, r0, r1), o1y = barrett_reduce_128(a1y, q, r0, r1);
    if (add.c && nid < size_ql) {  // + P (c0, c1): the key switch result stays P-scaled in QlP
      const uint64_t w = add.pmod[nid], ws = add.pmod_shoup[nid];
      const size_t ql_n = (size_t)size_ql << log_n;
      const u64x2 c0 = ld2(add.c + e), c1 = ld2(add.c + ql_n + e);
      o0x = add_mod(o0x, mul_shoup(c0.x, w, ws, q), q);
      o0y = add_mod(o0y, mul_shoup(c0.y, w, ws, q), q);
      o1x = add_mod(o1x, mul_shoup(c1.x, w, ws, q), q);
      o1y = add_mod(o1y, mul_shoup(c1.y, w, ws, q), q);
    }
    st2(cx + e, o0x, o0y);
    st2(cx + size_qlp_n + e, o1x, o1y);
  }
}

// coefficient-domain moddown tail feeding a modup: y = (c1 - delta) P^-1 (mod q_l) goes to the
// digit's own slot of t_mod_up and, times partQlHatInv, to the base-conversion input t_cks
__global__ __launch_bounds__(kBlock) void moddown_modup_finish_kernel(const uint64_t* c1, const uint64_t* delta,
                                                                      ModdownModupConsts k, uint64_t* t_cks,
                                                                      uint64_t* t_mod_up, uint32_t log_n, size_t pairs,
                                                                      uint32_t alpha, size_t qlp_n, size_t c1_stride,
                                                                      size_t mod_up_stride) {
  // blockIdx.y: polynomial (c1 at y c1_stride, t_mod_up at y mod_up_stride, delta / t_cks [y][ql][n])
  c1 += blockIdx.y * c1_stride;
  delta += blockIdx.y * 2 * pairs;
  t_cks += blockIdx.y * 2 * pairs;
  t_mod_up += blockIdx.y * mod_up_stride;
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < pairs; i += (size_t)gridDim.x * kBlock) {
    const size_t e = 2 * i;
    const uint32_t l = static_cast<uint32_t>(e >> log_n);
    const uint64_t m = k.q[l];
    const u64x2 c = ld2(c1 + e), d = ld2(delta + e);
    uint64_t yx = mul_shoup(sub_mod(c.x, d.x, m), k.pinv[l], k.pinv_shoup[l], m);
    uint64_t yy = mul_shoup(sub_mod(c.y, d.y, m), k.pinv[l], k.pinv_shoup[l], m);
    if (k.bias) {  // uniform: the opt-in unbiased moddown
      yx = add_mod(yx, k.bias, m);
      yy = add_mod(yy, k.bias, m);
    }
    st2(t_mod_up + (l / alpha) * qlp_n + e, yx, yy);
    st2(t_cks + e, mul_shoup(yx, k.hatinv[l], k.hatinv_shoup[l], m), mul_shoup(yy, k.hatinv[l], k.hatinv_shoup[l], m));
  }
}

// hoisted-rotation epilogue: out[t][l][j] (+)= x[t][l][perm j] with x = cx + (t == 0 ? c0 term : 0)
// (MODE 0: none, 1: P c0 on the Ql limbs, 2: an extended-basis c0 on every limb)
// NTT-domain automorphisms (src/galois.cu:104-119) move whole blocks: output index i = brv(j)
// reads brv(k) with k = ((2j + 1) g mod 2n) / 2, and the low m bits of k depend only on the low m
// bits of j, so the top m bits of the source index depend only on the top m bits of i.  Every
// output block of kGalB consecutive indices therefore reads one source block of kGalB consecutive
// indices: a workgroup stages that block in LDS with coalesced loads and gathers from LDS, instead
// of 64 scattered 8-byte reads per wave instruction from HBM.
constexpr uint32_t kGalB = kGaloisBlock;

template <int MODE>  // 0: permute; 1: + P c0 on the Ql limbs of polynomial 0, then permute; 2: + c0
__global__ __launch_bounds__(kBlock) void galois_finish_kernel(GaloisFinishArgs a, uint32_t log_n, uint32_t bsz) {
  __shared__ uint64_t sx[kGalB], sc[kGalB];
  const uint32_t nb = (1u << log_n) / bsz;  // blocks per limb
  const uint32_t row = blockIdx.x / nb, ob = blockIdx.x % nb;  // row = t * QlP + l
  const uint32_t t = row >= a.qlp ? 1 : 0, l = row - t * a.qlp;
  const size_t rbase = (size_t)row << log_n;
  const uint32_t* pm = a.perm + (size_t)ob * bsz;
  const uint32_t sb = pm[0] & ~(bsz - 1);
  const bool addc = t == 0 && (MODE == 2 || (MODE == 1 && l < a.ql));
  for (uint32_t i = threadIdx.x; i < bsz / 2; i += kBlock) {
    const u64x2 x = ld2(a.cx + rbase + sb + 2 * i);
    sx[2 * i] = x.x;
    sx[2 * i + 1] = x.y;
    if (addc) {
      const u64x2 c = ld2(a.c0 + rbase + sb + 2 * i);
      sc[2 * i] = c.x;
      sc[2 * i + 1] = c.y;
    }
  }
  __syncthreads();
  const uint64_t q = a.q[l];
  const uint64_t w = MODE == 1 && addc ? a.pmod[l] : 0, ws = MODE == 1 && addc ? a.pmod_shoup[l] : 0;
  for (uint32_t i = threadIdx.x; i < bsz; i += kBlock) {
    const uint32_t src = pm[i] & (bsz - 1);
    uint64_t v = sx[src];
    if (addc) {
      if constexpr (MODE == 1) v = add_mod(v, mul_shoup(sc[src], w, ws, q), q);
      else if constexpr (MODE == 2) v = add_mod(v, sc[src], q);
    }
    const size_t e = rbase + (size_t)ob * bsz + i;
    if (a.accumulate) v = add_mod(v, a.out[e], q);
    a.out[e] = v;
  }
}

// GROUP: the same rotation of `count` ciphertexts through one key in one launch (bootstraps in
// lockstep), their workgroups of an output block on one XCD 8 dispatches apart so that the
// followers read the key halves from that XCD's L2 (as ks_rotate_batch_full's GROUP form)
template <int MODE, bool GROUP>
__global__ __launch_bounds__(kBlock) void ks_rotate_kernel(KsRotateGroupArgs ga, uint32_t log_n, uint32_t bsz) {
  __shared__ uint64_t s0[kGalB], s1[kGalB];
  const uint32_t nb = (1u << log_n) / bsz;
  uint32_t bid = blockIdx.x;
  int c = 0;
  if constexpr (GROUP) {
    const uint32_t K = static_cast<uint32_t>(ga.count), x = bid % 8, k = bid / 8;
    c = static_cast<int>(k % K);
    bid = (k / K) * 8 + x;
  }
  const KsRotateArgs& a = ga.a[c];
  if (GROUP && bid >= a.qlp * nb) return;  // the rounding of the group grid (workgroup-uniform, no barrier passed)
  const uint32_t l = bid / nb, ob = bid % nb;
  const uint32_t twr = l >= a.ql ? a.size_q + (l - a.ql) : l;
  const uint64_t q = a.qp[twr], r0 = a.qp_barrett[2 * twr], r1 = a.qp_barrett[2 * twr + 1];
  const size_t n = size_t(1) << log_n;
  const size_t lbase = (size_t)l << log_n, kbase = (size_t)twr << log_n;
  const size_t qlp_n = (size_t)a.qlp << log_n, qp_n = (size_t)(a.size_q + a.size_p) << log_n;
  const uint32_t* pm = a.perm + (size_t)ob * bsz;
  const uint32_t sb = pm[0] & ~(bsz - 1);
  const bool addc = MODE == 2 || (MODE == 1 && l < a.ql);
  const uint64_t w = MODE == 1 && addc ? a.pmod[l] : 0, ws = MODE == 1 && addc ? a.pmod_shoup[l] : 0;
  for (uint32_t i = threadIdx.x; i < bsz / 2; i += kBlock) {
    const size_t j = sb + 2 * i;
    u128 a0x{0, 0}, a0y{0, 0}, a1x{0, 0}, a1y{0, 0};
    for (uint32_t b = 0; b < a.beta; ++b) {
      const u64x2 c = ld2(a.digits + b * qlp_n + lbase + j);
      const uint64_t* key = a.evk[b];
      const u64x2 k0 = ld2(key + kbase + j), k1 = ld2(key + qp_n + kbase + j);
      add128(a0x, mul_wide(c.x, k0.x));
      add128(a0y, mul_wide(c.y, k0.y));
      add128(a1x, mul_wide(c.x, k1.x));
      add128(a1y, mul_wide(c.y, k1.y));
    }
    uint64_t v0x = barrett_reduce_128(a0x, q, r0, r1), v0y = barrett_reduce_128(a0y, q, r0, r1);
    if (addc) {
      const u64x2 c0 = ld2(a.c0 + lbase + j);
      if constexpr (MODE == 1) {
        v0x = add_mod(v0x, mul_shoup(c0.x, w, ws, q), q);
        v0y = add_mod(v0y, mul_shoup(c0.y, w, ws, q), q);
      } else {
        v0x = add_mod(v0x, c0.x, q);
        v0y = add_mod(v0y, c0.y, q);
      }
    }
    s0[2 * i] = v0x;
    s0[2 * i + 1] = v0y;
    s1[2 * i] = barrett_reduce_128(a1x, q, r0, r1);
    s1[2 * i + 1] = barrett_reduce_128(a1y, q, r0, r1);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < bsz; i += kBlock) {
    const uint32_t src = pm[i] & (bsz - 1);
    const size_t e = lbase + (size_t)ob * bsz + i;
    uint64_t o0 = s0[src], o1 = s1[src];
    if (a.accumulate) {
      o0 = add_mod(o0, a.out[e], q);
      o1 = add_mod(o1, a.out[qlp_n + e], q);
    }
    a.out[e] = o0;
    a.out[qlp_n + e] = o1;
  }
  (void)n;
}

// a pointer every lane holds the same value of (read from LDS), in scalar registers
template <class T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return reinterpret_cast<T*>((static_cast<uint64_t>(hi) << 32) | lo);
}

// workgroup barrier after this wave's LDS writes (lgkmcnt(0)), leaving its global loads in flight
// (a __syncthreads also waits for every outstanding load); the memory clobbers keep the compiler
// from moving LDS accesses across it
__device__ __forceinline__ void ks_lt_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt / expcnt unconstrained
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// keyswitch_rotate_batch: workgroup = (limb l, source block sblk); entry k's products go to LDS
// buffer k & 1 (one barrier per entry: an entry's gather from buffer k & 1 finishes before any
// thread passes entry k + 1's barrier, so entry k + 2 may overwrite it).
//
// Full blocks (BETA > 0): the block's digits and P c0 are loaded once into registers and shared by
// every entry, so an entry reads only its key halves from HBM; those loads are issued for entry
// k + 1 before entry k's barrier and gather, so they are in flight while the gather runs.
//
// GROUP: `count` ciphertexts' baby steps through the same keys (bootstraps in lockstep) in one
// launch; the ciphertexts' workgroups of the same (limb, source block) are dealt to one XCD 8
// dispatches apart (blocks b and b + 8 share an XCD under round-robin placement), so the followers
// read the key halves from that XCD's L2.
constexpr uint32_t kKsBatchFullMax = 64;  // entries of one ks_rotate_batch_full launch
#ifndef PHX_KS_RED
#define PHX_KS_RED 2  // FAST reduction: 2 = split_reduce2 (two folded terms), 1 = split_reduce (three)
#endif
// FAST (GROUP launches over moduli below 2^60, KsRotateBatchArgs::q60): the approximate-quotient
// reduction.  The grouped kernel reads its keys from L2 and is issue-bound, so fewer instructions
// pay there; the single kernel is HBM-bound and keeps the exact form at 128 VGPRs (4 waves per SIMD).
template <int BETA, bool GROUP, bool FAST = false>
__global__ __launch_bounds__(kBlock, BETA <= 3 ? 4 : 3) void ks_rotate_batch_full(KsRotateBatchGroupArgs pa,
                                                                                   uint32_t log_n) {
  constexpr uint32_t bsz = kGalB;
  constexpr int PP = kGalB / 2 / kBlock;  // pairs per thread
  __shared__ uint64_t s0[2][kGalB], s1[2][kGalB];
  const uint32_t nb = (1u << log_n) / bsz;
  uint32_t bid = blockIdx.x;
  int c = 0;
  if constexpr (GROUP) {
    const uint32_t K = static_cast<uint32_t>(pa.count), x = bid % 8, k = bid / 8;
    c = static_cast<int>(k % K);
    bid = (k / K) * 8 + x;
  }
  const KsRotateBatchArgs& a = pa.a[c];
  if (GROUP && bid >= a.qlp * nb) return;  // the rounding of the group grid (workgroup-uniform, no barrier passed)
  const uint32_t l = bid / nb, sblk = bid % nb;
  const uint32_t twr = l >= a.ql ? a.size_q + (l - a.ql) : l;
  const uint64_t q = a.qp[twr], r0 = a.qp_barrett[2 * twr], r1 = a.qp_barrett[2 * twr + 1];
  const size_t lbase = (size_t)l << log_n, kbase = (size_t)twr << log_n;
  const size_t qlp_n = (size_t)a.qlp << log_n, ql_n = (size_t)a.ql << log_n;
  const size_t qp_n = (size_t)(a.size_q + a.size_p) << log_n;
  const size_t j0 = (size_t)sblk * bsz;
  const bool addc = l < a.ql;
  const uint64_t w = addc ? a.pmod[l] : 0, ws = addc ? a.pmod_shoup[l] : 0;
  // the digits split in 30-bit halves once (every entry's products use them), the products
  // accumulated as 30-bit partial sums (ll, mm, hh below 2^62, 2^63, 2^62 for BETA <= 4) and
  // reduced once per output (split_reduce) instead of 128-bit sums and a Barrett reduction
  static_assert(BETA <= 4, "split partial sums");
  constexpr uint64_t kM30 = (1ull << 30) - 1;
  const SplitRed sr = split_red(q, r0, r1);
  uint32_t dl[PP][BETA][2], dh[PP][BETA][2];
  u64x2 pc0[PP];
#pragma unroll
  for (int p = 0; p < PP; ++p) {
    const size_t j = j0 + 2 * (threadIdx.x + p * kBlock);
#pragma unroll
    for (int b = 0; b < BETA; ++b) {
      const u64x2 d = ld2(a.digits + b * qlp_n + lbase + j);
      dl[p][b][0] = static_cast<uint32_t>(d.x & kM30);
      dh[p][b][0] = static_cast<uint32_t>(d.x >> 30);
      dl[p][b][1] = static_cast<uint32_t>(d.y & kM30);
      dh[p][b][1] = static_cast<uint32_t>(d.y >> 30);
    }
    pc0[p] = make_ulonglong2(0, 0);
    if (addc) {
      const u64x2 c0 = ld2(a.ct + lbase + j);
      pc0[p] = make_ulonglong2(mul_shoup(c0.x, w, ws, q), mul_shoup(c0.y, w, ws, q));
    }
  }
  // the key-switched entries compacted in LDS (the identity entries, P (c0, c1) unpermuted, are
  // written first), so the loop below has no branch around its loads: a branch would make the
  // compiler wait for every load in flight where the paths join
  __shared__ const uint64_t* kp[kKsBatchFullMax][BETA];
  __shared__ const uint32_t* pp[kKsBatchFullMax];
  __shared__ uint32_t bi[kKsBatchFullMax];
  __shared__ int64_t oo[kKsBatchFullMax];
  __shared__ int nks;
  if (threadIdx.x < 64) {
    const uint32_t k = threadIdx.x;
    const bool live = k < a.count;
    const KsBatchEntry en = a.entries[live ? k : 0];
    const bool ks = live && en.evk != nullptr;
    const uint64_t m = __ballot(ks);
    const int pos = __popcll(m & ((1ull << threadIdx.x) - 1));
    if (ks) {
      pp[pos] = en.perm;
      bi[pos] = en.binv[sblk];
      oo[pos] = en.out_off;
#pragma unroll
      for (int b = 0; b < BETA; ++b) kp[pos][b] = en.evk[b];
    }
    if (threadIdx.x == 0) nks = __popcll(m);
  }
  for (uint32_t k = 0; k < a.count; ++k) {  // identity entries (workgroup-uniform; nothing in flight yet)
    const KsBatchEntry en = a.entries[k];
    if (en.evk) continue;
    uint64_t* out = a.out + en.out_off;
#pragma unroll
    for (int p = 0; p < PP; ++p) {
      const size_t j = j0 + 2 * (threadIdx.x + p * kBlock);
      uint64_t v1x = 0, v1y = 0;
      if (addc) {
        const u64x2 c1 = ld2(a.ct + ql_n + lbase + j);
        v1x = mul_shoup(c1.x, w, ws, q);
        v1y = mul_shoup(c1.y, w, ws, q);
      }
      st2(out + lbase + j, pc0[p].x, pc0[p].y);
      st2(out + qlp_n + lbase + j, v1x, v1y);
    }
  }
  __syncthreads();
  const int nk = __builtin_amdgcn_readfirstlane(nks);
  if (nk == 0) return;  // workgroup-uniform, no barrier below
  u64x2 k0[PP][BETA], k1[PP][BETA];
  auto load_keys = [&](int k) {
#pragma unroll
    for (int b = 0; b < BETA; ++b) {
      const uint64_t* key = uniform_ptr(kp[k][b]);
#pragma unroll
      for (int p = 0; p < PP; ++p) {
        const size_t j = j0 + 2 * (threadIdx.x + p * kBlock);
        // single: the keys are read once (nontemporal); GROUP: the followers on this XCD read
        // them again from L2, so they keep the default policy
        k0[p][b] = GROUP ? ld2(key + kbase + j) : ld2_nt(key + kbase + j);
        k1[p][b] = GROUP ? ld2(key + qp_n + kbase + j) : ld2_nt(key + qp_n + kbase + j);
      }
    }
  };
  load_keys(0);
  constexpr int GM = bsz / kBlock;  // gathered outputs per thread
  for (int k = 0; k < nk; ++k) {
    uint64_t* t0 = s0[k & 1];
    uint64_t* t1 = s1[k & 1];
    // the gather's permutation first: loads are waited for in issue order, so one issued after
    // the next entry's keys would make the gather wait for those keys too
    const uint32_t ob = bi[k];
    const __attribute__((address_space(1))) uint32_t* pm =
        (const __attribute__((address_space(1))) uint32_t*)uniform_ptr(pp[k]) + (size_t)ob * bsz;
    uint32_t src[GM];
#pragma unroll
    for (int m = 0; m < GM; ++m) src[m] = pm[threadIdx.x + m * kBlock];
    asm volatile("" ::: "memory");  // (issued here, not sunk to their use after the key loads)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int p = 0; p < PP; ++p) {
      const uint32_t i = threadIdx.x + p * kBlock;
      uint64_t ll[2][2] = {{0, 0}, {0, 0}}, mm[2][2] = {{0, 0}, {0, 0}}, hh[2][2] = {{0, 0}, {0, 0}};
#pragma unroll
      for (int b = 0; b < BETA; ++b) {
        const uint64_t kv[2][2] = {{k0[p][b].x, k0[p][b].y}, {k1[p][b].x, k1[p][b].y}};
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const uint32_t kl = static_cast<uint32_t>(kv[t][u] & kM30), kh = static_cast<uint32_t>(kv[t][u] >> 30);
            ll[t][u] += static_cast<uint64_t>(dl[p][b][u]) * kl;
            mm[t][u] += static_cast<uint64_t>(dl[p][b][u]) * kh;
            mm[t][u] += static_cast<uint64_t>(dh[p][b][u]) * kl;
            hh[t][u] += static_cast<uint64_t>(dh[p][b][u]) * kh;
          }
      }
      auto red = [&](uint64_t x, uint64_t y, uint64_t z) {
        if constexpr (FAST && PHX_KS_RED == 2) return split_reduce2(x, y, z, sr, q, r1);
        else if constexpr (FAST) return split_reduce(x, y, z, sr, q, r1);
        else return split_reduce_exact(x, y, z, sr, q, r1);
      };
      t0[2 * i] = add_mod(red(ll[0][0], mm[0][0], hh[0][0]), pc0[p].x, q);
      t0[2 * i + 1] = add_mod(red(ll[0][1], mm[0][1], hh[0][1]), pc0[p].y, q);
      t1[2 * i] = red(ll[1][0], mm[1][0], hh[1][0]);
      t1[2 * i + 1] = red(ll[1][1], mm[1][1], hh[1][1]);
    }
    // the next entry's keys (the last one's again at the end: L2 hits) in flight over the barrier
    // and the gather
    __builtin_amdgcn_sched_barrier(0);
    load_keys(min(k + 1, nk - 1));
    ks_lt_barrier();
    uint64_t* out = a.out + oo[k] + lbase + (size_t)ob * bsz;
#pragma unroll
    for (int m = 0; m < GM; ++m) {
      const uint32_t i = threadIdx.x + m * kBlock;
      out[i] = t0[src[m] & (bsz - 1)];
      out[qlp_n + i] = t1[src[m] & (bsz - 1)];
    }
  }
}

// any block size / beta: per entry, the digits and c0 re-read (L1 / L2 hits after the first)
__global__ __launch_bounds__(kBlock) void ks_rotate_batch_kernel(KsRotateBatchArgs a, uint32_t log_n, uint32_t bsz) {
  __shared__ uint64_t s0[2][kGalB], s1[2][kGalB];
  const uint32_t nb = (1u << log_n) / bsz;
  const uint32_t l = blockIdx.x / nb, sblk = blockIdx.x % nb;
  const uint32_t twr = l >= a.ql ? a.size_q + (l - a.ql) : l;
  const uint64_t q = a.qp[twr], r0 = a.qp_barrett[2 * twr], r1 = a.qp_barrett[2 * twr + 1];
  const size_t lbase = (size_t)l << log_n, kbase = (size_t)twr << log_n;
  const size_t qlp_n = (size_t)a.qlp << log_n, ql_n = (size_t)a.ql << log_n;
  const size_t qp_n = (size_t)(a.size_q + a.size_p) << log_n;
  const size_t j0 = (size_t)sblk * bsz;
  const bool addc = l < a.ql;
  const uint64_t w = addc ? a.pmod[l] : 0, ws = addc ? a.pmod_shoup[l] : 0;
  for (uint32_t k = 0; k < a.count; ++k) {
    const KsBatchEntry e = a.entries[k];
    uint64_t* t0 = s0[k & 1];
    uint64_t* t1 = s1[k & 1];
    for (uint32_t i = threadIdx.x; i < bsz / 2; i += kBlock) {
      const size_t j = j0 + 2 * i;
      uint64_t v0x = 0, v0y = 0, v1x = 0, v1y = 0;
      if (e.evk) {
        u128 a0x{0, 0}, a0y{0, 0}, a1x{0, 0}, a1y{0, 0};
        for (uint32_t b = 0; b < a.beta; ++b) {
          const u64x2 c = ld2(a.digits + b * qlp_n + lbase + j);
          const uint64_t* key = e.evk[b];
          const u64x2 k0 = ld2(key + kbase + j), k1 = ld2(key + qp_n + kbase + j);
          add128(a0x, mul_wide(c.x, k0.x));
          add128(a0y, mul_wide(c.y, k0.y));
          add128(a1x, mul_wide(c.x, k1.x));
          add128(a1y, mul_wide(c.y, k1.y));
        }
        v0x = barrett_reduce_128(a0x, q, r0, r1);
        v0y = barrett_reduce_128(a0y, q, r0, r1);
        v1x = barrett_reduce_128(a1x, q, r0, r1);
        v1y = barrett_reduce_128(a1y, q, r0, r1);
      }
      if (addc) {
        const u64x2 c0 = ld2(a.ct + lbase + j);
        v0x = add_mod(v0x, mul_shoup(c0.x, w, ws, q), q);
        v0y = add_mod(v0y, mul_shoup(c0.y, w, ws, q), q);
        if (!e.evk) {
          const u64x2 c1 = ld2(a.ct + ql_n + lbase + j);
          v1x = mul_shoup(c1.x, w, ws, q);
          v1y = mul_shoup(c1.y, w, ws, q);
        }
      }
      t0[2 * i] = v0x;
      t0[2 * i + 1] = v0y;
      t1[2 * i] = v1x;
      t1[2 * i + 1] = v1y;
    }
    __syncthreads();
    uint64_t* out = a.out + e.out_off;
    if (e.evk) {
      const uint32_t ob = e.binv[sblk];
      const uint32_t* pm = e.perm + (size_t)ob * bsz;
      for (uint32_t i = threadIdx.x; i < bsz; i += kBlock) {
        const uint32_t src = pm[i] & (bsz - 1);
        const size_t d = lbase + (size_t)ob * bsz + i;
        out[d] = t0[src];
        out[qlp_n + d] = t1[src];
      }
    } else {
      for (uint32_t i = threadIdx.x; i < bsz; i += kBlock) {
        out[lbase + j0 + i] = t0[i];
        out[qlp_n + lbase + j0 + i] = t1[i];
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void galois_kernel(const uint64_t* __restrict__ in, uint64_t* out,
                                                        const uint32_t* __restrict__ perm, uint32_t log_n,
                                                        uint32_t bsz) {
  __shared__ uint64_t sx[kGalB];
  const uint32_t nb = (1u << log_n) / bsz;
  const uint32_t row = blockIdx.x / nb, ob = blockIdx.x % nb;
  const size_t rbase = (size_t)row << log_n;
  const uint32_t* pm = perm + (size_t)ob * bsz;
  const uint32_t sb = pm[0] & ~(bsz - 1);
  for (uint32_t i = threadIdx.x; i < bsz / 2; i += kBlock) {
    const u64x2 x = ld2(in + rbase + sb + 2 * i);
    sx[2 * i] = x.x;
    sx[2 * i + 1] = x.y;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < bsz; i += kBlock) out[rbase + (size_t)ob * bsz + i] = sx[pm[i] & (bsz - 1)];
}

__global__ __launch_bounds__(kBlock) void raise_kernel(const uint64_t* in_q0, uint64_t* out, const uint64_t* q,
                                                       const uint64_t* qb, uint32_t log_n, size_t total) {
  const uint64_t q0 = q[0], half = q0 >> 1;
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < total; i += (size_t)gridDim.x * kBlock) {
    const uint32_t l = static_cast<uint32_t>(i >> log_n);
    const uint64_t v = in_q0[i & ((size_t(1) << log_n) - 1)];
    const uint64_t m = q[l];
    uint64_t r;
    if (l == 0) {
      r = v;
    } else if (m > q0) {
      r = v > half ? v + (m - q0) : v;
    } else {
      const uint64_t vv = v > half ? v + (m - q0 % m) : v;
      r = barrett_reduce_64(vv, m, qb[2 * l + 1]);
    }
    out[i] = r;
  }
}

}  // namespace

hipError_t poly_add(const uint64_t* a, const uint64_t* b, uint64_t* out, ModView m, size_t n, size_t L,
                    hipStream_t s, size_t polys, size_t b_stride) {
  const size_t pairs = n * L / 2;
  ew2_kernel<<<poly_grid(pairs, polys), kBlock, 0, s>>>(a, b, out, m, __builtin_ctzll(n), pairs, AddOp{},
                                                        b_stride == kContiguous ? n * L : b_stride);
  return hipGetLastError();
}

hipError_t poly_add_many(const AddManyArgs& a, uint64_t* out, ModView m, size_t n, size_t L, hipStream_t s,
                         size_t polys, size_t stride) {
  if (a.count < 1 || a.count > kAddManyMax) return hipErrorInvalidValue;
  const size_t pairs = n * L / 2;
  add_many_kernel<<<poly_grid(pairs, polys), kBlock, 0, s>>>(a, out, m, __builtin_ctzll(n), pairs, stride);
  return hipGetLastError();
}

hipError_t poly_sub(const uint64_t* a, const uint64_t* b, uint64_t* out, ModView m, size_t n, size_t L,
                    hipStream_t s, size_t polys, size_t b_stride) {
  const size_t pairs = n * L / 2;
  ew2_kernel<<<poly_grid(pairs, polys), kBlock, 0, s>>>(a, b, out, m, __builtin_ctzll(n), pairs, SubOp{},
                                                        b_stride == kContiguous ? n * L : b_stride);
  return hipGetLastError();
}

hipError_t poly_mul(const uint64_t* a, const uint64_t* b, uint64_t* out, ModView m, size_t n, size_t L,
                    hipStream_t s, size_t polys, size_t b_stride) {
  const size_t pairs = n * L / 2;
  ew2_kernel<<<poly_grid(pairs, polys), kBlock, 0, s>>>(a, b, out, m, __builtin_ctzll(n), pairs, MulOp{},
                                                        b_stride == kContiguous ? n * L : b_stride);
  return hipGetLastError();
}

hipError_t poly_negate(const uint64_t* a, uint64_t* out, ModView m, size_t n, size_t L, hipStream_t s,
                       size_t polys) {
  const size_t pairs = n * L / 2;
  negate_kernel<<<poly_grid(pairs, polys), kBlock, 0, s>>>(a, out, m, __builtin_ctzll(n), pairs);
  return hipGetLastError();
}

hipError_t poly_mul_add(const uint64_t* a, const uint64_t* b, const uint64_t* c, uint64_t* out, ModView m,
                        size_t n, size_t L, hipStream_t s) {
  const size_t pairs = n * L / 2;
  mul_add_kernel<<<grid_for(pairs), kBlock, 0, s>>>(a, b, c, out, m, __builtin_ctzll(n), pairs);
  return hipGetLastError();
}

hipError_t poly_mul_scalar(const uint64_t* a, const uint64_t* scalar, const uint64_t* scalar_shoup, uint64_t* out,
                           ModView m, size_t n, size_t L, hipStream_t s, size_t polys) {
  const size_t pairs = n * L / 2;
  mul_scalar_kernel<<<poly_grid(pairs, polys), kBlock, 0, s>>>(a, scalar, scalar_shoup, out, m, __builtin_ctzll(n), pairs);
  return hipGetLastError();
}

hipError_t poly_add_scalar(const uint64_t* a, const uint64_t* scalar, uint64_t* out, ModView m, size_t n, size_t L,
                           hipStream_t s) {
  const size_t pairs = n * L / 2;
  add_scalar_kernel<<<grid_for(pairs), kBlock, 0, s>>>(a, scalar, out, m, __builtin_ctzll(n), pairs);
  return hipGetLastError();
}

hipError_t tensor_prod_2x2(const uint64_t* ct1, const uint64_t* ct2, uint64_t* out, ModView m, size_t n, size_t L,
                           hipStream_t s) {
  const size_t pairs = n * L / 2;
  tensor_kernel<<<grid_for(pairs), kBlock, 0, s>>>(ct1, ct2, out, m, __builtin_ctzll(n), pairs, n * L);
  return hipGetLastError();
}

hipError_t tensor_square_2x2(const uint64_t* ct, uint64_t* out, ModView m, size_t n, size_t L, hipStream_t s) {
  const size_t pairs = n * L / 2;
  tensor_square_kernel<<<grid_for(pairs), kBlock, 0, s>>>(ct, out, m, __builtin_ctzll(n), pairs, n * L);
  return hipGetLastError();
}

size_t bconv_mfma_frag_bytes(int ibase, int obase) {
  return static_cast<size_t>((obase + 15) / 16) * 8 * ((ibase + 7) / 8) * 64 * 16;
}

void bconv_mfma_tables(const uint64_t* qhat_mod_p, const uint64_t* obase, int ibase, int obase_size, uint8_t* frag,
                       uint64_t* rows) {
  using u128h = unsigned __int128;
  constexpr uint64_t k80 = 0x8080808080808080ull;
  const int njb = (obase_size + 15) / 16, kt = (ibase + 7) / 8;
  // signed base-256 digits of m_{s,a,j} = c_sj 256^a mod p_j, packed in a uint64 each
  std::vector<uint64_t> sd((size_t)ibase * 8 * obase_size);
  for (int s = 0; s < ibase; ++s)
    for (int dig = 0; dig < 8; ++dig)
      for (int j = 0; j < obase_size; ++j) {
        const uint64_t p = obase[j];
        const uint64_t m =
            static_cast<uint64_t>((static_cast<u128h>(qhat_mod_p[(size_t)s * obase_size + j] % p) << (8 * dig)) % p);
        sd[((size_t)s * 8 + dig) * obase_size + j] = (m + k80) ^ k80;
      }
  // A fragment of v_mfma_i32_16x16x64_i8: lane (r, g) = (lane & 15, lane >> 4) holds row r and
  // bytes i = 0..15 of K slots 16 g + i <-> (limb 8 t + 2 g + i / 8, digit i % 8); the B fragment
  // (the kernel's inputs) uses the same K order
  for (int jb = 0; jb < njb; ++jb)
    for (int b = 0; b < 8; ++b)
      for (int t = 0; t < kt; ++t)
        for (int lane = 0; lane < 64; ++lane)
          for (int i = 0; i < 16; ++i) {
            const int j = jb * 16 + (lane & 15), s = 8 * t + 2 * (lane >> 4) + i / 8, dig = i % 8;
            const uint8_t v = j < obase_size && s < ibase
                                  ? static_cast<uint8_t>(sd[((size_t)s * 8 + dig) * obase_size + j] >> (8 * b))
                                  : 0;
            frag[((((size_t)jb * 8 + b) * kt + t) * 64 + lane) * 16 + i] = v;
          }
  for (int j = 0; j < njb * 16; ++j) {
    const double inv = j < obase_size ? 1.0 / static_cast<double>(obase[j]) : 0.0;
    uint64_t bits;
    static_assert(sizeof(bits) == sizeof(inv), "double");
    __builtin_memcpy(&bits, &inv, sizeof(bits));
    rows[2 * j] = j < obase_size ? obase[j] : 0;
    rows[2 * j + 1] = bits;
  }
}

namespace {
bool mfma_bconv_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("PHX_BCONV_MFMA");
    return !(e && e[0] == '0');
  }();
  return on;
}
}  // namespace

hipError_t bconv(const BconvArgs& a, size_t n, hipStream_t s) {
  if (a.ibase_size <= 0 || a.ibase_size > kMaxIbase || a.obase_size <= 0) return hipErrorInvalidValue;
  const uint32_t pairs = static_cast<uint32_t>(n / 2);
  if (a.polys < 1) return hipErrorInvalidValue;
  if (a.period < 0 || (a.period && a.polys % a.period)) return hipErrorInvalidValue;
  if (a.jobs > 1 && (a.jobs != (a.period ? a.period : a.polys) || a.jobs > BconvArgs::kMaxJobs))
    return hipErrorInvalidValue;
  bool mfma = mfma_bconv_enabled() && a.ibase_size <= kBconvMfmaMaxIbase && a.obase_size <= kBconvMfmaMaxObase &&
              n >= 16 && n % 16 == 0 &&
              static_cast<size_t>(a.obase_size + std::max(0, a.skip_len)) * n * 8 <= kDropRow;
  if (a.jobs > 1)
    for (int d = 0; d < a.jobs; ++d) mfma = mfma && a.job_mfma_frag[d] && a.job_mfma_rows[d];
  else
    mfma = mfma && a.mfma_frag && a.mfma_rows;
  if (mfma) {
    // two workgroups per CU over all polynomials, each wave looping over 16-column tiles
    const uint32_t tiles = static_cast<uint32_t>(n / 16);
    const uint32_t want = std::max<uint32_t>(1, static_cast<uint32_t>(2 * num_cus() / a.polys));
    const dim3 g(std::min<uint32_t>((tiles + kMfmaWaves - 1) / kMfmaWaves, want), 1, a.polys);
    const bool pre = a.qhat_inv != nullptr;
    const uint32_t nn = static_cast<uint32_t>(n);
    const int kt = (a.ibase_size + 7) / 8, njb = (a.obase_size + 15) / 16;
#define PHX_BCONV_MFMA_LAUNCH(KT, NJB)                                                             \
  if (kt == KT && njb == NJB) {                                                                    \
    if (pre) bconv_mfma_kernel<KT, NJB, true><<<g, kMfmaWaves * 64, 0, s>>>(a, nn);                \
    else bconv_mfma_kernel<KT, NJB, false><<<g, kMfmaWaves * 64, 0, s>>>(a, nn);                   \
    return hipGetLastError();                                                                      \
  }
    PHX_BCONV_MFMA_LAUNCH(1, 1) PHX_BCONV_MFMA_LAUNCH(1, 2) PHX_BCONV_MFMA_LAUNCH(1, 3) PHX_BCONV_MFMA_LAUNCH(1, 4)
    PHX_BCONV_MFMA_LAUNCH(2, 1) PHX_BCONV_MFMA_LAUNCH(2, 2) PHX_BCONV_MFMA_LAUNCH(2, 3) PHX_BCONV_MFMA_LAUNCH(2, 4)
#undef PHX_BCONV_MFMA_LAUNCH
    return hipErrorInvalidValue;
  }
  const dim3 g(((pairs + kBlock - 1) / kBlock) * ((a.obase_size + kBconvJ - 1) / kBconvJ), 1, a.polys);
  const bool pre = a.qhat_inv != nullptr;
  switch (a.ibase_size) {
#define PHX_BCONV_CASE(K)                                                                      \
  case K:                                                                                      \
    if (pre) bconv_fixed_kernel<K, true><<<g, kBlock, 0, s>>>(a, static_cast<uint32_t>(n), pairs); \
    else bconv_fixed_kernel<K, false><<<g, kBlock, 0, s>>>(a, static_cast<uint32_t>(n), pairs);    \
    break;
    PHX_BCONV_CASE(1) PHX_BCONV_CASE(2) PHX_BCONV_CASE(3) PHX_BCONV_CASE(4) PHX_BCONV_CASE(5)
    PHX_BCONV_CASE(6) PHX_BCONV_CASE(7) PHX_BCONV_CASE(8) PHX_BCONV_CASE(9) PHX_BCONV_CASE(10)
    PHX_BCONV_CASE(11) PHX_BCONV_CASE(12) PHX_BCONV_CASE(13) PHX_BCONV_CASE(14) PHX_BCONV_CASE(15)
#undef PHX_BCONV_CASE
    default: bconv_kernel<<<g, kBlock, 0, s>>>(a, static_cast<uint32_t>(n), pairs, pre);
  }
  return hipGetLastError();
}

hipError_t modup_copy_digits(const uint64_t* c2, uint64_t* t_mod_up, size_t n, size_t size_ql, size_t size_qlp,
                             size_t alpha, hipStream_t s) {
  if (size_ql == 0) return hipSuccess;
  if (alpha == 0 || n < 2) return hipErrorInvalidValue;
  const dim3 grid(static_cast<uint32_t>((n / 2 + kCopyPairs - 1) / kCopyPairs), static_cast<uint32_t>(size_ql));
  modup_copy_kernel<<<grid, kBlock, 0, s>>>(c2, t_mod_up, __builtin_ctzll(n), size_qlp * n, static_cast<uint32_t>(alpha));
  return hipGetLastError();
}

hipError_t keyswitch_inner_prod(const uint64_t* t_mod_up, const uint64_t* const* evk, uint64_t* cx,
                                const uint64_t* qp_mod, const uint64_t* qp_barrett, size_t n, size_t size_ql,
                                size_t size_q, size_t size_p, size_t beta, hipStream_t s, const KsAddend& add,
                                size_t first_limb) {
  const size_t size_qlp = size_ql + size_p;
  if (first_limb > size_qlp) return hipErrorInvalidValue;
  const size_t pairs = n * (size_qlp - first_limb) / 2;
  if (pairs == 0) return hipSuccess;
  ks_inner_kernel<<<grid_for(pairs), kBlock, 0, s>>>(t_mod_up, evk, cx, qp_mod, qp_barrett, __builtin_ctzll(n), pairs,
                                                    (uint32_t)size_ql, (uint32_t)size_q, size_qlp * n,
                                                    (size_q + size_p) * n, (uint32_t)beta, add, first_limb * n);
  return hipGetLastError();
}

hipError_t moddown_modup_finish(const uint64_t* c1, const uint64_t* delta, const ModdownModupConsts& k,
                                uint64_t* t_cks, uint64_t* t_mod_up, size_t n, size_t size_ql, size_t size_qlp,
                                size_t alpha, hipStream_t s, size_t polys, size_t c1_stride, size_t mod_up_stride) {
  const size_t pairs = n * size_ql / 2;
  if (polys < 1) return hipErrorInvalidValue;
  moddown_modup_finish_kernel<<<poly_grid(pairs, polys), kBlock, 0, s>>>(
      c1, delta, k, t_cks, t_mod_up, __builtin_ctzll(n), pairs, static_cast<uint32_t>(alpha), size_qlp * n, c1_stride,
      mod_up_stride);
  return hipGetLastError();
}

hipError_t galois_finish(const GaloisFinishArgs& a, int mode, size_t n, hipStream_t s) {
  if (mode < 0 || mode > 2 || a.qlp == 0) return mode < 0 || mode > 2 ? hipErrorInvalidValue : hipSuccess;
  const uint32_t log_n = __builtin_ctzll(n), bsz = static_cast<uint32_t>(std::min<size_t>(n, kGalB));
  const dim3 grid(static_cast<uint32_t>(2 * a.qlp * (n / bsz)));
  switch (mode) {
    case 0: galois_finish_kernel<0><<<grid, kBlock, 0, s>>>(a, log_n, bsz); break;
    case 1: galois_finish_kernel<1><<<grid, kBlock, 0, s>>>(a, log_n, bsz); break;
    default: galois_finish_kernel<2><<<grid, kBlock, 0, s>>>(a, log_n, bsz); break;
  }
  return hipGetLastError();
}

hipError_t keyswitch_rotate(const KsRotateArgs& a, int mode, size_t n, hipStream_t s) {
  if (mode < 0 || mode > 2 || !a.digits || !a.evk || !a.out || !a.perm || a.beta == 0) return hipErrorInvalidValue;
  if (mode > 0 && !a.c0) return hipErrorInvalidValue;
  if (mode == 1 && (!a.pmod || !a.pmod_shoup)) return hipErrorInvalidValue;
  if (a.qlp == 0) return hipSuccess;
  const uint32_t log_n = __builtin_ctzll(n), bsz = static_cast<uint32_t>(std::min<size_t>(n, kGalB));
  const dim3 grid(static_cast<uint32_t>(a.qlp * (n / bsz)));
  switch (mode) {
    case 0: ks_rotate_kernel<0, false><<<grid, kBlock, 0, s>>>(KsRotateGroupArgs{{a}, 1}, log_n, bsz); break;
    case 1: ks_rotate_kernel<1, false><<<grid, kBlock, 0, s>>>(KsRotateGroupArgs{{a}, 1}, log_n, bsz); break;
    default: ks_rotate_kernel<2, false><<<grid, kBlock, 0, s>>>(KsRotateGroupArgs{{a}, 1}, log_n, bsz); break;
  }
  return hipGetLastError();
}

hipError_t keyswitch_rotate_group(const KsRotateGroupArgs& ga, int mode, size_t n, hipStream_t s) {
  if (ga.count < 2 || ga.count > kKsGroupMax || mode < 0 || mode > 2) return hipErrorInvalidValue;
  const KsRotateArgs& a = ga.a[0];
  for (int c = 0; c < ga.count; ++c) {
    const KsRotateArgs& x = ga.a[c];
    if (!x.digits || !x.evk || !x.out || !x.perm || x.beta == 0) return hipErrorInvalidValue;
    if (mode > 0 && !x.c0) return hipErrorInvalidValue;
    if (mode == 1 && (!x.pmod || !x.pmod_shoup)) return hipErrorInvalidValue;
    if (x.evk != a.evk || x.perm != a.perm || x.qlp != a.qlp || x.ql != a.ql || x.beta != a.beta ||
        x.size_q != a.size_q || x.size_p != a.size_p)
      return hipErrorInvalidValue;
  }
  if (a.qlp == 0) return hipSuccess;
  const uint32_t log_n = __builtin_ctzll(n), bsz = static_cast<uint32_t>(std::min<size_t>(n, kGalB));
  const uint32_t per = (a.qlp * static_cast<uint32_t>(n / bsz) + 7) / 8 * 8;
  const dim3 grid(static_cast<uint32_t>(ga.count) * per);
  switch (mode) {
    case 0: ks_rotate_kernel<0, true><<<grid, kBlock, 0, s>>>(ga, log_n, bsz); break;
    case 1: ks_rotate_kernel<1, true><<<grid, kBlock, 0, s>>>(ga, log_n, bsz); break;
    default: ks_rotate_kernel<2, true><<<grid, kBlock, 0, s>>>(ga, log_n, bsz); break;
  }
  return hipGetLastError();
}

hipError_t keyswitch_rotate_batch(const KsRotateBatchArgs& a, size_t n, hipStream_t s) {
  if (!a.digits || !a.entries || !a.ct || !a.out || !a.pmod || !a.pmod_shoup || a.beta == 0 || a.ql > a.qlp)
    return hipErrorInvalidValue;
  if (a.qlp == 0 || a.count == 0) return hipSuccess;
  const uint32_t log_n = __builtin_ctzll(n), bsz = static_cast<uint32_t>(std::min<size_t>(n, kGalB));
  const dim3 grid(static_cast<uint32_t>(a.qlp * (n / bsz)));
  switch (bsz == kGalB && a.count <= kKsBatchFullMax ? a.beta : 0) {
    case 1: ks_rotate_batch_full<1, false><<<grid, kBlock, 0, s>>>(KsRotateBatchGroupArgs{{a}, 1}, log_n); break;
    case 2: ks_rotate_batch_full<2, false><<<grid, kBlock, 0, s>>>(KsRotateBatchGroupArgs{{a}, 1}, log_n); break;
    case 3: ks_rotate_batch_full<3, false><<<grid, kBlock, 0, s>>>(KsRotateBatchGroupArgs{{a}, 1}, log_n); break;
    case 4: ks_rotate_batch_full<4, false><<<grid, kBlock, 0, s>>>(KsRotateBatchGroupArgs{{a}, 1}, log_n); break;
    default: ks_rotate_batch_kernel<<<grid, kBlock, 0, s>>>(a, log_n, bsz); break;
  }
  return hipGetLastError();
}

hipError_t keyswitch_rotate_batch_group(const KsRotateBatchGroupArgs& ga, size_t n, hipStream_t s) {
  if (ga.count < 2 || ga.count > kKsGroupMax) return hipErrorInvalidValue;
  const KsRotateBatchArgs& a = ga.a[0];
  for (int c = 0; c < ga.count; ++c) {
    const KsRotateBatchArgs& x = ga.a[c];
    if (!x.digits || !x.entries || !x.ct || !x.out || !x.pmod || !x.pmod_shoup || x.beta == 0 || x.ql > x.qlp)
      return hipErrorInvalidValue;
    if (x.entries != a.entries || x.count != a.count || x.qlp != a.qlp || x.ql != a.ql || x.beta != a.beta ||
        x.size_q != a.size_q || x.size_p != a.size_p)
      return hipErrorInvalidValue;
  }
  if (a.qlp == 0 || a.count == 0) return hipSuccess;
  if (n < kGalB || a.beta > 4 || a.count > kKsBatchFullMax) {  // the shapes without the register-resident form: one launch each
    for (int c = 0; c < ga.count; ++c)
      if (hipError_t e = keyswitch_rotate_batch(ga.a[c], n, s)) return e;
    return hipSuccess;
  }
  const uint32_t log_n = __builtin_ctzll(n);
  const uint32_t per = (a.qlp * static_cast<uint32_t>(n / kGalB) + 7) / 8 * 8;
  const dim3 grid(static_cast<uint32_t>(ga.count) * per);
  bool fast = true;
  for (int c = 0; c < ga.count; ++c) fast = fast && ga.a[c].q60 != 0;
#define PHX_KSBF_GROUP(B)                                                              \
  case B:                                                                              \
    if (fast) ks_rotate_batch_full<B, true, true><<<grid, kBlock, 0, s>>>(ga, log_n);  \
    else ks_rotate_batch_full<B, true, false><<<grid, kBlock, 0, s>>>(ga, log_n);      \
    break;
  switch (a.beta) {
    PHX_KSBF_GROUP(1) PHX_KSBF_GROUP(2) PHX_KSBF_GROUP(3)
    default:
    PHX_KSBF_GROUP(4)
  }
#undef PHX_KSBF_GROUP
  return hipGetLastError();
}

hipError_t galois_ntt(const uint64_t* in, uint64_t* out, const uint32_t* perm, size_t n, size_t L,
                      hipStream_t s) {
  if (in == out) return hipErrorInvalidValue;  // blocks are read while others are written
  if (L == 0) return hipSuccess;
  const uint32_t bsz = static_cast<uint32_t>(std::min<size_t>(n, kGalB));
  galois_kernel<<<static_cast<uint32_t>(L * (n / bsz)), kBlock, 0, s>>>(in, out, perm, __builtin_ctzll(n), bsz);
  return hipGetLastError();
}

hipError_t switch_modulus_raise(const uint64_t* in_q0, uint64_t* out, const uint64_t* q, const uint64_t* barrett,
                                size_t n, size_t L, hipStream_t s) {
  const size_t total = n * L;
  raise_kernel<<<grid_for(total), kBlock, 0, s>>>(in_q0, out, q, barrett, __builtin_ctzll(n), total);
  return hipGetLastError();
}

}  // namespace phx
