// ckks.hip — sampling and small CKKS helper kernels (see ckks.h).
#include "ckks.h"

#include <algorithm>

#include "arith.h"
#include "chacha.h"

namespace phx {
namespace {

constexpr int kBlock = 256;

// Draw `nonce` of a ChaCha20 stream: block b holds 8 64-bit words.
// uniform: element e of [L][n] takes words 2(e mod 4), 2(e mod 4) + 1 of block e / 4, a 128-bit
// value reduced mod q (statistical distance from uniform < q / 2^128).
__global__ __launch_bounds__(kBlock) void uniform_kernel(uint64_t* out, const uint64_t* q, const uint64_t* barrett,
                                                         uint32_t log_n, size_t blocks, ChaChaKey key, uint64_t nonce) {
  for (size_t b = blockIdx.x * (size_t)kBlock + threadIdx.x; b < blocks; b += (size_t)gridDim.x * kBlock) {
    uint32_t w[16];
    chacha20_block(key, b, nonce, w);
    const uint32_t l = static_cast<uint32_t>((4 * b) >> log_n);  // n >= 4: the 4 elements share a limb
    const uint64_t ql = q[l], r0 = barrett[2 * l], r1 = barrett[2 * l + 1];
    uint64_t v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = barrett_reduce_128(u128{chacha_word64(w, 2 * i), chacha_word64(w, 2 * i + 1)}, ql, r0, r1);
    *reinterpret_cast<ulonglong2*>(out + 4 * b) = make_ulonglong2(v[0], v[1]);
    *reinterpret_cast<ulonglong2*>(out + 4 * b + 2) = make_ulonglong2(v[2], v[3]);
  }
}

// the reference's uniform expansion of a public 64-byte seed (sample_uniform_poly,
// src/prng.cu:164-197; salsa.h): thread t < (n / 8) L fills 8 coefficients of limb t / (n / 8)
// from the block of nonce t, rejecting words above max_multiple by replacing the whole block
// with the one of nonce t + tries n L.  barrett[2 l + 1] = floor(2^64 / q): the exact 64-bit
// remainder of barrett_reduce_64.
__global__ __launch_bounds__(kBlock) void uniform_salsa_kernel(uint64_t* out, const uint64_t* q,
                                                               const uint64_t* barrett, uint32_t log_n, size_t L,
                                                               SalsaSeed seed) {
  const size_t per = (size_t(1) << log_n) >> 3, total = per * L, nl = L << log_n;
  for (size_t t = blockIdx.x * (size_t)kBlock + threadIdx.x; t < total; t += (size_t)gridDim.x * kBlock) {
    const size_t l = t / per;
    const uint64_t ql = q[l], r1 = barrett[2 * l + 1];
    const uint64_t max_multiple = ~uint64_t(0) - barrett_reduce_64(~uint64_t(0), ql, r1) - 1;
    uint32_t w[16];
    salsa20_block(seed, t, w);
    uint64_t tries = 1;
    uint64_t v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint64_t r = static_cast<uint64_t>(w[2 * i]) | (static_cast<uint64_t>(w[2 * i + 1]) << 32);
      while (r > max_multiple) {
        salsa20_block(seed, t + tries * nl, w);
        ++tries;
        r = static_cast<uint64_t>(w[2 * i]) | (static_cast<uint64_t>(w[2 * i + 1]) << 32);
      }
      v[i] = barrett_reduce_64(r, ql, r1);
    }
#pragma unroll
    for (int i = 0; i < 8; i += 2) *reinterpret_cast<ulonglong2*>(out + 8 * t + i) = make_ulonglong2(v[i], v[i + 1]);
  }
}

// small signed samples, one 64-bit word per coefficient k (block k / 8), the same value written
// to every limb: MODE 0 centered binomial (21 + 21 bits, sigma = sqrt(10.5) ~ 3.24, as the
// reference's sample_error_poly draws a CBD), MODE 1 ternary {-1, 0, 1} uniform (word mod 3,
// bias < 2^-62; sample_ternary_poly)
template <int MODE>
__global__ __launch_bounds__(kBlock) void small_kernel(uint64_t* out, const uint64_t* q, uint32_t log_n, uint32_t L,
                                                       size_t blocks, ChaChaKey key, uint64_t nonce) {
  const size_t n = size_t(1) << log_n;
  for (size_t b = blockIdx.x * (size_t)kBlock + threadIdx.x; b < blocks; b += (size_t)gridDim.x * kBlock) {
    uint32_t w[16];
    chacha20_block(key, b, nonce, w);
    int v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t r = chacha_word64(w, i);
      if constexpr (MODE == 0) v[i] = __popcll(r & 0x1FFFFFull) - __popcll((r >> 21) & 0x1FFFFFull);
      else v[i] = static_cast<int>(r % 3) - 1;
    }
    const size_t k0 = 8 * b;
    if (k0 >= n) continue;
    const int cnt = n - k0 < 8 ? static_cast<int>(n - k0) : 8;
    for (uint32_t l = 0; l < L; ++l) {
      const uint64_t ql = q[l];
      for (int i = 0; i < cnt; ++i) out[(size_t)l * n + k0 + i] = v[i] >= 0 ? static_cast<uint64_t>(v[i]) : ql - static_cast<uint64_t>(-v[i]);
    }
  }
}

__global__ __launch_bounds__(kBlock) void mul_scalar_add_kernel(const uint64_t* in, const uint64_t* c,
                                                                const uint64_t* cs, const uint64_t* acc, uint64_t* out,
                                                                const uint64_t* q, uint32_t log_n, size_t total,
                                                                size_t poly_stride) {
  // blockIdx.y: polynomial (acc and out at y poly_stride; `in` shared)
  if (acc) acc += blockIdx.y * poly_stride;
  out += blockIdx.y * poly_stride;
  for (size_t e = blockIdx.x * (size_t)kBlock + threadIdx.x; e < total; e += (size_t)gridDim.x * kBlock) {
    const uint32_t l = static_cast<uint32_t>(e >> log_n);
    const uint64_t ql = q[l];
    uint64_t v = mul_shoup(in[e], c[l], cs[l], ql);
    if (acc) v = add_mod(v, acc[e], ql);
    out[e] = v;
  }
}

// One element (limb l, coefficient k) per thread and grid-stride step.  Babies are split into
// 30-bit halves once; each giant step issues all G plaintext loads together (the pointer row
// is one scalar block: no branches between the loads) and accumulates the 4 partial products
// of every term in 64-bit sums, folded to 128 bits every kChunk terms and Barrett-reduced once
// per output.  Inputs below q < 2^60 split into halves below 2^30, so 16 products stay below
// 2^64; with a 61-bit modulus the high halves reach 2^31 (products up to 2^62) and only 4 fit
// (Q60 = LtArgs::q60).
template <int G, bool Q60>
__global__ __launch_bounds__(kBlock, 2) void lt_bsgs_kernel(LtArgs a, uint32_t log_n, size_t total) {
  constexpr uint64_t kM30 = (1ull << 30) - 1;
  constexpr int kChunk = Q60 ? 16 : 4;
  // the [b][g] plaintext pointer table, staged in LDS once per workgroup (a global read of it
  // per giant step would add a memory round trip before the plaintext loads can issue)
  extern __shared__ const uint64_t* ptab[];
  for (int k = threadIdx.x; k < a.b * G; k += kBlock) ptab[k] = a.pts[k];
  __syncthreads();
  const size_t pstride = total;  // elements per polynomial ([Ql + P][n])
  for (size_t e = blockIdx.x * (size_t)kBlock + threadIdx.x; e < total; e += (size_t)gridDim.x * kBlock) {
    const int l = static_cast<int>(e >> log_n);
    const int row = l < a.Ql ? l : a.size_Q + (l - a.Ql);
    const uint64_t q = a.q[row], r0 = a.barrett[2 * row], r1 = a.barrett[2 * row + 1];
    uint32_t xl[2][G], xh[2][G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const uint64_t v0 = a.baby[j][e], v1 = a.baby[j][pstride + e];
      xl[0][j] = static_cast<uint32_t>(v0 & kM30);
      xh[0][j] = static_cast<uint32_t>(v0 >> 30);
      xl[1][j] = static_cast<uint32_t>(v1 & kM30);
      xh[1][j] = static_cast<uint32_t>(v1 >> 30);
    }
    for (int i = 0; i < a.b; ++i) {
      const uint64_t* const* prow = ptab + i * G;
      u128 acc[2] = {{0, 0}, {0, 0}};
#pragma unroll
      for (int c0 = 0; c0 < G; c0 += kChunk) {
        constexpr int C = G < kChunk ? G : kChunk;
        uint64_t w[C];
        // global (not flat) loads: they count in vmcnt only, so the LDS pointer reads between
        // them do not wait for the plaintext data
#pragma unroll
        for (int j = 0; j < C; ++j) w[j] = ((const __attribute__((address_space(1))) uint64_t*)prow[c0 + j])[e];
        // keep the chunk's loads together in flight: the scheduler would otherwise sink each load
        // to its first use (one memory round trip per term)
        __builtin_amdgcn_sched_barrier(0);
        uint64_t ll[2] = {0, 0}, m1[2] = {0, 0}, m2[2] = {0, 0}, hh[2] = {0, 0};
#pragma unroll
        for (int jj = 0; jj < C; ++jj) {
          const int j = c0 + jj;
          const uint32_t wl = static_cast<uint32_t>(w[jj] & kM30), wh = static_cast<uint32_t>(w[jj] >> 30);
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            ll[t] += static_cast<uint64_t>(xl[t][j]) * wl;
            m1[t] += static_cast<uint64_t>(xl[t][j]) * wh;
            m2[t] += static_cast<uint64_t>(xh[t][j]) * wl;
            hh[t] += static_cast<uint64_t>(xh[t][j]) * wh;
          }
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          add128(acc[t], u128{ll[t], 0});
          add128(acc[t], u128{m1[t] << 30, m1[t] >> 34});
          add128(acc[t], u128{m2[t] << 30, m2[t] >> 34});
          add128(acc[t], u128{hh[t] << 60, hh[t] >> 4});
        }
      }
      uint64_t* o = a.out[i];
      o[e] = barrett_reduce_128(acc[0], q, r0, r1);
      o[pstride + e] = barrett_reduce_128(acc[1], q, r0, r1);
    }
  }
}

// where the babies and the inner sums of one ciphertext live: LtArgs' pointer arrays, or the
// group form's contiguous buffers (baby j at baby0 + j baby_stride, inner sum i >= 1 at
// giant1 + (i - 1) giant_stride, inner sum 0 at acc)
struct LtSingleSrc {
  const LtArgs& a;
  __device__ const uint64_t* baby(int j) const { return a.baby[j]; }
  __device__ uint64_t* out(int i) const { return a.out[i]; }
};
struct LtGroupSrc {
  const LtGroupArgs& a;
  int c;
  __device__ const uint64_t* baby(int j) const { return a.baby0[c] + static_cast<size_t>(j) * a.baby_stride; }
  __device__ uint64_t* out(int i) const {
    return i == 0 ? a.acc[c] : a.giant1[c] + static_cast<size_t>(i - 1) * a.giant_stride;
  }
};

// G = 32 baby steps, at most 8 giant steps (the bootstrap's CoeffToSlot / SlotToCoeff levels):
// one workgroup = 8 waves over one tile of 64 E elements (E consecutive elements per lane, one
// 8E-byte load per lane), wave i computing giant step i.  The tile's 64 baby rows (32 babies x 2
// polynomials) are staged once in LDS as 30-bit halves (32 E KB); each wave then streams only its
// own 32 plaintexts, 4 at a time, double-buffered: chunk c + 1's loads are in flight while chunk
// c's products run, and chunk 0's over the staging barrier.  The register-resident form this
// replaces held all 8 giant steps' 128-bit sums per lane (220 VGPRs, 8 waves per CU) and read HBM
// at 4.7 TB/s.  Each baby and each plaintext is still read from HBM once; the sums are exact
// 128-bit values, so every result is bit-identical to lt_bsgs_kernel's.
#ifndef PHX_LT_EPL
#define PHX_LT_EPL 2
#endif
#ifndef PHX_LT_DEPTH
#define PHX_LT_DEPTH 2
#endif
constexpr int kLtWaves = 8, kLtChunk = 4, kLtEpl = PHX_LT_EPL, kLtDepth = PHX_LT_DEPTH;
static_assert(kLtDepth >= 2 && kLtDepth <= 4, "2 to 4 plaintext chunks in flight");
static_assert(kLtEpl == 1 || kLtEpl == 2, "1 or 2 elements per lane");

template <int E>
struct LtVec;  // E consecutive u64 of one lane
template <>
struct LtVec<1> {
  uint64_t v[1];
};
template <>
struct LtVec<2> {
  uint64_t v[2];
};

template <int E>
__device__ __forceinline__ LtVec<E> lt_ld(const uint64_t* p) {
  LtVec<E> r;
  if constexpr (E == 2) {
    typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
    const u64x2 x = *(const __attribute__((address_space(1))) u64x2*)p;
    r.v[0] = x.x;
    r.v[1] = x.y;
  } else {
    r.v[0] = *(const __attribute__((address_space(1))) uint64_t*)p;
  }
  return r;
}

using LtPtr = const __attribute__((address_space(4))) uint64_t*;

// chunk c (plaintexts 4c .. 4c + 3) of this wave's giant step
template <int E>
__device__ __forceinline__ void lt_load_chunk(LtVec<E> (&w)[kLtChunk], const __attribute__((address_space(4))) LtPtr* prow,
                                              int c, size_t e) {
#pragma unroll
  for (int j = 0; j < kLtChunk; ++j) w[j] = lt_ld<E>((const uint64_t*)prow[c * kLtChunk + j] + e);
}

// the four 64-bit partial sums of x * w per element and polynomial, x and w split in 30-bit halves
struct LtPart {
  uint64_t ll, m1, m2, hh;
};

// part += sum_j baby(4c + j) * w[j], the babies from LDS.  Folded every 2 chunks (8 products per
// partial sum) when every modulus is below 2^60 (each product < 2^60, the sum < 2^63), every chunk
// otherwise (61-bit moduli: a high-half product < 2^62, 4 of them < 2^64).  The memory clobbers
// (IR) and scheduling barriers (machine code) keep this chunk's LDS reads and products inside it,
// and binding the partial sums to the closing asm stops the products being deferred: hoisted to
// the top of the kernel the LDS reads alone cost 128 VGPRs.
template <int E>
__device__ __forceinline__ void lt_chunk_products(LtPart (&part)[E][2], const LtVec<E> (&w)[kLtChunk],
                                                  const uint2 (*xs)[64 * E], int c, int lane) {
  constexpr uint64_t kM30 = (1ull << 30) - 1;
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int jj = 0; jj < kLtChunk; ++jj) {
    const int j = c * kLtChunk + jj;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      uint2 x[E];
      if constexpr (E == 2) {
        const uint4 xx = *reinterpret_cast<const uint4*>(&xs[2 * j + t][2 * lane]);
        x[0] = make_uint2(xx.x, xx.y);
        x[1] = make_uint2(xx.z, xx.w);
      } else {
        x[0] = xs[2 * j + t][lane];
      }
#pragma unroll
      for (int k = 0; k < E; ++k) {
        const uint32_t wl = static_cast<uint32_t>(w[jj].v[k] & kM30), wh = static_cast<uint32_t>(w[jj].v[k] >> 30);
        LtPart& P = part[k][t];
        P.ll += static_cast<uint64_t>(x[k].x) * wl;
        P.m1 += static_cast<uint64_t>(x[k].x) * wh;
        P.m2 += static_cast<uint64_t>(x[k].y) * wl;
        P.hh += static_cast<uint64_t>(x[k].y) * wh;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < E; ++k)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      LtPart& P = part[k][t];
      asm volatile("" : "+v"(P.ll), "+v"(P.m1), "+v"(P.m2), "+v"(P.hh)::"memory");
    }
  __builtin_amdgcn_sched_barrier(0);
}

template <int E>
__device__ __forceinline__ void lt_fold(u128 (&acc)[E][2], LtPart (&part)[E][2]) {
#pragma unroll
  for (int k = 0; k < E; ++k)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      LtPart& P = part[k][t];
      add128(acc[k][t], u128{P.ll, 0});
      add128(acc[k][t], u128{P.m1 << 30, P.m1 >> 34});
      add128(acc[k][t], u128{P.m2 << 30, P.m2 >> 34});
      add128(acc[k][t], u128{P.hh << 60, P.hh >> 4});
      P = LtPart{0, 0, 0, 0};
      // folded here, not all at the end (which would keep every fold's partial sums live)
      asm volatile("" : "+v"(acc[k][t].lo), "+v"(acc[k][t].hi));
    }
}

template <int E, bool Q60, class Src>
__device__ __forceinline__ void lt_bsgs_tile(const Src& src, int nb, int Ql, int size_Q, const uint64_t* qv,
                                             const uint64_t* barrett, uint32_t log_n, size_t total, size_t tile,
                                             const uint64_t* const* pts) {
  constexpr int G = 32, T = 64 * E, NC = G / kLtChunk;
  constexpr uint64_t kM30 = (1ull << 30) - 1;
  __shared__ uint2 xs[2 * G][T];  // row 2j + t: baby j, polynomial t, as {low 30, high 30} bits
  // a memory clobber ahead of the loads: it keeps them where they are written
  asm volatile("" ::: "memory");
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const size_t e = tile * T + static_cast<size_t>(lane) * E;
  // staging: wave wv loads polynomial wv & 1 of babies (wv >> 1) + 4r, r < 8 (rows wv + 8r)
  LtVec<E> v[8];
  const size_t poff = static_cast<size_t>(wv & 1) * total + e;
#pragma unroll
  for (int r = 0; r < 8; ++r) v[r] = lt_ld<E>(src.baby((wv >> 1) + 4 * r) + poff);
  __builtin_amdgcn_sched_barrier(0);  // the babies' loads first: the staging writes wait for them only
  // waves past the last giant step repeat the last one (its plaintexts come from L2, and they
  // store the same values to the same places): with a branch around their loads and products the
  // backend sinks the plaintext loads past the barrier, or makes the staging writes wait for them
  const int wi = wv < nb ? wv : nb - 1;
  const __attribute__((address_space(4))) LtPtr* prow = (const __attribute__((address_space(4))) LtPtr*)(pts + wi * G);
  constexpr int D = kLtDepth;  // plaintext chunks in flight
  LtVec<E> wbuf[D][kLtChunk];
#pragma unroll
  for (int c = 0; c + 1 < D; ++c) lt_load_chunk<E>(wbuf[c], prow, c, e);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int k = 0; k < E; ++k)
      xs[wv + 8 * r][lane * E + k] =
          make_uint2(static_cast<uint32_t>(v[r].v[k] & kM30), static_cast<uint32_t>(v[r].v[k] >> 30));
  // LDS writes done, then the workgroup barrier; the plaintext loads stay in flight (a
  // __syncthreads would also drain vmcnt)
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), vmcnt and expcnt unconstrained
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  u128 acc[E][2];
  LtPart part[E][2];
#pragma unroll
  for (int k = 0; k < E; ++k)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      acc[k][t] = u128{0, 0};
      part[k][t] = LtPart{0, 0, 0, 0};
    }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (c + D - 1 < NC) lt_load_chunk<E>(wbuf[(c + D - 1) % D], prow, c + D - 1, e);
    lt_chunk_products<E>(part, wbuf[c % D], xs, c, lane);
    if ((c & 1) || !Q60) lt_fold<E>(acc, part);  // 8 (q < 2^60) or 4 products per partial sum
  }
  const int l = static_cast<int>((tile * T) >> log_n);
  const int row = l < Ql ? l : size_Q + (l - Ql);
  const uint64_t q = qv[row], r0 = barrett[2 * row], r1 = barrett[2 * row + 1];
  uint64_t* o = src.out(wi);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if constexpr (E == 2) {
      *reinterpret_cast<ulong2*>(o + t * total + e) =
          make_ulong2(barrett_reduce_128(acc[0][t], q, r0, r1), barrett_reduce_128(acc[1][t], q, r0, r1));
    } else {
      o[t * total + e] = barrett_reduce_128(acc[0][t], q, r0, r1);
    }
  }
}

template <int E, bool Q60>
__global__ __launch_bounds__(64 * kLtWaves) void lt_bsgs_tile_kernel(LtArgs a, uint32_t log_n, size_t total) {
  lt_bsgs_tile<E, Q60>(LtSingleSrc{a}, a.b, a.Ql, a.size_Q, a.q, a.barrett, log_n, total, blockIdx.x, a.pts);
}

// `count` ciphertexts through the same plaintexts (lt_bsgs_group): the workgroups of the
// ciphertexts that cover the same tile are dealt to one XCD 8 dispatches apart (workgroups w and
// w + 8 share an XCD under round-robin placement), so the followers' plaintext reads are served by
// that XCD's L2
template <int E, bool Q60>
__global__ __launch_bounds__(64 * kLtWaves) void lt_bsgs_group_kernel(LtGroupArgs ga, uint32_t log_n, size_t total) {
  const uint32_t K = static_cast<uint32_t>(ga.count);
  const uint32_t b = blockIdx.x, x = b % 8, k = b / 8;
  const uint32_t c = k % K, tile = (k / K) * 8 + x;
  if (static_cast<size_t>(tile) * 64 * E >= total) return;  // the grid rounds the tiles up to whole XCD rounds
  lt_bsgs_tile<E, Q60>(LtGroupSrc{ga, static_cast<int>(c)}, ga.b, ga.Ql, ga.size_Q, ga.q, ga.barrett, log_n, total, tile,
                  ga.pts);
}

// 16-byte global accesses of two consecutive elements
typedef uint64_t tl_u64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ tl_u64x2 tl_ld2(const uint64_t* p) {
  return *(const __attribute__((address_space(1))) tl_u64x2*)p;
}
__device__ __forceinline__ void tl_st2(uint64_t* p, uint64_t x, uint64_t y) {
  tl_u64x2 v;
  v.x = x;
  v.y = y;
  *(__attribute__((address_space(1))) tl_u64x2*)p = v;
}

template <bool MUL, bool ACC>
__global__ __launch_bounds__(kBlock) void scalar_v_kernel(const uint64_t* in, size_t in_stride, LimbScalars c,
                                                          const uint64_t* acc, uint64_t* out, const uint64_t* q,
                                                          uint32_t log_n, size_t total) {
  in += blockIdx.y * in_stride;
  out += blockIdx.y * total;
  if constexpr (ACC) acc += blockIdx.y * total;
  // two elements per thread, 16-byte accesses (n even: a pair shares its limb)
  for (size_t e = 2 * (blockIdx.x * (size_t)kBlock + threadIdx.x); e < total; e += 2 * (size_t)gridDim.x * kBlock) {
    const uint32_t l = static_cast<uint32_t>(e >> log_n);
    const uint64_t ql = q[l], cv = c.v[l];
    const tl_u64x2 x = tl_ld2(in + e);
    uint64_t v[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) v[u] = MUL ? mul_shoup(x[u], cv, c.vs[l], ql) : add_mod(x[u], cv, ql);
    if constexpr (ACC) {
      const tl_u64x2 y = tl_ld2(acc + e);
#pragma unroll
      for (int u = 0; u < 2; ++u) v[u] = add_mod(v[u], y[u], ql);
    }
    tl_st2(out + e, v[0], v[1]);
  }
}

// blockIdx.y: polynomial p < d_polys of d ([d_polys][L][n]):
//   d[p] = d[p] * ca (if SCALE) + (p < t_polys ? t[p] * cb : 0),  t[p] at t + p * t_stride
template <bool SCALE>
__global__ __launch_bounds__(kBlock) void lin_comb_kernel(uint64_t* d, LimbScalars ca, const uint64_t* t,
                                                          uint32_t t_polys, size_t t_stride, LimbScalars cb,
                                                          const uint64_t* q, uint32_t log_n, size_t total) {
  d += blockIdx.y * total;
  const bool with_t = t != nullptr && blockIdx.y < t_polys;
  if (with_t) t += blockIdx.y * t_stride;
  if (!SCALE && !with_t) return;
  for (size_t e = blockIdx.x * (size_t)kBlock + threadIdx.x; e < total; e += (size_t)gridDim.x * kBlock) {
    const uint32_t l = static_cast<uint32_t>(e >> log_n);
    const uint64_t ql = q[l];
    uint64_t v = d[e];
    if constexpr (SCALE) v = mul_shoup(v, ca.v[l], ca.vs[l], ql);
    if (with_t) v = add_mod(v, mul_shoup(t[e], cb.v[l], cb.vs[l], ql), ql);
    d[e] = v;
  }
}

// blockIdx.y = limb l, blockIdx.x strides over the 2 n elements (t, k) of that limb.  The
// limb's coefficients sit in LDS split into 30-bit halves; every output is sum_k x_k c_mk as
// four 64-bit partial sums of 30-bit products (<= 16 terms: no overflow), one Barrett per output.
template <int K>
__global__ __launch_bounds__(kBlock) void leaf_combine_kernel(LeafArgs a, uint32_t log_n) {
  constexpr uint64_t kM30 = (1ull << 30) - 1;
  __shared__ uint32_t clo[kLeafMaxM][K], chi[kLeafMaxM][K];
  __shared__ uint64_t cadd[kLeafMaxM];
  const int l = blockIdx.y;
  const size_t n = size_t(1) << log_n;
  for (int e = threadIdx.x; e < a.M * K; e += kBlock) {
    const int m = e / K, k = e % K;
    const uint64_t c = a.coef[(static_cast<size_t>(m) * K + k) * a.L + l];
    clo[m][k] = static_cast<uint32_t>(c & kM30);
    chi[m][k] = static_cast<uint32_t>(c >> 30);
  }
  if (threadIdx.x < a.M) cadd[threadIdx.x] = a.cadd[static_cast<size_t>(threadIdx.x) * a.L + l];
  __syncthreads();
  const uint64_t q = a.q[l], r0 = a.barrett[2 * l], r1 = a.barrett[2 * l + 1];
  const size_t ln = static_cast<size_t>(a.L) << log_n;
  for (size_t e = blockIdx.x * (size_t)kBlock + threadIdx.x; e < 2 * n; e += (size_t)gridDim.x * kBlock) {
    const uint32_t t = e >= n ? 1 : 0;
    const size_t el = (static_cast<size_t>(l) << log_n) + (e - t * n);  // offset inside the polynomial
    uint32_t xl[K], xh[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint64_t v = a.in[k][t * a.in_stride[k] + el];
      xl[k] = static_cast<uint32_t>(v & kM30);
      xh[k] = static_cast<uint32_t>(v >> 30);
    }
    for (int m = 0; m < a.M; ++m) {
      uint64_t ll = 0, m1 = 0, m2 = 0, hh = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const uint32_t cl = clo[m][k], ch = chi[m][k];
        ll += static_cast<uint64_t>(xl[k]) * cl;
        m1 += static_cast<uint64_t>(xl[k]) * ch;
        m2 += static_cast<uint64_t>(xh[k]) * cl;
        hh += static_cast<uint64_t>(xh[k]) * ch;
      }
      u128 acc{ll, 0};
      add128(acc, u128{m1 << 30, m1 >> 34});
      add128(acc, u128{m2 << 30, m2 >> 34});
      add128(acc, u128{hh << 60, hh >> 4});
      uint64_t v = barrett_reduce_128(acc, q, r0, r1);
      if (t == 0) v = add_mod(v, cadd[m], q);
      a.out[m][t * ln + el] = v;
    }
  }
}

// tensor product with the fused linear epilogue of MulAddRescale (see ckks.h)
template <bool SCALE, bool TERM>
__global__ __launch_bounds__(kBlock) void tensor_lin_kernel(TensorLinArgs a, uint32_t log_n, size_t total) {
  const size_t stride = total;  // elements per polynomial
  for (size_t e = blockIdx.x * (size_t)kBlock + threadIdx.x; e < total; e += (size_t)gridDim.x * kBlock) {
    const uint32_t l = static_cast<uint32_t>(e >> log_n);
    const uint64_t q = a.q[l], r0 = a.barrett[2 * l], r1 = a.barrett[2 * l + 1];
    const uint64_t a0 = a.ct1[e], a1 = a.ct1[stride + e], b0 = a.ct2[e], b1 = a.ct2[stride + e];
    u128 c1 = mul_wide(a0, b1);
    add128(c1, mul_wide(a1, b0));
    uint64_t d0 = mul_mod(a0, b0, q, r0, r1), d1 = barrett_reduce_128(c1, q, r0, r1), d2 = mul_mod(a1, b1, q, r0, r1);
    if constexpr (SCALE) {
      d0 = mul_shoup(d0, a.f.v[l], a.f.vs[l], q);
      d1 = mul_shoup(d1, a.f.v[l], a.f.vs[l], q);
      d2 = mul_shoup(d2, a.f.v[l], a.f.vs[l], q);
    }
    if constexpr (TERM) {
      d0 = add_mod(d0, mul_shoup(a.t[e], a.c.v[l], a.c.vs[l], q), q);
      d1 = add_mod(d1, mul_shoup(a.t[a.t_stride + e], a.c.v[l], a.c.vs[l], q), q);
    }
    a.out[e] = d0;
    a.out[stride + e] = d1;
    a.out[2 * stride + e] = d2;
  }
}

// tensor_lin over the products of one batch: grid row blockIdx.y = product (see ckks.h).  Two
// elements per thread and 16-byte accesses; the factor 2 (the EvalMod products' only factor
// besides 1) is a modular doubling instead of a 128-bit product and Barrett reduction.

__global__ __launch_bounds__(kBlock) void tensor_lin_batch_kernel(TensorLinBatchArgs a, uint32_t log_n, size_t total) {
  const uint32_t k = blockIdx.y;
  const TensorLinJob& J = a.job[k];
  const uint64_t* cl = a.limb + static_cast<size_t>(k) * 2 * a.L;
  const size_t stride = total;
  const bool dbl = J.factor == 2, scaled = J.factor != 1;  // product-uniform branches
  for (size_t e = 2 * (blockIdx.x * (size_t)kBlock + threadIdx.x); e < total; e += 2 * (size_t)gridDim.x * kBlock) {
    const uint32_t l = static_cast<uint32_t>(e >> log_n);  // (n even: the pair shares a limb)
    const uint64_t q = a.q[l], r0 = a.barrett[2 * l], r1 = a.barrett[2 * l + 1];
    const tl_u64x2 A0 = tl_ld2(J.ct1 + e), A1 = tl_ld2(J.ct1 + stride + e);
    const tl_u64x2 B0 = tl_ld2(J.ct2 + e), B1 = tl_ld2(J.ct2 + stride + e);
    tl_u64x2 T0, T1;
    if (J.t) {
      T0 = tl_ld2(J.t + e);
      T1 = tl_ld2(J.t + J.t_stride + e);
    }
    uint64_t d[3][2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint64_t a0 = A0[u], a1 = A1[u], b0 = B0[u], b1 = B1[u];
      u128 c1 = mul_wide(a0, b1);
      add128(c1, mul_wide(a1, b0));
      d[0][u] = mul_mod(a0, b0, q, r0, r1);
      d[1][u] = barrett_reduce_128(c1, q, r0, r1);
      d[2][u] = mul_mod(a1, b1, q, r0, r1);
    }
    if (dbl) {
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int u = 0; u < 2; ++u) d[p][u] = add_mod(d[p][u], d[p][u], q);
    } else if (scaled) {
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int u = 0; u < 2; ++u) d[p][u] = mul_mod(d[p][u], J.factor, q, r0, r1);
    }
    if (J.t) {
      const uint64_t c = cl[l];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        d[0][u] = add_mod(d[0][u], mul_mod(T0[u], c, q, r0, r1), q);
        d[1][u] = add_mod(d[1][u], mul_mod(T1[u], c, q, r0, r1), q);
      }
    }
    if (J.has_const) {
      const uint64_t cc = cl[a.L + l];
#pragma unroll
      for (int u = 0; u < 2; ++u) d[0][u] = add_mod(d[0][u], cc, q);
    }
    tl_st2(J.out + e, d[0][0], d[0][1]);
    tl_st2(J.out + stride + e, d[1][0], d[1][1]);
    tl_st2(J.out + 2 * stride + e, d[2][0], d[2][1]);
  }
}

int grid_for(size_t items) {
  const size_t b = (items + kBlock - 1) / kBlock;
  return static_cast<int>(std::max<size_t>(1, std::min<size_t>(b, 2048)));
}

}  // namespace

hipError_t sample_uniform(uint64_t* out, const uint64_t* q, const uint64_t* barrett, size_t n, size_t L,
                          const ChaChaKey& key, uint64_t nonce, hipStream_t s) {
  if (n < 8 || (n & (n - 1))) return hipErrorInvalidValue;
  const size_t blocks = n * L / 4;
  uniform_kernel<<<grid_for(blocks), kBlock, 0, s>>>(out, q, barrett, __builtin_ctzll(n), blocks, key, nonce);
  return hipGetLastError();
}

hipError_t sample_uniform_seeded(uint64_t* out, const uint64_t* q, const uint64_t* barrett, size_t n, size_t L,
                                 const SalsaSeed& seed, hipStream_t s) {
  if (n < 8 || (n & (n - 1))) return hipErrorInvalidValue;
  uniform_salsa_kernel<<<grid_for(n / 8 * L), kBlock, 0, s>>>(out, q, barrett, __builtin_ctzll(n), L, seed);
  return hipGetLastError();
}

hipError_t sample_cbd(uint64_t* out, const uint64_t* q, size_t n, size_t L, const ChaChaKey& key, uint64_t nonce,
                      hipStream_t s) {
  if (n < 8 || (n & (n - 1))) return hipErrorInvalidValue;
  const size_t blocks = n / 8;
  small_kernel<0><<<grid_for(blocks), kBlock, 0, s>>>(out, q, __builtin_ctzll(n), static_cast<uint32_t>(L), blocks, key,
                                                     nonce);
  return hipGetLastError();
}

hipError_t sample_ternary(uint64_t* out, const uint64_t* q, size_t n, size_t L, const ChaChaKey& key, uint64_t nonce,
                          hipStream_t s) {
  if (n < 8 || (n & (n - 1))) return hipErrorInvalidValue;
  const size_t blocks = n / 8;
  small_kernel<1><<<grid_for(blocks), kBlock, 0, s>>>(out, q, __builtin_ctzll(n), static_cast<uint32_t>(L), blocks, key,
                                                     nonce);
  return hipGetLastError();
}

hipError_t mul_scalar_add(const uint64_t* in, const uint64_t* c, const uint64_t* c_shoup, const uint64_t* acc,
                          uint64_t* out, const uint64_t* q, size_t n, size_t L, hipStream_t s) {
  const size_t total = n * L;
  mul_scalar_add_kernel<<<grid_for(total), kBlock, 0, s>>>(in, c, c_shoup, acc, out, q, __builtin_ctzll(n), total, 0);
  return hipGetLastError();
}

hipError_t mul_scalar_accumulate(const uint64_t* in, const uint64_t* c, const uint64_t* c_shoup, uint64_t* out,
                                 size_t poly_stride, size_t polys, const uint64_t* q, size_t n, size_t L, hipStream_t s) {
  const size_t total = n * L;
  if (polys == 0 || total == 0) return hipSuccess;
  if (polys > 65535) return hipErrorInvalidValue;  // grid.y
  const dim3 grid(static_cast<unsigned>(std::max<size_t>(1, grid_for(total) / polys)), static_cast<unsigned>(polys));
  mul_scalar_add_kernel<<<grid, kBlock, 0, s>>>(in, c, c_shoup, out, out, q, __builtin_ctzll(n), total, poly_stride);
  return hipGetLastError();
}

hipError_t lt_bsgs(const LtArgs& a, size_t n, hipStream_t s) {
  if (a.g < 1 || a.g > kLtMaxG || a.b < 1 || a.b > kLtMaxB || a.pts == nullptr) return hipErrorInvalidValue;
  for (int i = 0; i < a.b; ++i)
    if (!a.out[i]) return hipErrorInvalidValue;
  const size_t total = n * static_cast<size_t>(a.Ql + a.P);
  const uint32_t log_n = __builtin_ctzll(n);
  const int grid = grid_for(total);
  const size_t lds = static_cast<size_t>(a.b) * a.g * sizeof(const uint64_t*);
  const bool tile = a.g == 32 && a.b <= kLtWaves && n >= 64 * kLtEpl;
#define PHX_LT_CASES(Q)                                                                                         \
  switch (a.g) {                                                                                                \
    case 1: lt_bsgs_kernel<1, Q><<<grid, kBlock, lds, s>>>(a, log_n, total); break;                            \
    case 2: lt_bsgs_kernel<2, Q><<<grid, kBlock, lds, s>>>(a, log_n, total); break;                            \
    case 4: lt_bsgs_kernel<4, Q><<<grid, kBlock, lds, s>>>(a, log_n, total); break;                            \
    case 8: lt_bsgs_kernel<8, Q><<<grid, kBlock, lds, s>>>(a, log_n, total); break;                            \
    case 16: lt_bsgs_kernel<16, Q><<<grid, kBlock, lds, s>>>(a, log_n, total); break;                          \
    case 32:                                                                                                    \
      if (tile)                                                                                                 \
        lt_bsgs_tile_kernel<kLtEpl, Q>                                                                          \
            <<<static_cast<unsigned>(total / (64 * kLtEpl)), 64 * kLtWaves, 0, s>>>(a, log_n, total);           \
      else                                                                                                      \
        lt_bsgs_kernel<32, Q><<<grid, kBlock, lds, s>>>(a, log_n, total);                                       \
      break;                                                                                                    \
    default: return hipErrorInvalidValue;                                                                       \
  }
  if (a.q60) {
    PHX_LT_CASES(true)
  } else {
    PHX_LT_CASES(false)
  }
#undef PHX_LT_CASES
  return hipGetLastError();
}

hipError_t lt_bsgs_group(const LtGroupArgs& ga, size_t n, hipStream_t s) {
  if (ga.count < 2 || ga.count > kLtGroupMax || ga.g != 32 || ga.b < 1 || ga.b > 8 || !ga.pts || !ga.q || !ga.barrett)
    return hipErrorInvalidValue;
  for (int c = 0; c < ga.count; ++c)
    if (!ga.baby0[c] || !ga.acc[c] || (ga.b > 1 && !ga.giant1[c])) return hipErrorInvalidValue;
  if (n < 64 * kLtEpl) return hipErrorInvalidValue;
  const size_t total = n * static_cast<size_t>(ga.Ql + ga.P);
  const size_t per = (total / (64 * kLtEpl) + 7) / 8 * 8;  // workgroups per ciphertext, whole XCD rounds
  const unsigned grid = static_cast<unsigned>(ga.count * per);
  if (ga.q60)
    lt_bsgs_group_kernel<kLtEpl, true><<<grid, 64 * kLtWaves, 0, s>>>(ga, __builtin_ctzll(n), total);
  else
    lt_bsgs_group_kernel<kLtEpl, false><<<grid, 64 * kLtWaves, 0, s>>>(ga, __builtin_ctzll(n), total);
  return hipGetLastError();
}

hipError_t tensor_lin(const TensorLinArgs& a, size_t n, size_t L, hipStream_t s) {
  if (L > static_cast<size_t>(kMaxScalarLimbs)) return hipErrorInvalidValue;
  const size_t total = n * L;
  const uint32_t log_n = __builtin_ctzll(n);
  const int grid = grid_for(total);
  if (a.scale && a.t) tensor_lin_kernel<true, true><<<grid, kBlock, 0, s>>>(a, log_n, total);
  else if (a.scale) tensor_lin_kernel<true, false><<<grid, kBlock, 0, s>>>(a, log_n, total);
  else if (a.t) tensor_lin_kernel<false, true><<<grid, kBlock, 0, s>>>(a, log_n, total);
  else tensor_lin_kernel<false, false><<<grid, kBlock, 0, s>>>(a, log_n, total);
  return hipGetLastError();
}

hipError_t tensor_lin_batch(const TensorLinBatchArgs& a, size_t n, hipStream_t s) {
  if (a.count < 1 || a.count > static_cast<uint32_t>(kTensorBatchMax) || a.L < 1 ||
      static_cast<size_t>(a.count) * 2 * a.L > static_cast<size_t>(kTensorBatchLimbWords) || !a.q || !a.barrett)
    return hipErrorInvalidValue;
  for (uint32_t k = 0; k < a.count; ++k)
    if (!a.job[k].ct1 || !a.job[k].ct2 || !a.job[k].out || a.job[k].factor == 0) return hipErrorInvalidValue;
  const size_t total = n * a.L;
  const dim3 grid(static_cast<unsigned>(std::max(1, grid_for(total) / static_cast<int>(a.count))), a.count);
  tensor_lin_batch_kernel<<<grid, kBlock, 0, s>>>(a, __builtin_ctzll(n), total);
  return hipGetLastError();
}

hipError_t leaf_combine(const LeafArgs& a, size_t n, hipStream_t s) {
  if (a.K < 1 || a.K > kLeafMaxK || a.M < 1 || a.M > kLeafMaxM || a.L < 1 || !a.coef || !a.cadd || !a.barrett)
    return hipErrorInvalidValue;
  const uint32_t log_n = __builtin_ctzll(n);
  // x: enough workgroups per limb to fill the chip, y: limb
  const unsigned gx = static_cast<unsigned>(std::max<int>(1, std::min<int>(2 * n / kBlock, grid_for(2 * n * a.L) / a.L)));
  const dim3 grid(gx, static_cast<unsigned>(a.L));
  switch (a.K) {
#define PHX_LEAF_CASE(K) \
  case K: leaf_combine_kernel<K><<<grid, kBlock, 0, s>>>(a, log_n); break;
    PHX_LEAF_CASE(1) PHX_LEAF_CASE(2) PHX_LEAF_CASE(3) PHX_LEAF_CASE(4) PHX_LEAF_CASE(5) PHX_LEAF_CASE(6)
    PHX_LEAF_CASE(7) PHX_LEAF_CASE(8) PHX_LEAF_CASE(9) PHX_LEAF_CASE(10) PHX_LEAF_CASE(11) PHX_LEAF_CASE(12)
    PHX_LEAF_CASE(13) PHX_LEAF_CASE(14) PHX_LEAF_CASE(15) PHX_LEAF_CASE(16)
#undef PHX_LEAF_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t lin_comb_v(uint64_t* d, size_t d_polys, const LimbScalars* ca, const uint64_t* t, size_t t_polys,
                      size_t t_stride, const LimbScalars& cb, const uint64_t* q, size_t n, size_t L, hipStream_t s) {
  if (L > static_cast<size_t>(kMaxScalarLimbs) || d_polys < 1 || t_polys > d_polys) return hipErrorInvalidValue;
  const size_t total = n * L;
  const dim3 g(std::max<int>(1, grid_for(total * d_polys) / static_cast<int>(d_polys)), static_cast<unsigned>(d_polys));
  const uint32_t log_n = __builtin_ctzll(n);
  if (ca)
    lin_comb_kernel<true><<<g, kBlock, 0, s>>>(d, *ca, t, static_cast<uint32_t>(t_polys), t_stride, cb, q, log_n, total);
  else
    lin_comb_kernel<false><<<g, kBlock, 0, s>>>(d, LimbScalars{}, t, static_cast<uint32_t>(t_polys), t_stride, cb, q,
                                                log_n, total);
  return hipGetLastError();
}

hipError_t mul_scalar_v(const uint64_t* in, const LimbScalars& c, uint64_t* out, const uint64_t* q, size_t n,
                        size_t L, hipStream_t s, size_t polys, size_t in_stride, const uint64_t* acc) {
  if (L > static_cast<size_t>(kMaxScalarLimbs) || polys < 1) return hipErrorInvalidValue;
  const size_t total = n * L;
  const dim3 g(std::max<int>(1, grid_for(total * polys) / static_cast<int>(polys)), static_cast<unsigned>(polys));
  const size_t is = in_stride ? in_stride : total;
  if (acc)
    scalar_v_kernel<true, true><<<g, kBlock, 0, s>>>(in, is, c, acc, out, q, __builtin_ctzll(n), total);
  else
    scalar_v_kernel<true, false><<<g, kBlock, 0, s>>>(in, is, c, nullptr, out, q, __builtin_ctzll(n), total);
  return hipGetLastError();
}

hipError_t add_scalar_v(const uint64_t* in, const LimbScalars& c, uint64_t* out, const uint64_t* q, size_t n,
                        size_t L, hipStream_t s) {
  if (L > static_cast<size_t>(kMaxScalarLimbs)) return hipErrorInvalidValue;
  const size_t total = n * L;
  scalar_v_kernel<false, false><<<grid_for(total), kBlock, 0, s>>>(in, total, c, nullptr, out, q, __builtin_ctzll(n),
                                                                    total);
  return hipGetLastError();
}

}  // namespace phx
