// ntt.hip — two-pass negacyclic NTT / INTT for gfx950.
//
// Decomposition (the same factorisation the reference's 2-D radix-8 NTT uses,
// src/ntt/fntt_2d.cu:9-198, re-designed for wave64 and 64-bit Shoup arithmetic):
//   n = S1 * S2.  The first log2(S1) Cooley-Tukey stages only pair elements of the same
//   column (index mod S2), the last log2(S2) stages only pair elements of the same row
//   (contiguous S2-element block).  Pass C ("column pass") runs the first stages on a
//   tile of COLS consecutive columns, pass R ("row pass") runs the last stages on a tile
//   of whole rows.  Each tile goes HBM -> registers -> (radix-16 rounds with LDS
//   transposes between them) -> LDS -> HBM with coalesced accesses.
//
// Stage g of a sub-transform of size S = 2^s pairs local indices p and p + S/2^(g+1)
// inside block iloc = p >> (s - g); the twiddle is tw[B * 2^g + iloc] with B = 1 for
// the column pass and B = S1 + row for the row pass, which is exactly the global
// table index m + i of the reference's in-place CT loop (m = 2^g or S1 * 2^g).
#include "ntt.h"

#include "arith.h"

namespace phx {
namespace {

constexpr int E_LOG = 4;  // elements per thread per round = 16 (radix-16 rounds)
constexpr int E = 1 << E_LOG;
constexpr int COLS = 16;  // columns per column-pass tile (16 x 8 B = one 128 B line per row)
constexpr int BLOCK = 256;

__host__ __device__ constexpr int cmin(int a, int b) { return a < b ? a : b; }

// Round r of a size-2^S_LOG sub-transform: stages [g0, g0 + er).
template <int S_LOG, int R>
struct Round {
  static constexpr int g0 = R * E_LOG;
  static constexpr int er = cmin(E_LOG, S_LOG - g0);
  static constexpr int a_hi = S_LOG - 1 - g0;       // highest active bit
  static constexpr int a_lo = S_LOG - g0 - er;      // lowest active bit
  static constexpr int ex = E_LOG - er;             // extra (inactive) bits held per thread
  // bit position of the thread's E_LOG-bit window is [a_lo, a_lo + E_LOG)
  __device__ static __forceinline__ uint32_t p_thread(uint32_t t) {
    return (t & ((1u << a_lo) - 1u)) | ((t >> a_lo) << (a_lo + E_LOG));
  }
  __host__ __device__ static constexpr uint32_t p_elem(uint32_t j) {
    return ((j >> ex) << a_lo) | ((j & ((1u << ex) - 1u)) << (a_hi + 1));
  }
};

template <int S_LOG>
struct Sub {
  static constexpr int S = 1 << S_LOG;
  static constexpr int T = S / E;  // threads per sub-transform
  static constexpr int ROUNDS = (S_LOG + E_LOG - 1) / E_LOG;
};

// forward CT round: values in [0, 4q)
template <int S_LOG, int R>
__device__ __forceinline__ void ct_round(uint64_t (&v)[E], uint32_t pt, uint32_t B, const uint64_t* __restrict__ tw,
                                         const uint64_t* __restrict__ tws, uint64_t q) {
  using Rd = Round<S_LOG, R>;
#pragma unroll
  for (int gl = 0; gl < Rd::er; ++gl) {
    const int g = Rd::g0 + gl;
    const int h = 1 << (E_LOG - 1 - gl);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      if (j & h) continue;
      const uint32_t p = pt | Rd::p_elem(j);
      const uint32_t idx = (B << g) + (p >> (S_LOG - g));
      ct_bfly(v[j], v[j | h], tw[idx], tws[idx], q);
    }
  }
}

// inverse GS round: stages in reverse order, values in [0, 2q)
template <int S_LOG, int R>
__device__ __forceinline__ void gs_round(uint64_t (&v)[E], uint32_t pt, uint32_t B, const uint64_t* __restrict__ itw,
                                         const uint64_t* __restrict__ itws, uint64_t q) {
  using Rd = Round<S_LOG, R>;
#pragma unroll
  for (int gl = Rd::er - 1; gl >= 0; --gl) {
    const int g = Rd::g0 + gl;
    const int h = 1 << (E_LOG - 1 - gl);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      if (j & h) continue;
      const uint32_t p = pt | Rd::p_elem(j);
      const uint32_t idx = (B << g) + (p >> (S_LOG - g));
      gs_bfly(v[j], v[j | h], itw[idx], itws[idx], q);
    }
  }
}

struct KArgs {
  const uint64_t* in;
  uint64_t* out;
  const uint64_t* modulus;
  const uint64_t* tw;       // forward or inverse table base
  const uint64_t* tws;
  const uint64_t* n_inv;
  const uint64_t* n_inv_shoup;
  const uint64_t* scale;        // optional, per buffer limb
  const uint64_t* scale_shoup;
  LimbMap map;
  int n;
};

__device__ __forceinline__ void resolve_limb(const LimbMap& m, int y, int& buf_limb, int& row) {
  int i = y;
  if (i >= m.skip_begin) i += (m.skip_end - m.skip_begin);
  buf_limb = i;
  row = i < m.split ? m.first_a + i : m.first_b + (i - m.split);
}

// LDS padding: one 8-byte pad word every 16 words (rows) / one 16-word pad row every 16 rows (columns)
__device__ __forceinline__ uint32_t rpad(uint32_t p) { return p + (p >> 4); }

// ---------------------------------------------------------------------------------------
// Row pass: a tile of ROWS whole rows (S2 contiguous words each) of one limb.
// FWD: rounds 0..ROUNDS-1 of the last log2(S2) CT stages; INV: the same stages in reverse
// (the first log2(S2) GS stages of the inverse transform).
// ---------------------------------------------------------------------------------------
template <int S1_LOG, int S2_LOG, bool INV>
__global__ __launch_bounds__(BLOCK) void ntt_row_pass(KArgs a) {
  using SB = Sub<S2_LOG>;
  constexpr int S2 = SB::S, T = SB::T, ROWS = cmin(BLOCK / T, 1 << S1_LOG), RSTR = S2 + S2 / 16;
  __shared__ uint64_t lds[ROWS * RSTR];

  int buf_limb, trow;
  resolve_limb(a.map, blockIdx.y, buf_limb, trow);
  const uint64_t q = a.modulus[trow];
  const uint64_t* tw = a.tw + (size_t)trow * a.n;
  const uint64_t* tws = a.tws + (size_t)trow * a.n;
  const uint64_t* src = a.in + (size_t)buf_limb * a.n;
  uint64_t* dst = a.out + (size_t)buf_limb * a.n;

  const uint32_t tid = threadIdx.x;
  const uint32_t lr = tid / T, t = tid % T;
  const uint32_t row = blockIdx.x * ROWS + lr;
  const uint32_t B = (1u << S1_LOG) + row;
  uint64_t* L = lds + lr * RSTR;

  uint64_t v[E];
  // coalesced load, round-0 layout p = t + j*T
#pragma unroll
  for (int j = 0; j < E; ++j) v[j] = src[(size_t)row * S2 + t + j * T];

  if constexpr (!INV) {
    ct_round<S2_LOG, 0>(v, Round<S2_LOG, 0>::p_thread(t), B, tw, tws, q);
    if constexpr (SB::ROUNDS > 1) {
#pragma unroll
      for (int j = 0; j < E; ++j) L[rpad(Round<S2_LOG, 0>::p_thread(t) | Round<S2_LOG, 0>::p_elem(j))] = v[j];
      __syncthreads();
      constexpr int R1 = 1;
      const uint32_t pt1 = Round<S2_LOG, R1>::p_thread(t);
#pragma unroll
      for (int j = 0; j < E; ++j) v[j] = L[rpad(pt1 | Round<S2_LOG, R1>::p_elem(j))];
      ct_round<S2_LOG, R1>(v, pt1, B, tw, tws, q);
      if constexpr (SB::ROUNDS > 2) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < E; ++j) L[rpad(pt1 | Round<S2_LOG, R1>::p_elem(j))] = v[j];
        __syncthreads();
        constexpr int R2 = 2;
        const uint32_t pt2 = Round<S2_LOG, R2>::p_thread(t);
#pragma unroll
        for (int j = 0; j < E; ++j) v[j] = L[rpad(pt2 | Round<S2_LOG, R2>::p_elem(j))];
        ct_round<S2_LOG, R2>(v, pt2, B, tw, tws, q);
        static_assert(SB::ROUNDS <= 3, "row pass supports up to 3 rounds");
        __syncthreads();
#pragma unroll
        for (int j = 0; j < E; ++j) L[rpad(pt2 | Round<S2_LOG, R2>::p_elem(j))] = v[j];
      } else {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < E; ++j) L[rpad(pt1 | Round<S2_LOG, R1>::p_elem(j))] = v[j];
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < E; ++j) v[j] = L[rpad(t + j * T)];
    }
    // final stages of the forward transform: reduce to [0, q)
    const uint64_t q2 = q << 1;
#pragma unroll
    for (int j = 0; j < E; ++j) dst[(size_t)row * S2 + t + j * T] = csub(csub(v[j], q2), q);
  } else {
    // inverse: rounds in reverse order
    constexpr int RL = SB::ROUNDS - 1;
    if constexpr (SB::ROUNDS > 1) {
#pragma unroll
      for (int j = 0; j < E; ++j) L[rpad(t + j * T)] = v[j];
      __syncthreads();
      const uint32_t ptl = Round<S2_LOG, RL>::p_thread(t);
#pragma unroll
      for (int j = 0; j < E; ++j) v[j] = L[rpad(ptl | Round<S2_LOG, RL>::p_elem(j))];
      gs_round<S2_LOG, RL>(v, ptl, B, tw, tws, q);
      if constexpr (SB::ROUNDS > 2) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < E; ++j) L[rpad(ptl | Round<S2_LOG, RL>::p_elem(j))] = v[j];
        __syncthreads();
        const uint32_t ptm = Round<S2_LOG, 1>::p_thread(t);
#pragma unroll
        for (int j = 0; j < E; ++j) v[j] = L[rpad(ptm | Round<S2_LOG, 1>::p_elem(j))];
        gs_round<S2_LOG, 1>(v, ptm, B, tw, tws, q);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < E; ++j) L[rpad(ptm | Round<S2_LOG, 1>::p_elem(j))] = v[j];
      } else {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < E; ++j) L[rpad(ptl | Round<S2_LOG, RL>::p_elem(j))] = v[j];
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < E; ++j) v[j] = L[rpad(t + j * T)];
    }
    gs_round<S2_LOG, 0>(v, Round<S2_LOG, 0>::p_thread(t), B, tw, tws, q);
#pragma unroll
    for (int j = 0; j < E; ++j) dst[(size_t)row * S2 + t + j * T] = v[j];  // [0, 2q), column pass follows
  }
}

// ---------------------------------------------------------------------------------------
// Column pass: a tile of COLS consecutive columns (stride S2) of one limb, all S1 rows.
// FWD: the first log2(S1) CT stages (values stay lazy in [0, 4q) for the row pass);
// INV: the last log2(S1) GS stages, then n^-1 (and the optional per-limb scale).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t cidx(uint32_t p, uint32_t c) { return p * COLS + c + (p >> 4) * COLS; }

template <int S1_LOG, int S2_LOG, bool INV>
__global__ __launch_bounds__(BLOCK) void ntt_col_pass(KArgs a) {
  using SB = Sub<S1_LOG>;
  constexpr int S1 = SB::S, T = SB::T, S2 = 1 << S2_LOG;
  constexpr int NT = COLS * T;  // threads actually used
  static_assert(NT <= BLOCK, "column tile too large");
  __shared__ uint64_t lds[(S1 + S1 / 16) * COLS];

  int buf_limb, trow;
  resolve_limb(a.map, blockIdx.y, buf_limb, trow);
  const uint64_t q = a.modulus[trow];
  const uint64_t* tw = a.tw + (size_t)trow * a.n;
  const uint64_t* tws = a.tws + (size_t)trow * a.n;
  const uint64_t* src = a.in + (size_t)buf_limb * a.n;
  uint64_t* dst = a.out + (size_t)buf_limb * a.n;

  const uint32_t tid = threadIdx.x;
  const bool active = tid < NT;
  const uint32_t c = tid % COLS, t = tid / COLS;
  const uint32_t col = blockIdx.x * COLS + c;
  constexpr uint32_t B = 1;

  uint64_t v[E];
  if (active) {
#pragma unroll
    for (int j = 0; j < E; ++j) v[j] = src[(size_t)(t + j * T) * S2 + col];
  }

  if constexpr (!INV) {
    if (active) ct_round<S1_LOG, 0>(v, Round<S1_LOG, 0>::p_thread(t), B, tw, tws, q);
    if constexpr (SB::ROUNDS > 1) {
      static_assert(SB::ROUNDS == 2, "column pass supports 2 rounds");
      if (active) {
#pragma unroll
        for (int j = 0; j < E; ++j) lds[cidx(Round<S1_LOG, 0>::p_thread(t) | Round<S1_LOG, 0>::p_elem(j), c)] = v[j];
      }
      __syncthreads();
      const uint32_t pt1 = Round<S1_LOG, 1>::p_thread(t);
      if (active) {
#pragma unroll
        for (int j = 0; j < E; ++j) v[j] = lds[cidx(pt1 | Round<S1_LOG, 1>::p_elem(j), c)];
        ct_round<S1_LOG, 1>(v, pt1, B, tw, tws, q);
      }
      __syncthreads();
      if (active) {
#pragma unroll
        for (int j = 0; j < E; ++j) lds[cidx(pt1 | Round<S1_LOG, 1>::p_elem(j), c)] = v[j];
      }
      __syncthreads();
      if (active) {
#pragma unroll
        for (int j = 0; j < E; ++j) v[j] = lds[cidx(t + j * T, c)];
      }
    }
    if (active) {
#pragma unroll
      for (int j = 0; j < E; ++j) dst[(size_t)(t + j * T) * S2 + col] = v[j];  // lazy [0, 4q)
    }
  } else {
    if constexpr (SB::ROUNDS > 1) {
      static_assert(SB::ROUNDS == 2, "column pass supports 2 rounds");
      if (active) {
#pragma unroll
        for (int j = 0; j < E; ++j) lds[cidx(t + j * T, c)] = v[j];
      }
      __syncthreads();
      const uint32_t pt1 = Round<S1_LOG, 1>::p_thread(t);
      if (active) {
#pragma unroll
        for (int j = 0; j < E; ++j) v[j] = lds[cidx(pt1 | Round<S1_LOG, 1>::p_elem(j), c)];
        gs_round<S1_LOG, 1>(v, pt1, B, tw, tws, q);
      }
      __syncthreads();
      if (active) {
#pragma unroll
        for (int j = 0; j < E; ++j) lds[cidx(pt1 | Round<S1_LOG, 1>::p_elem(j), c)] = v[j];
      }
      __syncthreads();
      if (active) {
#pragma unroll
        for (int j = 0; j < E; ++j) v[j] = lds[cidx(t + j * T, c)];
      }
    }
    if (active) {
      gs_round<S1_LOG, 0>(v, Round<S1_LOG, 0>::p_thread(t), B, tw, tws, q);
      const uint64_t ni = a.n_inv[trow], nis = a.n_inv_shoup[trow];
      const bool scaled = a.scale != nullptr;
      const uint64_t sc = scaled ? a.scale[buf_limb] : 0, scs = scaled ? a.scale_shoup[buf_limb] : 0;
#pragma unroll
      for (int j = 0; j < E; ++j) {
        uint64_t x = mul_shoup(v[j], ni, nis, q);
        if (scaled) x = mul_shoup(x, sc, scs, q);
        dst[(size_t)(t + j * T) * S2 + col] = x;
      }
    }
  }
}

template <int S1_LOG, int S2_LOG>
hipError_t launch(const NttTables& tb, const uint64_t* in, uint64_t* out, const LimbMap& map, bool inverse,
                  const uint64_t* scale, const uint64_t* scale_shoup, hipStream_t stream) {
  const int limbs = map.num_limbs - (map.skip_end - map.skip_begin);
  if (limbs <= 0) return hipSuccess;
  KArgs a;
  a.in = in; a.out = out; a.modulus = tb.modulus;
  a.tw = inverse ? tb.itw : tb.tw;
  a.tws = inverse ? tb.itw_shoup : tb.tw_shoup;
  a.n_inv = tb.n_inv; a.n_inv_shoup = tb.n_inv_shoup;
  a.scale = scale; a.scale_shoup = scale_shoup;
  a.map = map; a.n = (int)tb.n;
  constexpr int S1 = 1 << S1_LOG, S2 = 1 << S2_LOG;
  constexpr int ROWS = cmin(BLOCK / Sub<S2_LOG>::T, S1);
  const dim3 grid_r(S1 / ROWS, limbs), grid_c(S2 / COLS, limbs);
  const dim3 block_r(ROWS * Sub<S2_LOG>::T);
  if (!inverse) {
    hipLaunchKernelGGL((ntt_col_pass<S1_LOG, S2_LOG, false>), grid_c, dim3(BLOCK), 0, stream, a);
    a.in = out;
    hipLaunchKernelGGL((ntt_row_pass<S1_LOG, S2_LOG, false>), grid_r, block_r, 0, stream, a);
  } else {
    hipLaunchKernelGGL((ntt_row_pass<S1_LOG, S2_LOG, true>), grid_r, block_r, 0, stream, a);
    a.in = out;
    hipLaunchKernelGGL((ntt_col_pass<S1_LOG, S2_LOG, true>), grid_c, dim3(BLOCK), 0, stream, a);
  }
  return hipGetLastError();
}

hipError_t dispatch(const NttTables& tb, const uint64_t* in, uint64_t* out, const LimbMap& map, bool inverse,
                    const uint64_t* scale, const uint64_t* scale_shoup, hipStream_t stream) {
  switch (tb.log_n) {
    case 10: return launch<5, 5>(tb, in, out, map, inverse, scale, scale_shoup, stream);
    case 11: return launch<5, 6>(tb, in, out, map, inverse, scale, scale_shoup, stream);
    case 12: return launch<6, 6>(tb, in, out, map, inverse, scale, scale_shoup, stream);
    case 13: return launch<6, 7>(tb, in, out, map, inverse, scale, scale_shoup, stream);
    case 14: return launch<7, 7>(tb, in, out, map, inverse, scale, scale_shoup, stream);
    case 15: return launch<7, 8>(tb, in, out, map, inverse, scale, scale_shoup, stream);
    case 16: return launch<8, 8>(tb, in, out, map, inverse, scale, scale_shoup, stream);
    case 17: return launch<8, 9>(tb, in, out, map, inverse, scale, scale_shoup, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t ntt_forward(const NttTables& t, const uint64_t* in, uint64_t* out, const LimbMap& map,
                       hipStream_t stream) {
  return dispatch(t, in, out, map, false, nullptr, nullptr, stream);
}

hipError_t ntt_inverse(const NttTables& t, const uint64_t* in, uint64_t* out, const LimbMap& map,
                       const uint64_t* scale, const uint64_t* scale_shoup, hipStream_t stream) {
  return dispatch(t, in, out, map, true, scale, scale_shoup, stream);
}

}  // namespace phx
