// ntt.hip — two-pass negacyclic NTT / INTT for gfx950.
//
// Decomposition (the same factorisation the reference's 2-D radix-8 NTT uses,
// src/ntt/fntt_2d.cu:9-198, re-designed for wave64 and this engine's arithmetic):
//   n = S1 * S2.  The first log2(S1) Cooley-Tukey stages only pair elements of the same
//   column (index mod S2); the last log2(S2) stages only pair elements of the same row
//   (contiguous S2-element block).  The column pass runs the first stages on tiles of COLS
//   consecutive columns, the row pass runs the last stages on tiles of whole rows.  Each
//   tile goes HBM -> registers -> (radix-16 rounds, LDS transposes between rounds) -> HBM.
//
// Stage g of a sub-transform of size S = 2^s pairs local indices p and p + S/2^(g+1) inside
// block iloc = p >> (s - g); the twiddle is tw[B * 2^g + iloc] with B = 1 for the column
// pass and B = S1 + row for the row pass: exactly the table index m + i of the reference's
// in-place CT loop (m = 2^g or S1 * 2^g).
//
// Arithmetic per limb (wave-uniform branch): primes q < 2^50 use exact FP64 arithmetic
// (farith.h; ~half the instructions of a 64-bit integer Shoup butterfly on gfx950), other
// primes use integer Shoup butterflies (arith.h).  In the FP64 forward path the column pass
// leaves IEEE doubles (exact integers, |x| <= 3q) in the buffer for the row pass, which
// writes canonical residues; the integer path keeps the reference's lazy [0, 4q) values.
//
// Latency hiding: both passes are persistent — a workgroup (column pass) or a wavefront
// (row pass) walks a strided list of tiles and prefetches the next tile's data into
// registers before computing the current one.
#include "ntt.h"

#include <algorithm>
#include <type_traits>
#include <utility>

#include "arith.h"
#include "farith.h"

namespace phx {
namespace {

constexpr int E_LOG = 4;  // elements per thread per round = 16 (radix-16 rounds)
constexpr int E = 1 << E_LOG;
constexpr int COLS = 16;  // columns per column-pass tile (16 x 8 B = one 128 B line per row)
constexpr int BLOCK = 256;
#ifndef PHX_NTT_GRID_MULT
#define PHX_NTT_GRID_MULT 0  // persistent workgroups per CU (0: one workgroup per tile)
#endif
#ifndef PHX_NTT_WAVES_PER_EU
#define PHX_NTT_WAVES_PER_EU 4  // __launch_bounds__ occupancy target (waves per SIMD)
#endif
#ifndef PHX_NTT_PREFETCH
#define PHX_NTT_PREFETCH 0   // prefetch the next tile into registers
#endif

__host__ __device__ constexpr int cmin(int a, int b) { return a < b ? a : b; }

// Round r of a size-2^S_LOG sub-transform: stages [g0, g0 + er).
template <int S_LOG, int R>
struct Round {
  static constexpr int g0 = R * E_LOG;
  static constexpr int er = cmin(E_LOG, S_LOG - g0);
  static constexpr int a_hi = S_LOG - 1 - g0;   // highest active bit
  static constexpr int a_lo = S_LOG - g0 - er;  // lowest active bit
  static constexpr int ex = E_LOG - er;         // extra (inactive) bits held per thread
  // the thread's E_LOG-bit window occupies bit positions [a_lo, a_lo + E_LOG)
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

// ---------------------------------------------------------------------------------------
// per-limb arithmetic context
// ---------------------------------------------------------------------------------------
struct LimbCtx {
  uint64_t q;
  double qd, qinv;
  const uint64_t* tw;   // integer table (forward or inverse)
  const uint64_t* tws;  // its Shoup quotients
  const double* twf;    // FP64 table (centered), forward only
};

// Distinct twiddles of one round: stage gl has 2^(gl + ex) of them, keyed by the element's
// active bits above the pair bit and its extra bits; slots are packed stage after stage.
template <int EX>
__host__ __device__ constexpr int tw_slot(int gl, int key) { return (((1 << gl) - 1) << EX) + key; }
template <int EX>
__host__ __device__ constexpr int tw_key(int gl, int j) { return ((j >> (E_LOG - gl)) << EX) | (j & ((1 << EX) - 1)); }

// Twiddles of one round, loaded into registers before the next tile's prefetch is issued
// (vmcnt counts loads in issue order, so a twiddle load issued after the prefetch would
// make the compute wait for the prefetch).  w[gl][k]: stage gl, k-th butterfly.
template <int S_LOG, int R, typename W>
__device__ __forceinline__ void load_tw(W (&w)[E], const W* __restrict__ tab, uint32_t pt, uint32_t B) {
  using Rd = Round<S_LOG, R>;
#pragma unroll
  for (int gl = 0; gl < Rd::er; ++gl) {
    const int g = Rd::g0 + gl;
#pragma unroll
    for (int key = 0; key < (1 << (gl + Rd::ex)); ++key) {
      // a representative element j with this key: active bits above the pair bit from key's
      // high part, extra bits from key's low part
      const int j = ((key >> Rd::ex) << (E_LOG - gl)) | (key & ((1 << Rd::ex) - 1));
      const uint32_t p = pt | Rd::p_elem(j);
      w[tw_slot<Rd::ex>(gl, key)] = tab[(B << g) + (p >> (S_LOG - g))];
    }
  }
}

// Row-pass FP64 twiddles computed on the fly: tw = A_g(row) * B_g(iloc) mod q (ntt.h), so the
// row pass reads 8 per-row factors and a 2 KB per-limb table instead of an n-entry table.
template <int S_LOG, int R>
__device__ __forceinline__ void make_tw_row_f64(double (&w)[E], const double* __restrict__ A,
                                                const double* __restrict__ Btab, uint32_t pt, double qd,
                                                double qinv) {
  using Rd = Round<S_LOG, R>;
#pragma unroll
  for (int gl = 0; gl < Rd::er; ++gl) {
    const int g = Rd::g0 + gl;
    const double ag = A[g];
#pragma unroll
    for (int key = 0; key < (1 << (gl + Rd::ex)); ++key) {
      const int j = ((key >> Rd::ex) << (E_LOG - gl)) | (key & ((1 << Rd::ex) - 1));
      const uint32_t p = pt | Rd::p_elem(j);
      const double b = Btab[(1u << g) + (p >> (S_LOG - g))];
      w[tw_slot<Rd::ex>(gl, key)] = freduce(fmodmul(b, ag, qd, qinv), qd, qinv);
    }
  }
}

// forward CT round, integer path: values in [0, 4q)
template <int S_LOG, int R>
__device__ __forceinline__ void ct_round_int(uint64_t (&v)[E], const uint64_t (&w)[E], const uint64_t (&ws)[E],
                                             uint64_t q) {
  using Rd = Round<S_LOG, R>;
#pragma unroll
  for (int gl = 0; gl < Rd::er; ++gl) {
    const int h = 1 << (E_LOG - 1 - gl);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      if (j & h) continue;
      const int sl = tw_slot<Rd::ex>(gl, tw_key<Rd::ex>(gl, j));
      ct_bfly(v[j], v[j | h], w[sl], ws[sl], q);
    }
  }
}

// forward CT round, FP64 path.  GOFF = global stage index of local stage 0 of this
// sub-transform; every value is reduced before global stages 3, 6, 9, ... (farith.h bounds).
template <int S_LOG, int R, int GOFF>
__device__ __forceinline__ void ct_round_f64(double (&v)[E], const double (&w)[E], double qd, double qinv) {
  using Rd = Round<S_LOG, R>;
#ifdef PHX_NTT_NO_COMPUTE
  return;
#endif
#pragma unroll
  for (int gl = 0; gl < Rd::er; ++gl) {
    const int g = Rd::g0 + gl;
    if ((GOFF + g) % 3 == 0 && (GOFF + g) > 0) {
#pragma unroll
      for (int j = 0; j < E; ++j) v[j] = freduce(v[j], qd, qinv);
    }
    const int h = 1 << (E_LOG - 1 - gl);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      if (j & h) continue;
      const double t = fmodmul(v[j | h], w[tw_slot<Rd::ex>(gl, tw_key<Rd::ex>(gl, j))], qd, qinv);
      v[j | h] = v[j] - t;
      v[j] = v[j] + t;
    }
  }
}

// inverse GS round (integer path): stages in reverse order, values in [0, 2q)
template <int S_LOG, int R>
__device__ __forceinline__ void gs_round_int(uint64_t (&v)[E], const uint64_t (&w)[E], const uint64_t (&ws)[E],
                                             uint64_t q) {
  using Rd = Round<S_LOG, R>;
#pragma unroll
  for (int gl = Rd::er - 1; gl >= 0; --gl) {
    const int h = 1 << (E_LOG - 1 - gl);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      if (j & h) continue;
      const int sl = tw_slot<Rd::ex>(gl, tw_key<Rd::ex>(gl, j));
      gs_bfly(v[j], v[j | h], w[sl], ws[sl], q);
    }
  }
}

struct KArgs {
  const uint64_t* in;
  uint64_t* out;
  const uint64_t* modulus;
  const double* modulus_f;    // q as double
  const double* modulus_inv;  // 1/q rounded
  const uint8_t* is_f64;      // per table row: FP64 path usable (q < 2^50)
  const uint64_t* tw;         // forward or inverse integer table base
  const uint64_t* tws;
  const double* twf;          // forward FP64 table
  const double* row_a;        // row-pass factored twiddles (ntt.h)
  const double* row_b;
  const uint64_t* n_inv;
  const uint64_t* n_inv_shoup;
  const uint64_t* scale;      // optional, per buffer limb
  const uint64_t* scale_shoup;
  LimbMap map;
  int n;
  int limbs;                  // number of processed limbs (excluding skipped)
  int f64_fwd;                // 1: forward transform may use the FP64 path
};

__device__ __forceinline__ void resolve_limb(const LimbMap& m, int y, int& buf_limb, int& row) {
  int i = y;
  if (i >= m.skip_begin) i += (m.skip_end - m.skip_begin);
  buf_limb = i;
  row = i < m.split ? m.first_a + i : m.first_b + (i - m.split);
}

__device__ __forceinline__ LimbCtx limb_ctx(const KArgs& a, int row, bool& f64) {
  // row is wave-uniform: readfirstlane lets the per-limb constants come through scalar loads
  // (a vector load here would carry an s_waitcnt vmcnt(0) that drains the tile prefetch)
  row = __builtin_amdgcn_readfirstlane(row);
  LimbCtx c;
  c.q = a.modulus[row];
  c.qd = a.modulus_f[row];
  c.qinv = a.modulus_inv[row];
  c.tw = a.tw + (size_t)row * a.n;
  c.tws = a.tws + (size_t)row * a.n;
  c.twf = a.twf + (size_t)row * a.n;
  f64 = a.f64_fwd && c.q < (1ull << 50);
  return c;
}

// LDS padding: one pad word every 16 words (row tiles) / one 16-word pad row every 16 rows
// (column tiles) — keeps the transposed round's ds_read_b64 accesses conflict-free.
__device__ __forceinline__ uint32_t rpad(uint32_t p) { return p + (p >> 4); }
__device__ __forceinline__ uint32_t cidx(uint32_t p, uint32_t c) { return p * COLS + c + (p >> 4) * COLS; }

template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) { (f(std::integral_constant<int, I>{}), ...); }
  (std::make_integer_sequence<int, N>{});
}

// All twiddles of one sub-transform for one thread, in registers.
template <int S_LOG>
struct TwF64 {
  double w[Sub<S_LOG>::ROUNDS][E];
};
template <int S_LOG>
struct TwInt {
  uint64_t w[Sub<S_LOG>::ROUNDS][E];
  uint64_t ws[Sub<S_LOG>::ROUNDS][E];
};

template <int S_LOG>
__device__ __forceinline__ void load_all(TwF64<S_LOG>& tw, const double* tab, uint32_t t, uint32_t B) {
  static_for<Sub<S_LOG>::ROUNDS>([&](auto r) {
    constexpr int R = decltype(r)::value;
    load_tw<S_LOG, R>(tw.w[R], tab, Round<S_LOG, R>::p_thread(t), B);
  });
}
template <int S_LOG>
__device__ __forceinline__ void load_all(TwInt<S_LOG>& tw, const uint64_t* tab, const uint64_t* tabs, uint32_t t,
                                         uint32_t B) {
  static_for<Sub<S_LOG>::ROUNDS>([&](auto r) {
    constexpr int R = decltype(r)::value;
    load_tw<S_LOG, R>(tw.w[R], tab, Round<S_LOG, R>::p_thread(t), B);
    load_tw<S_LOG, R>(tw.ws[R], tabs, Round<S_LOG, R>::p_thread(t), B);
  });
}

// One full sub-transform (all rounds) on registers v, which hold the load layout
// p = t + j*T on entry and on exit.  L is this thread-group's LDS tile of element type V
// indexed by idx(p); sync() orders the LDS exchanges (workgroup or wavefront barrier).
// Twiddles of one round in registers (FP64: w; integer: w and Shoup quotients ws)
struct RoundTwF64 {
  double w[E];
};
struct RoundTwInt {
  uint64_t w[E], ws[E];
};

// get_tw(integral_constant<R>) produces round R's twiddles; it runs right before the round so
// only one round's twiddles are live (keeps VGPR use low enough for 4 waves per SIMD).
template <int S_LOG, int GOFF, bool FWD, typename V, typename GetTw, typename Idx, typename Sync>
__device__ __forceinline__ void sub_transform(V (&v)[E], GetTw get_tw, V* L, Idx idx, Sync sync, uint32_t t,
                                              uint64_t q, double qd, double qinv) {
  using SB = Sub<S_LOG>;
  constexpr int RN = SB::ROUNDS;
  constexpr bool F = !std::is_same_v<V, uint64_t>;
  auto round = [&](auto r) {
    constexpr int R = decltype(r)::value;
    const auto tw = get_tw(r);
    if constexpr (F) {
      static_assert(FWD, "FP64 path is forward-only");
      ct_round_f64<S_LOG, R, GOFF>(v, tw.w, qd, qinv);
    } else if constexpr (FWD) {
      ct_round_int<S_LOG, R>(v, tw.w, tw.ws, q);
    } else {
      gs_round_int<S_LOG, R>(v, tw.w, tw.ws, q);
    }
  };
  auto put = [&](uint32_t pt, auto r) {
    constexpr int R = decltype(r)::value;
#pragma unroll
    for (int j = 0; j < E; ++j) L[idx(pt | Round<S_LOG, R>::p_elem(j))] = v[j];
  };
  auto get = [&](uint32_t pt, auto r) {
    constexpr int R = decltype(r)::value;
#pragma unroll
    for (int j = 0; j < E; ++j) v[j] = L[idx(pt | Round<S_LOG, R>::p_elem(j))];
  };
  if constexpr (FWD) {
    round(std::integral_constant<int, 0>{});
    static_for<RN - 1>([&](auto rm1) {
      constexpr int R = decltype(rm1)::value + 1;
      put(Round<S_LOG, R - 1>::p_thread(t), std::integral_constant<int, R - 1>{});
      sync();
      get(Round<S_LOG, R>::p_thread(t), std::integral_constant<int, R>{});
      sync();
      round(std::integral_constant<int, R>{});
    });
    if constexpr (RN > 1) {
      put(Round<S_LOG, RN - 1>::p_thread(t), std::integral_constant<int, RN - 1>{});
      sync();
      get(Round<S_LOG, 0>::p_thread(t), std::integral_constant<int, 0>{});
      sync();
    }
  } else {
    if constexpr (RN > 1) {
      put(Round<S_LOG, 0>::p_thread(t), std::integral_constant<int, 0>{});
      sync();
      get(Round<S_LOG, RN - 1>::p_thread(t), std::integral_constant<int, RN - 1>{});
      sync();
    }
    static_for<RN - 1>([&](auto i) {
      constexpr int R = RN - 1 - decltype(i)::value;  // RN-1 .. 1
      round(std::integral_constant<int, R>{});
      put(Round<S_LOG, R>::p_thread(t), std::integral_constant<int, R>{});
      sync();
      get(Round<S_LOG, R - 1>::p_thread(t), std::integral_constant<int, R - 1>{});
      sync();
    });
    round(std::integral_constant<int, 0>{});
  }
}

__device__ __forceinline__ void fence_loads() { __builtin_amdgcn_sched_barrier(0); }

// ---------------------------------------------------------------------------------------
// Column pass: tile = COLS consecutive columns x S1 rows of one limb; 256-thread workgroup.
// FWD: first log2(S1) CT stages (FP64: output doubles |x| <= 3q; int: lazy [0, 4q)).
// INV: last log2(S1) GS stages, then n^-1 and the optional per-limb scale.
// ---------------------------------------------------------------------------------------
template <int S1_LOG, int S2_LOG, bool FWD>
__global__ __launch_bounds__(BLOCK, PHX_NTT_WAVES_PER_EU) void ntt_col(KArgs a) {
  using SB = Sub<S1_LOG>;
  constexpr int T = SB::T, S2 = 1 << S2_LOG, NT = COLS * T, CT = S2 / COLS;
  static_assert(NT <= BLOCK, "column tile too large");
  __shared__ uint64_t lds[(SB::S + SB::S / 16) * COLS];

  const uint32_t tid = threadIdx.x;
  const bool active = tid < NT;
  const uint32_t c = tid % COLS, t = tid / COLS;
  const int ntiles = a.limbs * CT;
  const int ntiles_or_items = ntiles;
  auto idx = [c](uint32_t p) { return cidx(p, c); };
  auto sync = [] { __syncthreads(); };

  uint64_t cur[E], nxt[E];
  auto load = [&](int tile, uint64_t (&dst)[E]) {
    int buf_limb, row;
    resolve_limb(a.map, tile / CT, buf_limb, row);
    const uint64_t* src = a.in + (size_t)buf_limb * a.n + (tile % CT) * COLS + c;
    if (active) {
#pragma unroll
      for (int j = 0; j < E; ++j) dst[j] = __builtin_nontemporal_load(src + (size_t)(t + j * T) * S2);
    }
  };
  int tile = blockIdx.x;
  if (tile < ntiles) load(tile, cur);
  for (; tile < ntiles; tile += gridDim.x) {
    const int next = tile + gridDim.x;
    int buf_limb, row;
    resolve_limb(a.map, tile / CT, buf_limb, row);
    bool f64;
    const LimbCtx lc = limb_ctx(a, row, f64);
    uint64_t* dst = a.out + (size_t)buf_limb * a.n + (tile % CT) * COLS + c;
    if (FWD && f64) {
      auto tw = [&](auto r) {
        constexpr int R = decltype(r)::value;
        RoundTwF64 x;
        load_tw<S1_LOG, R>(x.w, lc.twf, Round<S1_LOG, R>::p_thread(t), 1);
        return x;
      };
      if (PHX_NTT_PREFETCH && next < ntiles) load(next, nxt);
      double v[E];
#pragma unroll
      for (int j = 0; j < E; ++j) v[j] = u64_to_f64(cur[j]);
      if constexpr (FWD)
        sub_transform<S1_LOG, 0, true>(v, tw, reinterpret_cast<double*>(lds), idx, sync, t, lc.q, lc.qd, lc.qinv);
      if (active) {
#pragma unroll
        for (int j = 0; j < E; ++j) dst[(size_t)(t + j * T) * S2] = as_bits(v[j]);
      }
    } else {
      auto tw = [&](auto r) {
        constexpr int R = decltype(r)::value;
        RoundTwInt x;
        load_tw<S1_LOG, R>(x.w, lc.tw, Round<S1_LOG, R>::p_thread(t), 1);
        load_tw<S1_LOG, R>(x.ws, lc.tws, Round<S1_LOG, R>::p_thread(t), 1);
        return x;
      };
      if (PHX_NTT_PREFETCH && next < ntiles) load(next, nxt);
      sub_transform<S1_LOG, 0, FWD>(cur, tw, lds, idx, sync, t, lc.q, lc.qd, lc.qinv);
      if (active) {
        if constexpr (FWD) {
#pragma unroll
          for (int j = 0; j < E; ++j) dst[(size_t)(t + j * T) * S2] = cur[j];  // lazy [0, 4q)
        } else {
          const uint64_t ni = a.n_inv[row], nis = a.n_inv_shoup[row];
          const bool scaled = a.scale != nullptr;
          const uint64_t sc = scaled ? a.scale[buf_limb] : 0, scs = scaled ? a.scale_shoup[buf_limb] : 0;
#pragma unroll
          for (int j = 0; j < E; ++j) {
            uint64_t x = mul_shoup(cur[j], ni, nis, lc.q);
            if (scaled) x = mul_shoup(x, sc, scs, lc.q);
            dst[(size_t)(t + j * T) * S2] = x;
          }
        }
      }
    }
    if constexpr (PHX_NTT_PREFETCH) {
#pragma unroll
      for (int j = 0; j < E; ++j) cur[j] = nxt[j];
    } else if (next < ntiles_or_items) {
      load(next, cur);
    }
  }
}

// ---------------------------------------------------------------------------------------
// Row pass: each wavefront owns RW = 64/T whole rows at a time (T lanes per row), so the
// LDS transposes are wave-private and need no workgroup barrier.
// FWD: last log2(S2) CT stages, canonical output.  INV: first log2(S2) GS stages.
// ---------------------------------------------------------------------------------------
template <int S1_LOG, int S2_LOG, bool FWD>
__global__ __launch_bounds__(BLOCK, PHX_NTT_WAVES_PER_EU) void ntt_row(KArgs a) {
  using SB = Sub<S2_LOG>;
  constexpr int S2 = SB::S, T = SB::T, RW = cmin(64 / T, 1 << S1_LOG), RSTR = S2 + S2 / 16;
  constexpr int WAVES = BLOCK / 64;
  constexpr int GROUPS = (1 << S1_LOG) / RW;  // row groups per limb
  __shared__ uint64_t lds[WAVES * RW * RSTR];

  const uint32_t lane = threadIdx.x % 64, wave = threadIdx.x / 64;
  const uint32_t lr = lane / T, t = lane % T;
  uint64_t* lrow = lds + (wave * RW + lr) * RSTR;
  const int nitems = a.limbs * GROUPS;
  const int ntiles_or_items = nitems;
  const int stride = gridDim.x * WAVES;
  auto idx = [](uint32_t p) { return rpad(p); };
  auto sync = [] { __builtin_amdgcn_wave_barrier(); };

  uint64_t cur[E], nxt[E];
  auto load = [&](int item, uint64_t (&dst)[E]) {
    int buf_limb, row;
    resolve_limb(a.map, item / GROUPS, buf_limb, row);
    const uint32_t r = (item % GROUPS) * RW + lr;
    const uint64_t* src = a.in + (size_t)buf_limb * a.n + (size_t)r * S2 + t;
#pragma unroll
    for (int j = 0; j < E; ++j) dst[j] = src[j * T];
  };
  int item = __builtin_amdgcn_readfirstlane(blockIdx.x * WAVES + wave);
  if (item < nitems) load(item, cur);
  for (; item < nitems; item += stride) {
    const int next = item + stride;
    int buf_limb, row;
    resolve_limb(a.map, item / GROUPS, buf_limb, row);
    buf_limb = __builtin_amdgcn_readfirstlane(buf_limb);
    bool f64;
    const LimbCtx lc = limb_ctx(a, row, f64);
    const uint32_t r = (item % GROUPS) * RW + lr;
    const uint32_t B = (1u << S1_LOG) + r;
    uint64_t* dst = a.out + (size_t)buf_limb * a.n + (size_t)r * S2 + t;
    if (FWD && f64) {
      const double* A = a.row_a + ((size_t)row * (1u << S1_LOG) + r) * 16;
      const double* Bt = a.row_b + (size_t)row * S2;
      auto tw = [&](auto rr) {
        constexpr int RR = decltype(rr)::value;
        RoundTwF64 x;
        make_tw_row_f64<S2_LOG, RR>(x.w, A, Bt, Round<S2_LOG, RR>::p_thread(t), lc.qd, lc.qinv);
        return x;
      };
      if (PHX_NTT_PREFETCH && next < nitems) load(next, nxt);
      double v[E];
#pragma unroll
      for (int j = 0; j < E; ++j) v[j] = as_f64(cur[j]);
      if constexpr (FWD)
        sub_transform<S2_LOG, S1_LOG, true>(v, tw, reinterpret_cast<double*>(lrow), idx, sync, t, lc.q, lc.qd,
                                            lc.qinv);
#pragma unroll
      for (int j = 0; j < E; ++j) __builtin_nontemporal_store(f64_to_canonical(v[j], lc.qd, lc.qinv), dst + j * T);
    } else {
      auto tw = [&](auto rr) {
        constexpr int RR = decltype(rr)::value;
        RoundTwInt x;
        load_tw<S2_LOG, RR>(x.w, lc.tw, Round<S2_LOG, RR>::p_thread(t), B);
        load_tw<S2_LOG, RR>(x.ws, lc.tws, Round<S2_LOG, RR>::p_thread(t), B);
        return x;
      };
      if (PHX_NTT_PREFETCH && next < nitems) load(next, nxt);
      sub_transform<S2_LOG, S1_LOG, FWD>(cur, tw, lrow, idx, sync, t, lc.q, lc.qd, lc.qinv);
      if constexpr (FWD) {
        const uint64_t q2 = lc.q << 1;
#pragma unroll
        for (int j = 0; j < E; ++j) __builtin_nontemporal_store(csub(csub(cur[j], q2), lc.q), dst + j * T);
      } else {
#pragma unroll
        for (int j = 0; j < E; ++j) dst[j * T] = cur[j];  // [0, 2q), column pass follows
      }
    }
    if constexpr (PHX_NTT_PREFETCH) {
#pragma unroll
      for (int j = 0; j < E; ++j) cur[j] = nxt[j];
    } else if (next < ntiles_or_items) {
      load(next, cur);
    }
  }
}

int g_num_cus = 0;

int num_cus() {
  if (!g_num_cus) {
    int dev = 0;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess) g_num_cus = p.multiProcessorCount;
    if (g_num_cus <= 0) g_num_cus = 256;
  }
  return g_num_cus;
}

template <int S1_LOG, int S2_LOG>
hipError_t launch(const NttTables& tb, const uint64_t* in, uint64_t* out, const LimbMap& map, bool inverse,
                  const uint64_t* scale, const uint64_t* scale_shoup, hipStream_t stream) {
  const int limbs = map.num_limbs - (map.skip_end - map.skip_begin);
  if (limbs <= 0) return hipSuccess;
  KArgs a;
  a.in = in; a.out = out; a.modulus = tb.modulus;
  a.modulus_f = tb.modulus_f; a.modulus_inv = tb.modulus_inv; a.is_f64 = tb.is_f64;
  a.tw = inverse ? tb.itw : tb.tw;
  a.tws = inverse ? tb.itw_shoup : tb.tw_shoup;
  a.twf = tb.twf;
  a.row_a = tb.row_a;
  a.row_b = tb.row_b;
  a.n_inv = tb.n_inv; a.n_inv_shoup = tb.n_inv_shoup;
  a.scale = scale; a.scale_shoup = scale_shoup;
  a.map = map; a.n = (int)tb.n; a.limbs = limbs;
  a.f64_fwd = inverse ? 0 : 1;
  constexpr int S1 = 1 << S1_LOG, S2 = 1 << S2_LOG;
  constexpr int RW = cmin(64 / Sub<S2_LOG>::T, S1);
  const int col_tiles = limbs * (S2 / COLS);
  const int row_items = limbs * (S1 / RW);
  const int cus = num_cus();
  const int gm = PHX_NTT_GRID_MULT > 0 ? PHX_NTT_GRID_MULT : 1 << 20;
  const dim3 grid_c(std::min(col_tiles, cus * gm)), grid_r(std::min((row_items + 3) / 4, cus * gm));
  const dim3 block(BLOCK);
  if (!inverse) {
    hipLaunchKernelGGL((ntt_col<S1_LOG, S2_LOG, true>), grid_c, block, 0, stream, a);
    a.in = out;
    hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, true>), grid_r, block, 0, stream, a);
  } else {
    hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, false>), grid_r, block, 0, stream, a);
    a.in = out;
    hipLaunchKernelGGL((ntt_col<S1_LOG, S2_LOG, false>), grid_c, block, 0, stream, a);
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
