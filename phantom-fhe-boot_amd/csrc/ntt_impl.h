// ntt_impl.h — two-pass negacyclic NTT / INTT for gfx950: kernels and the launch<S1, S2> template.
// csrc/ntt.hip holds the launchers (dispatch over the degree) and the 1-D path; each csrc/ntt_n*.hip
// instantiates launch<> for some degrees, so the heavy template instantiations compile in parallel.
//
// Decomposition (the factorisation the reference's 2-D radix-8 NTT uses, src/ntt/fntt_2d.cu:9-198
// and src/ntt/intt_2d.cu:9-207, re-designed for wave64 and this engine's arithmetic):
//   n = S1 * S2, coefficient k = row * S2 + col.  The first log2(S1) Cooley-Tukey stages only
//   pair elements of one column, the last log2(S2) only elements of one row.  The column pass
//   runs those stages on tiles of COLS consecutive columns (16 x 8 B = one 128 B line per row),
//   the row pass on whole rows; each tile goes HBM -> registers -> (radix-16 rounds, LDS
//   transposes between rounds) -> HBM.  The inverse runs the Gentleman-Sande stages in the
//   reverse order: row pass, then column pass.
//
// Stage g of a sub-transform of size S = 2^s pairs local indices p and p + S/2^(g+1) inside
// block iloc = p >> (s - g); its twiddle is tw[B 2^g + iloc] with B = 1 in the column pass and
// B = S1 + row in the row pass: the table index m + i of the reference's in-place loops.
//
// Arithmetic per limb (wave-uniform branch): primes q < 2^50 use exact FP64 arithmetic
// (farith.h), other primes the integer Shoup butterflies of arith.h.
//  * FP64 forward: the column pass stores exact-integer doubles (|x| < 7.75 q) for the row pass,
//    which writes canonical residues.  Reductions are placed at compile time (Bound, farith.h).
//  * FP64 inverse: GS butterflies; n^-1 is folded into the last stage (x' = (x + y) n^-1,
//    y' = (x - y) itw[1] n^-1) as the reference does (src/ntt/intt_2d.cu:195-198).
//  * Column-pass twiddles come from a per-limb S1-entry table (cache resident); row-pass
//    twiddles are generated: tw = A_g(row) * B_g(iloc) (host/ntt_tables.cpp), the 15 twiddles
//    of the first radix-16 round (the same for all lanes of a row) cooperatively through LDS.
//  * Integer path: the reference's butterflies with an approximate Shoup quotient and doubled lazy
//    ranges ([0, 8q) forward, [0, 4q) inverse; arith.h), twiddles and Shoup quotients read from
//    the full tables, n^-1 applied after the last stage.  Forward limbs with q < 2^60 (every
//    prime of the bootstrap chain) run with a 16q lazy range and reduce x only every other stage
//    (Plan::col_lz / row_lz): the column pass hands values < 12q to the row pass.
#pragma once

#include "ntt.h"

#include <algorithm>
#include <type_traits>
#include <utility>

#include "arith.h"
#include "farith.h"

namespace phx {
namespace nttd {  // the 2-D NTT kernels and launch<>; ntt.hip dispatches, ntt_n*.hip instantiate

#ifndef PHX_E_LOG
#define PHX_E_LOG 4
#endif
constexpr int E_LOG = PHX_E_LOG;  // elements per thread per round = 16 (radix-16 rounds)
constexpr int E = 1 << E_LOG;
// columns per column-pass tile: 16 x 8 B = one 128 B line per row (8 / 16 / 32 measured 36.7 /
// 26.6 / 28.4 us for the 50-bit forward, profiles/r03/ntt_experiments/cols_*.txt)
constexpr int COLS = 16;
constexpr int BLOCK = 256;
constexpr int CBLOCK = COLS * (256 >> E_LOG) > BLOCK ? COLS * (256 >> E_LOG) : BLOCK;  // column-pass workgroup bound (S1 <= 256)
constexpr int kNttWavesPerEU = 3;  // __launch_bounds__ occupancy target (waves per SIMD) of one-tile grids
#ifndef PHX_ROW_WAVES
#define PHX_ROW_WAVES 3
#endif
constexpr int kRowWaves = PHX_ROW_WAVES;  // ... of the plain row pass (no prologue / epilogue)

__host__ __device__ constexpr int cmin(int a, int b) { return a < b ? a : b; }

// Round R of a size-2^S_LOG sub-transform: stages [g0, g0 + er).
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

template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) { (f(std::integral_constant<int, I>{}), ...); }
  (std::make_integer_sequence<int, N>{});
}

// ---------------------------------------------------------------------------------------
// FP64 reduction schedules (compile time): bit g of `mask` = reduce every value before stage g.
// ---------------------------------------------------------------------------------------
struct Sched {
  uint32_t mask;
  double out;  // bound of the pass output (units of q)
};
constexpr double dmax(double a, double b) { return a > b ? a : b; }
// Cooley-Tukey stages g = 0 .. s-1: x' = x +- fmodmul(y, w)
constexpr Sched sched_ct(int s, double x0, double w) {
  Sched r{0u, x0};
  double x = x0;
  for (int g = 0; g < s; ++g) {
    if (x + Bound::prod(x, w) > Bound::kLimit) {
      r.mask |= 1u << g;
      x = Bound::kReduced;
    }
    x = x + Bound::prod(x, w);
  }
  r.out = x;
  return r;
}
// Gentleman-Sande stages g = s-1 .. 0: x' = x + y, y' = fmodmul(x - y, w); with `fold` the
// last stage also multiplies x' by n^-1
constexpr Sched sched_gs(int s, double x0, double w, bool fold) {
  Sched r{0u, x0};
  double x = x0;
  for (int g = s - 1; g >= 0; --g) {
    auto next = [&](double v) { return (fold && g == 0) ? Bound::prod(2 * v, w) : dmax(2 * v, Bound::prod(2 * v, w)); };
    if (next(x) > Bound::kLimit) {
      r.mask |= 1u << g;
      x = Bound::kReduced;
    }
    x = next(x);
  }
  r.out = x;
  return r;
}

// Integer forward path for q < 2^60 (arith.h ct_bfly_nored / ct_bfly_c8): values stay below
// 16q < 2^64; bit g of `mask` = reduce x below 8q before stage g, needed only when the bound
// would pass 16q.  `out` = bound of the pass output (units of q).
struct LazySched {
  uint32_t mask;
  int out;
};
constexpr LazySched lazy_ct(int s, int start) {
  LazySched r{0u, start};
  int b = start;
  for (int g = 0; g < s; ++g) {
    if (b + 4 <= 16) {
      b += 4;
    } else {
      r.mask |= 1u << g;
      b = 12;  // x < 16q reduced below 8q, plus t < 4q
    }
  }
  r.out = b;
  return r;
}

// Integer inverse path for q < 2^60 (arith.h gs_bfly8): every value stays below 8q between
// stages and rounds.  The bound of each of a thread's E elements is tracked through a round's
// stages (x' = x + y sums the two bounds, y' = the product < 4q); bit j of m[gl] = reduce x' of
// element j below 8q at stage gl, needed only when the sum's bound passes 8q.  A full round
// from inputs < 8q reduces 20 of its 32 sums; the eager form (gs_bfly4) reduced all 32.
struct LazyGs {
  uint32_t m[E_LOG];
};
constexpr LazyGs lazy_gs(int er, int b_in) {
  LazyGs r{};
  int b[E] = {};
  for (int j = 0; j < E; ++j) b[j] = b_in;
  for (int gl = er - 1; gl >= 0; --gl) {
    const int h = 1 << (E_LOG - 1 - gl);
    for (int j = 0; j < E; ++j) {
      if (j & h) continue;
      int sum = b[j] + b[j | h];
      if (sum > 8) {
        r.m[gl] |= 1u << j;
        sum = 8;
      }
      b[j] = sum;
      b[j | h] = 4;
    }
  }
  return r;
}

template <int S1_LOG, int S2_LOG>
struct Plan {
  static constexpr LazySched col_lz = lazy_ct(S1_LOG, 1);
  static constexpr LazySched row_lz = lazy_ct(S2_LOG, col_lz.out);
  static_assert(col_lz.out <= 16 && row_lz.out <= 16, "lazy bound");
  static constexpr Sched col_fwd = sched_ct(S1_LOG, 1.0, Bound::kTableW);
  static constexpr Sched row_fwd = sched_ct(S2_LOG, col_fwd.out, Bound::kGenW);
  static constexpr Sched row_inv = sched_gs(S2_LOG, 1.0, Bound::kGenW, false);
  static constexpr Sched col_inv = sched_gs(S1_LOG, row_inv.out, Bound::kGenW, true);
  static_assert(col_fwd.out < Bound::kLimit && row_fwd.out < Bound::kLimit, "bound");
  static_assert(row_inv.out < Bound::kLimit && col_inv.out < Bound::kLimit, "bound");
};

// ---------------------------------------------------------------------------------------
// twiddles of one round
// ---------------------------------------------------------------------------------------
// Distinct twiddles of one round: stage gl has 2^(gl + ex) of them, keyed by the element's
// active bits above the pair bit and its extra bits; slots are packed stage after stage.
template <int EX>
__host__ __device__ constexpr int tw_slot(int gl, int key) { return (((1 << gl) - 1) << EX) + key; }
template <int EX>
__host__ __device__ constexpr int tw_key(int gl, int j) { return ((j >> (E_LOG - gl)) << EX) | (j & ((1 << EX) - 1)); }

// representative element j of key `key` at local stage gl
template <int EX>
__host__ __device__ constexpr int key_elem(int gl, int key) {
  return ((key >> EX) << (E_LOG - gl)) | (key & ((1 << EX) - 1));
}

// twiddles read from a table: w[slot] = tab[(B << g) + (p >> (S_LOG - g))]
template <int S_LOG, int R, typename W>
__device__ __forceinline__ void load_tw(W (&w)[E], const W* __restrict__ tab, uint32_t pt, uint32_t B) {
  using Rd = Round<S_LOG, R>;
#pragma unroll
  for (int gl = 0; gl < Rd::er; ++gl) {
    const int g = Rd::g0 + gl;
#pragma unroll
    for (int key = 0; key < (1 << (gl + Rd::ex)); ++key) {
      const uint32_t p = pt | Rd::p_elem(key_elem<Rd::ex>(gl, key));
      w[tw_slot<Rd::ex>(gl, key)] = tab[(B << g) + (p >> (S_LOG - g))];
    }
  }
}

// A twiddle from its Shoup quotient alone.  ws = floor(w 2^64 / q) with 0 < w < q and q prime:
// w 2^64 = ws q + rem with 0 < rem < q < 2^64, so floor(ws q / 2^64) = w - 1 exactly.  (Every
// table twiddle is a power of a root of unity, never 0.)
__device__ __forceinline__ uint64_t w_from_shoup(uint64_t ws, uint64_t q) { return __umul64hi(ws, q) + 1; }

template <int S_LOG, int R>
__device__ __forceinline__ void w_from_shoup_round(uint64_t (&w)[E], const uint64_t (&ws)[E], uint64_t q) {
  using Rd = Round<S_LOG, R>;
#pragma unroll
  for (int gl = 0; gl < Rd::er; ++gl)
#pragma unroll
    for (int key = 0; key < (1 << (gl + Rd::ex)); ++key) {
      const int s = tw_slot<Rd::ex>(gl, key);
      w[s] = w_from_shoup(ws[s], q);
    }
}

// row-pass FP64 twiddles generated per lane: tw = A[g] * Btab[2^g + iloc] (unreduced, |tw| <= kGenW q)
template <int S_LOG, int R>
__device__ __forceinline__ void gen_tw_row(double (&w)[E], const double* __restrict__ A,
                                           const double* __restrict__ Btab, uint32_t pt, double qd, double qinv) {
  using Rd = Round<S_LOG, R>;
#pragma unroll
  for (int gl = 0; gl < Rd::er; ++gl) {
    const int g = Rd::g0 + gl;
    const double ag = A[g];
#pragma unroll
    for (int key = 0; key < (1 << (gl + Rd::ex)); ++key) {
      const uint32_t p = pt | Rd::p_elem(key_elem<Rd::ex>(gl, key));
      w[tw_slot<Rd::ex>(gl, key)] = fmodmul(Btab[(1u << g) + (p >> (S_LOG - g))], ag, qd, qinv);
    }
  }
}

// ---------------------------------------------------------------------------------------
// rounds
// ---------------------------------------------------------------------------------------
template <int S_LOG, int R, uint32_t MASK>
__device__ __forceinline__ void ct_round_f64(double (&v)[E], const double (&w)[E], double qd, double qinv) {
  using Rd = Round<S_LOG, R>;
  static_for<Rd::er>([&](auto glc) {
    constexpr int gl = decltype(glc)::value;
    constexpr int g = Rd::g0 + gl;
    if constexpr ((MASK >> g) & 1u) {
#pragma unroll
      for (int j = 0; j < E; ++j) v[j] = freduce(v[j], qd, qinv);
    }
    constexpr int h = 1 << (E_LOG - 1 - gl);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      if (j & h) continue;
      const double t = fmodmul(v[j | h], w[tw_slot<Rd::ex>(gl, tw_key<Rd::ex>(gl, j))], qd, qinv);
      v[j | h] = v[j] - t;
      v[j] = v[j] + t;
    }
  });
}

// GS round, stages in reverse order.  FOLD: the sub-transform's stage 0 is the transform's last
// stage; x' = (x + y) c0 and y' = (x - y) c1 (c0 = n^-1 [* scale], c1 = itw[1] n^-1 [* scale]).
template <int S_LOG, int R, uint32_t MASK, bool FOLD>
__device__ __forceinline__ void gs_round_f64(double (&v)[E], const double (&w)[E], double qd, double qinv,
                                             double c0, double c1) {
  using Rd = Round<S_LOG, R>;
  static_for<Rd::er>([&](auto ic) {
    constexpr int gl = Rd::er - 1 - decltype(ic)::value;
    constexpr int g = Rd::g0 + gl;
    if constexpr ((MASK >> g) & 1u) {
#pragma unroll
      for (int j = 0; j < E; ++j) v[j] = freduce(v[j], qd, qinv);
    }
    constexpr int h = 1 << (E_LOG - 1 - gl);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      if (j & h) continue;
      const double x = v[j], y = v[j | h];
      if constexpr (FOLD && g == 0) {
        v[j] = fmodmul(x + y, c0, qd, qinv);
        v[j | h] = fmodmul(x - y, c1, qd, qinv);
      } else {
        v[j] = x + y;
        v[j | h] = fmodmul(x - y, w[tw_slot<Rd::ex>(gl, tw_key<Rd::ex>(gl, j))], qd, qinv);
      }
    }
  });
}

// forward CT round, integer path: values in [0, 8q) (ct_bfly8)
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
      ct_bfly8(v[j], v[j | h], w[sl], ws[sl], q);
    }
  }
}

// forward CT round, integer path for q < 2^60: values in [0, 16q), x reduced only at the stages
// of CMASK (Plan::col_lz / row_lz)
template <int S_LOG, int R, uint32_t CMASK>
__device__ __forceinline__ void ct_round_int16(uint64_t (&v)[E], const uint64_t (&w)[E], const uint64_t (&ws)[E],
                                               uint64_t q) {
  using Rd = Round<S_LOG, R>;
#pragma unroll
  for (int gl = 0; gl < Rd::er; ++gl) {
    const int h = 1 << (E_LOG - 1 - gl);
    const bool reduce = (CMASK >> (Rd::g0 + gl)) & 1u;
#pragma unroll
    for (int j = 0; j < E; ++j) {
      if (j & h) continue;
      const int sl = tw_slot<Rd::ex>(gl, tw_key<Rd::ex>(gl, j));
      if (reduce)
        ct_bfly_c8(v[j], v[j | h], w[sl], ws[sl], q);
      else
        ct_bfly_nored(v[j], v[j | h], w[sl], ws[sl], q);
    }
  }
}

// inverse GS round, integer path: stages in reverse order, values in [0, 4q) (gs_bfly4)
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
      gs_bfly4(v[j], v[j | h], w[sl], ws[sl], q);
    }
  }
}

// inverse GS round, integer path for q < 2^60: values below 8q (gs_bfly8, lazy_gs); B_IN = the
// bound of the round's input in units of q
template <int S_LOG, int R, int B_IN>
__device__ __forceinline__ void gs_round_int8(uint64_t (&v)[E], const uint64_t (&w)[E], const uint64_t (&ws)[E],
                                              uint64_t q) {
  using Rd = Round<S_LOG, R>;
  constexpr LazyGs lz = lazy_gs(Rd::er, B_IN);
#pragma unroll
  for (int gl = Rd::er - 1; gl >= 0; --gl) {
    const int h = 1 << (E_LOG - 1 - gl);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      if (j & h) continue;
      const int sl = tw_slot<Rd::ex>(gl, tw_key<Rd::ex>(gl, j));
      if ((lz.m[gl] >> j) & 1u)
        gs_bfly8<true>(v[j], v[j | h], w[sl], ws[sl], q);
      else
        gs_bfly8<false>(v[j], v[j | h], w[sl], ws[sl], q);
    }
  }
}

// Move a thread-group's values from round RA's layout to round RB's through its LDS tile.
template <int S_LOG, int RA, int RB, typename V, typename Idx, typename Sync>
__device__ __forceinline__ void relayout(V (&v)[E], V* L, Idx idx, Sync sync, uint32_t t) {
  const uint32_t pa = Round<S_LOG, RA>::p_thread(t), pb = Round<S_LOG, RB>::p_thread(t);
#pragma unroll
  for (int j = 0; j < E; ++j) L[idx(pa | Round<S_LOG, RA>::p_elem(j))] = v[j];
  sync();
#pragma unroll
  for (int j = 0; j < E; ++j) v[j] = L[idx(pb | Round<S_LOG, RB>::p_elem(j))];
  sync();
}

struct KArgs {
  const uint64_t* in;
  uint64_t* out;
  const uint64_t* modulus;
  const double* modulus_f;    // q as double
  const double* modulus_inv;  // fl(1/q)
  const uint64_t* tw;         // integer table (forward or inverse)
  const uint64_t* tws;
  const double* col;          // FP64 column table (forward or inverse)
  const double* row_a;        // FP64 row factors (forward or inverse)
  const double* row_b;
  const uint64_t* n_inv;
  const uint64_t* n_inv_shoup;
  const uint64_t* scale;      // optional, per buffer limb
  const uint64_t* scale_shoup;
  LimbMap map;
  int n;
  int limbs;                  // number of processed limbs over all polynomials (excluding skipped)
  int limbs_per_poly;
  const uint64_t* barrett;    // [row][2] (prologue reduction)
  const uint64_t* bcast;      // forward prologue (see ntt.h), column pass only
  size_t bcast_stride;
  NttEpilogue epi;            // forward epilogue (see ntt.h), row pass only
  BconvPrologue bcv;          // forward base-conversion prologue (see ntt.h), column pass only
  NttCopy copy;               // inverse: the row pass also stores its input here (see ntt.h)
};

// y: processed-limb index over the batch -> polynomial, buffer limb within it, table row
__device__ __forceinline__ void resolve_limb(const KArgs& a, int y, int& poly, int& buf_limb, int& row) {
  const LimbMap& m = a.map;
  poly = m.polys > 1 ? y / a.limbs_per_poly : 0;
  int i = y - poly * a.limbs_per_poly;
  if (i >= m.skip_begin + m.skip_index(poly) * m.skip_step) i += (m.skip_end - m.skip_begin);
  buf_limb = i;
  row = i < m.split ? m.first_a + i : m.first_b + (i - m.split);
}

// which arithmetic a pass instantiates: both with a per-limb (wave-uniform) branch, or one alone
constexpr int kKindAny = 0, kKindInt = 1, kKindF64 = 2;
#ifndef PHX_NTT_SPLIT
#define PHX_NTT_SPLIT 1
#endif
// processed limb y of the batch takes the FP64 path (q < 2^50); workgroup-uniform
__device__ __forceinline__ bool limb_is_f64(const KArgs& a, int y) {
  int poly, buf_limb, row;
  resolve_limb(a, y, poly, buf_limb, row);
  return a.modulus[__builtin_amdgcn_readfirstlane(row)] < (1ull << 50);
}

struct LimbCtx {
  uint64_t q;
  double qd, qinv;
  bool f64;
};
__device__ __forceinline__ LimbCtx limb_ctx(const KArgs& a, int row) {
  // row is wave-uniform: readfirstlane lets the per-limb constants come through scalar loads
  row = __builtin_amdgcn_readfirstlane(row);
  LimbCtx c;
  c.q = a.modulus[row];
  c.qd = a.modulus_f[row];
  c.qinv = a.modulus_inv[row];
  c.f64 = c.q < (1ull << 50);
  return c;
}

// Pass outputs use write-through stores (global_store_dwordx2 sc1): the lines leave the XCD's
// L2 at once instead of sitting dirty until the end-of-kernel write-back.  Measured on the
// column/row pass access patterns (tools/ubench_fused.hip, profiles/r01/ubench_fused.txt):
// -2 us per pass at [44][65536].  Plain relaxed atomic stores carry no ordering.
// every buffer these kernels touch is global memory: the explicit global address space keeps a
// pointer the compiler cannot trace to a kernel argument (a key digit read from a pointer table)
// off FLAT instructions, which count in lgkmcnt too and so make every LDS wait also wait for them
using GU64 = __attribute__((address_space(1))) uint64_t;
__device__ __forceinline__ void store_wt(uint64_t* p, uint64_t v) {
  __hip_atomic_store((GU64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t gload_nt(const uint64_t* p) { return __builtin_nontemporal_load((const GU64*)p); }

__device__ __forceinline__ double centered_f64(uint64_t w, uint64_t q) {
  return w > (q >> 1) ? -u52_to_f64(q - w) : u52_to_f64(w);
}

// LDS padding: one pad word every 16 words (row tiles) / one 16-word pad row every 16 rows
// (column tiles) — keeps the transposed rounds' ds_read_b64 accesses conflict-free.
__device__ __forceinline__ uint32_t rpad(uint32_t p) { return p + (p >> 4); }
__device__ __forceinline__ uint32_t cidx(uint32_t p, uint32_t c) { return p * COLS + c + (p >> 4) * COLS; }

// ---------------------------------------------------------------------------------------
// Launch structure: one tile per workgroup, the grid covers every tile and all of it is resident
// at once (2.75 waves per SIMD at [44][65536]).  Every twiddle load of a tile is issued right
// after its data loads, so no twiddle round trip sits between two butterfly rounds.  (Persistent
// grids that prefetch the next tile were measured slower in round 1, profiles/r01/ntt_variants.txt,
// and were removed.)
// ---------------------------------------------------------------------------------------
// PHX_NTT_STAMP = 1 (diagnostic builds only, tools/ntt_timeline.py): every wave of the forward
// passes records s_memrealtime (100 MHz, chip-wide) at entry, when its data has arrived, after
// its butterflies, after its stores are issued and once they are complete, plus HW_ID / XCC_ID,
// into g_ntt_stamps[slot][8] (column pass slots from 0, row pass slots from kStampRow).
#ifndef PHX_NTT_STAMP
#define PHX_NTT_STAMP 0
#endif
#if PHX_NTT_STAMP
constexpr int kStampSlots = 32768, kStampRow = 16384;
static __device__ uint64_t g_ntt_stamps[kStampSlots * 8];
__device__ __forceinline__ void stamp_now(int slot, int i, bool wait) {
  if (wait) __builtin_amdgcn_s_waitcnt(0);
  const uint64_t t = __builtin_amdgcn_s_memrealtime();
  if (slot < kStampSlots && (threadIdx.x & 63) == 0) {
    g_ntt_stamps[slot * 8 + i] = t;
    if (i == 0) {
      g_ntt_stamps[slot * 8 + 5] = __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_ID
      g_ntt_stamps[slot * 8 + 6] = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // XCC_ID
    }
  }
}
#define PHX_STAMP(slot, i, wait) stamp_now(slot, i, wait)
#else
#define PHX_STAMP(slot, i, wait) ((void)0)
#endif

struct TileRef {
  int buf_limb, row, poly;
  size_t off;     // element offset of this lane's first element in the output
  size_t in_off;  // ... and in the input
  size_t k;       // ... and inside its limb
};

// Forward epilogue: out = (c - y) * w (+ out).  Its operand c is loaded with the last round's
// twiddles, so its latency hides under that round's butterflies instead of sitting between the
// last round and the stores; the accumulated `out` (moddown into an existing ciphertext only) is
// read in the store loop, so that no second operand set is held through the round (the finish
// then runs at 3 waves per SIMD without spilling).
struct EpiOperands {
  uint64_t c[E];
};
__device__ __forceinline__ void epilogue_load(const KArgs& a, const TileRef& tr, uint32_t T, EpiOperands& eo) {
  const size_t e = (size_t)tr.buf_limb * a.n + tr.k;
  const uint64_t* c = a.epi.c + tr.poly * a.epi.c_stride + e;
#pragma unroll
  for (int j = 0; j < E; ++j) eo.c[j] = __builtin_nontemporal_load(c + j * T);
}
__device__ __forceinline__ void epilogue_store(const KArgs& a, const TileRef& tr, uint32_t j, uint32_t T,
                                               const EpiOperands& eo, uint64_t y, uint64_t q) {
  const size_t e = (size_t)tr.buf_limb * a.n + tr.k + j * T;
  uint64_t* o = a.epi.ks_out(tr.poly) + e;
  uint64_t v = mul_shoup(sub_mod(eo.c[j], y, q), a.epi.w[tr.buf_limb], a.epi.ws[tr.buf_limb], q);
  if (a.epi.accumulate) v = add_mod(v, __builtin_nontemporal_load(o), q);
  store_wt(o, v);
}

// Key-switch epilogue (NttEpilogue::ks_beta > 0): out = (sum_d tmu[d] evk[d][p] (+ P add) mod q
// - y) w (+ out), the inner product of eval_key_switch.cu:26-85 (128-bit sums, one Barrett-128
// per element) formed where the moddown finish consumes it.  KC (kKsKC) elements at a time;
// the next group's loads are issued before the current group's products.  BETA is a template parameter
// and every load is unconditional (the third operand stream is `out` when accumulating, else the
// addend, else a harmless re-read of tmu), so the compiler can count the loads in flight
// (s_waitcnt vmcnt(N)) instead of draining them all (vmcnt(0)) before every group.
// Elements per load group of the key-switch epilogue / prologue, and waves per SIMD of the
// epilogue's row pass.  One element per group (loads of the next element in flight) at 3 waves
// (158 VGPRs, no spill) beat 4 per group at 2 waves (234 VGPRs): C3 relinearize 0.274-0.288 ->
// 0.268-0.274 ms, bootstrap 23.41-23.57 -> 23.17-23.37 ms (profiles/r03/ks_waves/).
#ifndef PHX_KS_WAVES
#define PHX_KS_WAVES 3
#endif
#ifndef PHX_KSP_WAVES
#define PHX_KSP_WAVES 2
#endif
constexpr int kKsKC = 1, kKsWaves = PHX_KS_WAVES;
constexpr int kKspWaves = PHX_KSP_WAVES;  // ... and of the inverse row pass with the key-switch prologue
#ifndef PHX_EPI_WAVES
#define PHX_EPI_WAVES 3
#endif
constexpr int kEpiWaves = PHX_EPI_WAVES;  // ... and of the row pass with the rescale / moddown finish
// Integer-only launches (IO: every modulus of the table >= 2^50, and < 2^60 for the lazy ranges;
// every limb of the bootstrap chain) instantiate the kernels without the FP64 branch, whose FP64
// twiddles and factors otherwise set the register allocation of the whole kernel: every integer
// pass then fits 4 waves per SIMD without spilling (column 104-110 VGPRs, row 108-128; the mixed
// row passes hold 138-161 at 3 waves).  40-limb C4-chain forward 31.2 -> 30.3 us, 120 limbs
// 78.3 -> 75.2, bootstrap 22.5 -> 21.9 ms, C5 +2% (profiles/r06/ntt_io/).  5 waves on the column
// pass (93 VGPRs with an unpadded, swizzled 32 KB tile) measured slower: 34.6 us.
#ifndef PHX_NTT_IO
#define PHX_NTT_IO 1
#endif
constexpr int kIoColWaves = 4, kIoRowWaves = 4, kIoEpiWaves = 4, kIoKsWaves = 4, kIoKspWaves = 4;
template <int T, int BETA>
__device__ __forceinline__ void ks_epilogue_b(const KArgs& a, const TileRef& tr, const uint64_t (&y)[E], uint64_t q,
                                              uint64_t r0, uint64_t r1) {
  constexpr int KC = kKsKC, NC = E / KC;
  const size_t e = (size_t)tr.buf_limb * a.n + tr.k;
  const bool acc_out = a.epi.accumulate;
  const uint64_t* tm = a.epi.ks_tmu(tr.poly) + e;
  const uint64_t* kp[BETA];
#pragma unroll
  for (int d = 0; d < BETA; ++d) kp[d] = a.epi.evk[d] + (tr.poly & 1) * a.epi.evk_poly_stride + e;
  uint64_t* o = a.epi.ks_out(tr.poly) + e;
  const uint64_t w = a.epi.w[tr.buf_limb], ws = a.epi.ws[tr.buf_limb];
  const uint64_t* ad = a.epi.add_c ? a.epi.ks_add(tr.poly) + e : nullptr;
  const uint64_t pm = ad ? a.epi.pmod[tr.buf_limb] : 0, pms = ad ? a.epi.pmod_shoup[tr.buf_limb] : 0;
  const uint64_t* third = acc_out ? o : (ad ? ad : tm);  // (accumulate and addend never come together)
  uint64_t tb[2][BETA][KC], kb[2][BETA][KC], ob[2][KC];
  auto load = [&](int c, int s) {
#pragma unroll
    for (int d = 0; d < BETA; ++d)
#pragma unroll
      for (int i = 0; i < KC; ++i) {
        tb[s][d][i] = gload_nt(tm + d * a.epi.tmu_stride + (c * KC + i) * T);
        kb[s][d][i] = gload_nt(kp[d] + (c * KC + i) * T);
      }
#pragma unroll
    for (int i = 0; i < KC; ++i) ob[s][i] = gload_nt(third + (c * KC + i) * T);
  };
  load(0, 0);
  static_for<NC>([&](auto cc) {
    constexpr int c = decltype(cc)::value, s = c & 1;
    if constexpr (c + 1 < NC) load(c + 1, s ^ 1);
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      u128 acc{0, 0};
#pragma unroll
      for (int d = 0; d < BETA; ++d) add128(acc, mul_wide(tb[s][d][i], kb[s][d][i]));
      uint64_t cx = barrett_reduce_128(acc, q, r0, r1);
      if (ad) cx = add_mod(cx, mul_shoup(ob[s][i], pm, pms, q), q);
      uint64_t v = mul_shoup(sub_mod(cx, y[c * KC + i], q), w, ws, q);
      if (acc_out) v = add_mod(v, ob[s][i], q);
      store_wt(o + (c * KC + i) * T, v);
    }
  });
}

template <int T>
__device__ __forceinline__ void ks_epilogue(const KArgs& a, const TileRef& tr, const uint64_t (&y)[E], uint64_t q,
                                            uint64_t r0, uint64_t r1) {
  switch (__builtin_amdgcn_readfirstlane(a.epi.ks_beta)) {
    case 1: ks_epilogue_b<T, 1>(a, tr, y, q, r0, r1); break;
    case 2: ks_epilogue_b<T, 2>(a, tr, y, q, r0, r1); break;
    case 3: ks_epilogue_b<T, 3>(a, tr, y, q, r0, r1); break;
    default: break;  // rejected on the host (check_ks)
  }
}

// Key-switch prologue of the inverse row pass (ntt_inverse_ks): x = sum_d tmu[d] evk[d][p] (+ P add)
// mod q for the row's E elements, in KC-element groups whose next loads are issued before the
// current products (as ks_epilogue_b).  The third stream is the addend, else a re-read of tmu.
template <int T, int BETA>
__device__ __forceinline__ void ks_prologue_b(const KArgs& a, const TileRef& tr, uint64_t (&x)[E]) {
  constexpr int KC = kKsKC, NC = E / KC;
  const size_t n = static_cast<size_t>(a.n);
  const size_t tl = a.epi.tmu_limb0 + tr.buf_limb;
  const uint64_t* tm = a.epi.ks_tmu(tr.poly) + tl * n + tr.k;
  const uint64_t* kp[BETA];
#pragma unroll
  for (int d = 0; d < BETA; ++d)
    kp[d] = a.epi.evk[d] + (tr.poly & 1) * a.epi.evk_poly_stride + (size_t)tr.row * n + tr.k;
  const bool add = tr.buf_limb < a.epi.add_limbs;  // wave-uniform
  const uint64_t* ad = add ? a.epi.ks_add(tr.poly) + tl * n + tr.k : tm;
  const uint64_t pm = add ? a.epi.pmod[tl] : 0, pms = add ? a.epi.pmod_shoup[tl] : 0;
  const uint64_t q = a.modulus[tr.row], r0 = a.barrett[2 * tr.row], r1 = a.barrett[2 * tr.row + 1];
  uint64_t tb[2][BETA][KC], kb[2][BETA][KC], ob[2][KC];
  auto load = [&](int c, int s) {
#pragma unroll
    for (int d = 0; d < BETA; ++d)
#pragma unroll
      for (int i = 0; i < KC; ++i) {
        tb[s][d][i] = gload_nt(tm + d * a.epi.tmu_stride + (c * KC + i) * T);
        kb[s][d][i] = gload_nt(kp[d] + (c * KC + i) * T);
      }
#pragma unroll
    for (int i = 0; i < KC; ++i) ob[s][i] = gload_nt(ad + (c * KC + i) * T);
  };
  load(0, 0);
  static_for<NC>([&](auto cc) {
    constexpr int c = decltype(cc)::value, s = c & 1;
    if constexpr (c + 1 < NC) load(c + 1, s ^ 1);
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      u128 acc{0, 0};
#pragma unroll
      for (int d = 0; d < BETA; ++d) add128(acc, mul_wide(tb[s][d][i], kb[s][d][i]));
      uint64_t v = barrett_reduce_128(acc, q, r0, r1);
      if (add) v = add_mod(v, mul_shoup(ob[s][i], pm, pms, q), q);
      x[c * KC + i] = v;
    }
  });
}

template <int T>
__device__ __forceinline__ void ks_prologue(const KArgs& a, const TileRef& tr, uint64_t (&x)[E]) {
  switch (__builtin_amdgcn_readfirstlane(a.epi.ks_beta)) {
    case 1: ks_prologue_b<T, 1>(a, tr, x); break;
    case 2: ks_prologue_b<T, 2>(a, tr, x); break;
    case 3: ks_prologue_b<T, 3>(a, tr, x); break;
    default: break;  // rejected on the host (check_ks)
  }
}

// Row-pass block order of the key-switch epilogue: the polynomials' blocks of one row group are
// dealt to one XCD back to back (blocks b and b + 8 share an XCD under round-robin placement;
// speed only, any placement is correct), so the second polynomial reads tmu from that XCD's L2.
// PHX_ROW_DEAL: the same order for every batched row pass, whose later polynomials then read the
// row group's twiddles (the same limb's table rows) from L2.
#ifndef PHX_ROW_DEAL
#define PHX_ROW_DEAL 1
#endif
__device__ __forceinline__ int ks_row_block(const KArgs& a, int b, int waves, int groups) {
  const int polys = a.map.polys;
  if (polys < 2 || (a.limbs_per_poly * groups) % waves != 0) return b;
  const int per = a.limbs_per_poly * groups / waves;  // blocks per polynomial
  if (per % 8 != 0 || (int)gridDim.x != polys * per) return b;
  const int x = b % 8, k = b / 8;
  return (k % polys) * per + (k / polys) * 8 + x;
}

// Base-conversion prologue (ntt.h BconvPrologue): the tile's 16 elements of output limb j are
// sum_s in[s][k] * mat[s][j] mod q, in two halves of 8 elements; per half the input loads of 4
// limbs are issued together.  30-bit halves: every partial sum of <= 15 products of 30-bit
// values stays below 2^64 (the split of bconv_fixed_kernel, rns.hip), one Barrett-128 per element.
template <int S1_LOG, int S2_LOG, int RF>
__device__ __forceinline__ void bconv_prologue(uint64_t (&x)[E], const KArgs& a, int tile, const TileRef& tr,
                                               uint32_t pf, uint64_t q, uint64_t r0, uint64_t r1) {
  constexpr uint64_t kM30 = (1ull << 30) - 1;
  constexpr int CT = (1 << S2_LOG) / COLS, H = E / 2, SB = 4;
  const int poly = tr.poly;
  const int j = tile / CT - poly * a.limbs_per_poly;  // index among the polynomial's converted limbs
  const int ib = __builtin_amdgcn_readfirstlane(a.bcv.ib[poly]);
  const uint64_t* mat = a.bcv.mat[poly] + j;
  const uint64_t* in = a.bcv.in + poly * a.bcv.in_stride + tr.k;
  const size_t n = static_cast<size_t>(a.n);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint64_t ll[H] = {}, m1[H] = {}, m2[H] = {}, hh[H] = {};
    for (int s0 = 0; s0 < ib; s0 += SB) {
      uint64_t v[SB][H];
#pragma unroll
      for (int u = 0; u < SB; ++u)
#pragma unroll
        for (int e = 0; e < H; ++e)
          v[u][e] = s0 + u < ib ? __builtin_nontemporal_load(in + (size_t)(s0 + u) * n +
                                                             (size_t)(pf | Round<S1_LOG, RF>::p_elem(h * H + e)) * (1 << S2_LOG))
                                : 0;
#pragma unroll
      for (int u = 0; u < SB; ++u) {
        const uint64_t c = s0 + u < ib ? mat[(size_t)(s0 + u) * a.bcv.ob] : 0;
        const uint32_t cl = static_cast<uint32_t>(c & kM30), ch = static_cast<uint32_t>(c >> 30);
#pragma unroll
        for (int e = 0; e < H; ++e) {
          const uint32_t xl = static_cast<uint32_t>(v[u][e] & kM30), xh = static_cast<uint32_t>(v[u][e] >> 30);
          ll[e] += static_cast<uint64_t>(xl) * cl;
          m1[e] += static_cast<uint64_t>(xl) * ch;
          m2[e] += static_cast<uint64_t>(xh) * cl;
          hh[e] += static_cast<uint64_t>(xh) * ch;
        }
      }
    }
#pragma unroll
    for (int e = 0; e < H; ++e) {
      u128 acc{ll[e], 0};
      add128(acc, u128{m1[e] << 30, m1[e] >> 34});
      add128(acc, u128{m2[e] << 30, m2[e] >> 34});
      add128(acc, u128{hh[e] << 60, hh[e] >> 4});
      x[h * H + e] = barrett_reduce_128(acc, q, r0, r1);
    }
  }
}

// Tile order of the base-conversion column pass: the converted limbs of one (polynomial, column
// tile) read the same input tiles, so they are dealt to one XCD back to back (blocks b and b + 8
// share an XCD under round-robin placement; speed only, any placement is correct) and the inputs
// come from that XCD's L2 after the first read.
template <int S2_LOG>
__device__ __forceinline__ int bcv_tile(const KArgs& a, int b) {
  constexpr int CT = (1 << S2_LOG) / COLS;
  const int per = a.limbs_per_poly, groups = a.map.polys * CT;
  if (groups % 8 != 0) return b;
  const int x = b % 8, k = b / 8, g = x + 8 * (k / per), jj = k % per;
  return ((g / CT) * per + jj) * CT + g % CT;
}

// ---------------------------------------------------------------------------------------
// Column pass: tile = COLS consecutive columns x S1 rows of one limb; 256-thread workgroup.
// Any round layout is coalesced here (16 lanes cover one 128 B row segment), so the pass loads
// in the layout of its first round and stores from its last: RN - 1 LDS transposes.
// FWD: first log2(S1) CT stages.  INV: last log2(S1) GS stages (n^-1 and the optional scale).
// ---------------------------------------------------------------------------------------
template <int S2_LOG>
__device__ __forceinline__ TileRef col_ref(const KArgs& a, int tile, uint32_t c) {
  constexpr int CT = (1 << S2_LOG) / COLS;
  TileRef r;
  int poly;
  resolve_limb(a, tile / CT, poly, r.buf_limb, r.row);
  poly = __builtin_amdgcn_readfirstlane(poly);
  r.buf_limb = __builtin_amdgcn_readfirstlane(r.buf_limb);
  r.row = __builtin_amdgcn_readfirstlane(r.row);
  r.poly = poly;
  r.k = (tile % CT) * COLS + c;
  const size_t e = (size_t)r.buf_limb * a.n + r.k;
  r.off = a.map.out_off(poly) + e;
  r.in_off = a.bcast ? poly * a.bcast_stride + r.k : a.map.in_off(poly) + e;
  return r;
}

template <int S1_LOG, int S2_LOG, int RF>
__device__ __forceinline__ void col_load(uint64_t (&x)[E], const uint64_t* src, uint32_t pf) {
#pragma unroll
  for (int j = 0; j < E; ++j)
    x[j] = __builtin_nontemporal_load(src + (size_t)(pf | Round<S1_LOG, RF>::p_elem(j)) * (1 << S2_LOG));
}

// LZ (forward, every modulus of the table < 2^60): the integer path runs with the 16q lazy range
template <int S1_LOG>
constexpr int col_lds_words() { return (Sub<S1_LOG>::S + Sub<S1_LOG>::S / 16) * COLS; }

// One column tile (the calling workgroup's threads tid < NT; `lds`: col_lds_words words).
template <int S1_LOG, int S2_LOG, bool FWD, bool BCV, bool LZ, int KIND>
__device__ __forceinline__ void col_tile(const KArgs& a, int tile, uint64_t* lds, [[maybe_unused]] int sslot) {
  using SB = Sub<S1_LOG>;
  using P = Plan<S1_LOG, S2_LOG>;
  constexpr int T = SB::T, S2 = 1 << S2_LOG, NT = COLS * T, RN = SB::ROUNDS;
  constexpr int RF = FWD ? 0 : RN - 1;  // first round executed
  constexpr int RL = FWD ? RN - 1 : 0;  // last round executed
  static_assert(NT <= CBLOCK, "column tile too large");
  const uint32_t tid = threadIdx.x;
  const uint32_t c = tid % COLS, t = tid / COLS;
  auto idx = [c](uint32_t p) { return cidx(p, c); };
  auto sync = [] { __syncthreads(); };
  const uint32_t pf = Round<S1_LOG, RF>::p_thread(t), pl = Round<S1_LOG, RL>::p_thread(t);
  const uint64_t* src = a.bcast ? a.bcast : a.in;
  {
    const TileRef tr = col_ref<S2_LOG>(a, tile, c);
    uint64_t x[E];
    if constexpr (!BCV) col_load<S1_LOG, S2_LOG, RF>(x, src + tr.in_off, pf);
    const LimbCtx lc = limb_ctx(a, tr.row);
    if constexpr (BCV)
      bconv_prologue<S1_LOG, S2_LOG, RF>(x, a, tile, tr, pf, lc.q, a.barrett[2 * tr.row], a.barrett[2 * tr.row + 1]);
    uint64_t* dst = a.out + tr.off;
    if (FWD && !BCV && a.bcast) {  // prologue: the broadcast limb reduced mod this limb's prime
      const uint64_t r1 = a.barrett[2 * tr.row + 1];
#pragma unroll
      for (int j = 0; j < E; ++j) x[j] = barrett_reduce_64(x[j], lc.q, r1);
    }
    if (KIND == kKindF64 || (KIND == kKindAny && lc.f64)) {
      const double* tab = a.col + (size_t)tr.row * SB::S;
      double w[RN][E];
      static_for<RN>([&](auto rc) {
        constexpr int R = decltype(rc)::value;
        load_tw<S1_LOG, R>(w[R], tab, Round<S1_LOG, R>::p_thread(t), 1);
      });
      double v[E];
#pragma unroll
      for (int j = 0; j < E; ++j) v[j] = FWD ? u52_to_f64(x[j]) : as_f64(x[j]);
      if constexpr (FWD) {
        if constexpr (!BCV) PHX_STAMP(sslot, 1, true);
        static_for<RN>([&](auto rc) {
          constexpr int R = decltype(rc)::value;
          if constexpr (R > 0) relayout<S1_LOG, R - 1, R>(v, reinterpret_cast<double*>(lds), idx, sync, t);
          ct_round_f64<S1_LOG, R, P::col_fwd.mask>(v, w[R], lc.qd, lc.qinv);
        });
        if constexpr (!BCV) PHX_STAMP(sslot, 2, false);
#pragma unroll
        for (int j = 0; j < E; ++j) store_wt(dst + (size_t)(pl | Round<S1_LOG, RL>::p_elem(j)) * S2, as_bits(v[j]));
        if constexpr (!BCV) PHX_STAMP(sslot, 3, false);
        if constexpr (!BCV) PHX_STAMP(sslot, 4, true);
      } else {
        double c0 = tab[0], c1 = tab[1];
        if (a.scale) {
          const double sc = centered_f64(a.scale[tr.buf_limb], lc.q);
          c0 = fmodmul(c0, sc, lc.qd, lc.qinv);
          c1 = fmodmul(c1, sc, lc.qd, lc.qinv);
        }
        static_for<RN>([&](auto rc) {
          constexpr int R = RN - 1 - decltype(rc)::value;
          if constexpr (R < RN - 1) relayout<S1_LOG, R + 1, R>(v, reinterpret_cast<double*>(lds), idx, sync, t);
          gs_round_f64<S1_LOG, R, P::col_inv.mask, true>(v, w[R], lc.qd, lc.qinv, c0, c1);
        });
#pragma unroll
        for (int j = 0; j < E; ++j)
          store_wt(dst + (size_t)(pl | Round<S1_LOG, RL>::p_elem(j)) * S2, f64_to_canonical(v[j], lc.qd, lc.qinv));
      }
    } else {
      const uint64_t* tw = a.tw + (size_t)tr.row * a.n;
      const uint64_t* tws = a.tws + (size_t)tr.row * a.n;
      // integer path (primes >= 2^50): twiddles and Shoup quotients per round
      uint64_t(&v)[E] = x;
      // LZ: forward with the 16q lazy range; stores values < col_lz.out q
      {
        if constexpr (FWD && !BCV) PHX_STAMP(sslot, 1, true);
        static_for<RN>([&](auto rc) {
          constexpr int R = FWD ? decltype(rc)::value : RN - 1 - decltype(rc)::value;
          if constexpr (FWD && R > 0) relayout<S1_LOG, R - 1, R>(v, lds, idx, sync, t);
          if constexpr (!FWD && R < RN - 1) relayout<S1_LOG, R + 1, R>(v, lds, idx, sync, t);
          uint64_t w[E], ws[E];
          load_tw<S1_LOG, R>(w, tw, Round<S1_LOG, R>::p_thread(t), 1);
          load_tw<S1_LOG, R>(ws, tws, Round<S1_LOG, R>::p_thread(t), 1);
          if constexpr (FWD && LZ)
            ct_round_int16<S1_LOG, R, P::col_lz.mask>(v, w, ws, lc.q);
          else if constexpr (FWD)
            ct_round_int<S1_LOG, R>(v, w, ws, lc.q);
          else if constexpr (LZ)
            gs_round_int8<S1_LOG, R, 8>(v, w, ws, lc.q);  // the row pass hands over values < 8q
          else
            gs_round_int<S1_LOG, R>(v, w, ws, lc.q);
        });
        if constexpr (FWD) {
          if constexpr (!BCV) PHX_STAMP(sslot, 2, false);
#pragma unroll
          for (int j = 0; j < E; ++j) store_wt(dst + (size_t)(pl | Round<S1_LOG, RL>::p_elem(j)) * S2, v[j]);  // lazy
          if constexpr (!BCV) PHX_STAMP(sslot, 3, false);
          if constexpr (!BCV) PHX_STAMP(sslot, 4, true);
        } else {
          const uint64_t ni = a.n_inv[tr.row], nis = a.n_inv_shoup[tr.row];
          const uint64_t sc = a.scale ? a.scale[tr.buf_limb] : 1, scs = a.scale ? a.scale_shoup[tr.buf_limb] : 0;
          const bool scaled = sc != 1;  // (a scale of 1 is the identity on canonical values)
#pragma unroll
          for (int j = 0; j < E; ++j) {
            uint64_t y = mul_shoup(v[j], ni, nis, lc.q);
            if (scaled) y = mul_shoup(y, sc, scs, lc.q);
            store_wt(dst + (size_t)(pl | Round<S1_LOG, RL>::p_elem(j)) * S2, y);
          }
        }
      }
    }
  }
}

template <int S1_LOG, int S2_LOG, bool FWD, bool BCV = false, bool LZ = false, bool IO = false>
__global__ __launch_bounds__(CBLOCK, BCV ? 2 : IO ? kIoColWaves : kNttWavesPerEU) void ntt_col(KArgs a) {
  constexpr int NT = COLS * Sub<S1_LOG>::T, CT = (1 << S2_LOG) / COLS;
  __shared__ uint64_t lds[col_lds_words<S1_LOG>()];
  if (threadIdx.x >= NT) return;  // no barrier involves the idle threads' absence (NT is a multiple of 64)
  const int tile = BCV ? bcv_tile<S2_LOG>(a, blockIdx.x) : blockIdx.x;  // workgroup-uniform
  if (tile >= a.limbs * CT) return;
  [[maybe_unused]] const int sslot = blockIdx.x * (CBLOCK / 64) + threadIdx.x / 64;
  if constexpr (FWD && !BCV) PHX_STAMP(sslot, 0, false);
  if constexpr (IO) {
    col_tile<S1_LOG, S2_LOG, FWD, BCV, LZ, kKindInt>(a, tile, lds, sslot);
  } else if constexpr (PHX_NTT_SPLIT) {  // one code path per limb kind, chosen before any load
    if (limb_is_f64(a, tile / CT))
      col_tile<S1_LOG, S2_LOG, FWD, BCV, LZ, kKindF64>(a, tile, lds, sslot);
    else
      col_tile<S1_LOG, S2_LOG, FWD, BCV, LZ, kKindInt>(a, tile, lds, sslot);
  } else {
    col_tile<S1_LOG, S2_LOG, FWD, BCV, LZ, kKindAny>(a, tile, lds, sslot);
  }
}

// ---------------------------------------------------------------------------------------
// Row pass: each wavefront owns RW = 64/T whole rows at a time (T lanes per row), so the
// LDS transposes are wave-private and need no workgroup barrier.  Loads and stores use the
// round-0 layout (p = t + 16 j: 16 lanes cover one 128 B segment).
// FWD: last log2(S2) CT stages, canonical output.  INV: first log2(S2) GS stages.
// FP64 twiddles: tw = A_g(row) * B_g(iloc), both factors loaded (before the prefetch) and
// multiplied after it; round 0's 15 row-uniform twiddles are made once per row through LDS.
// ---------------------------------------------------------------------------------------
template <int S1_LOG, int S2_LOG>
__device__ __forceinline__ TileRef row_ref(const KArgs& a, int item, uint32_t lr, uint32_t t, uint32_t& r) {
  constexpr int S2 = 1 << S2_LOG, RW = cmin(64 / Sub<S2_LOG>::T, 1 << S1_LOG), GROUPS = (1 << S1_LOG) / RW;
  TileRef tr;
  int poly;
  resolve_limb(a, item / GROUPS, poly, tr.buf_limb, tr.row);
  poly = __builtin_amdgcn_readfirstlane(poly);
  tr.buf_limb = __builtin_amdgcn_readfirstlane(tr.buf_limb);
  tr.row = __builtin_amdgcn_readfirstlane(tr.row);
  r = (item % GROUPS) * RW + lr;
  tr.poly = poly;
  tr.k = (size_t)r * S2 + t;
  const size_t e = (size_t)tr.buf_limb * a.n + tr.k;
  tr.off = a.map.out_off(poly) + e;
  tr.in_off = a.map.in_off(poly) + e;
  return tr;
}

template <int S2_LOG>
__device__ __forceinline__ void row_load(uint64_t (&x)[E], const uint64_t* src) {
#pragma unroll
  for (int j = 0; j < E; ++j) x[j] = __builtin_nontemporal_load(src + j * Sub<S2_LOG>::T);
}

// inverse row pass with NttCopy: the loaded input limb stored unchanged into its digit's slot
template <int S2_LOG>
__device__ __forceinline__ void row_copy(const KArgs& a, const TileRef& tr, const uint64_t (&x)[E]) {
  uint64_t* dst = a.copy.out + tr.poly * a.copy.poly_stride + (size_t)(tr.buf_limb / a.copy.alpha) * a.copy.digit_stride +
                  (size_t)tr.buf_limb * a.n + tr.k;
#pragma unroll
  for (int j = 0; j < E; ++j) store_wt(dst + j * Sub<S2_LOG>::T, x[j]);
}

template <int S1_LOG, int S2_LOG>
struct RowShape {
  static constexpr int S1 = 1 << S1_LOG, S2 = 1 << S2_LOG, T = Sub<S2_LOG>::T, RW = cmin(64 / T, S1);
  static constexpr int RSTR = S2 + S2 / 16, WAVES = BLOCK / 64;
  static constexpr int GROUPS = S1 / RW;  // row groups (wave items) per limb
  static constexpr int LDS_WORDS = WAVES * RW * RSTR, TW0 = WAVES * RW * 16;
};

// One row item (the calling wave's RW rows; lds: RowShape::LDS_WORDS words, tw0: RowShape::TW0).
template <int S1_LOG, int S2_LOG, bool FWD, bool EPI, bool LZ, bool KS, int KIND>
__device__ __forceinline__ void row_item(const KArgs& a, int item, uint64_t* lds, double* tw0,
                                         [[maybe_unused]] int sslot) {
  using SB = Sub<S2_LOG>;
  using P = Plan<S1_LOG, S2_LOG>;
  using RS = RowShape<S1_LOG, S2_LOG>;
  constexpr int S1 = RS::S1, S2 = RS::S2, T = RS::T, RW = RS::RW, RSTR = RS::RSTR, RN = SB::ROUNDS;
  constexpr int ER0 = Round<S2_LOG, 0>::er;  // stages of round 0 (its twiddles are row-uniform)
  constexpr int K0 = ((1 << ER0) - 1 + T - 1) / T;  // round-0 twiddles made per lane
  static_assert(Round<S2_LOG, 0>::ex == 0, "round 0 must be a full radix-16 round");
  const uint32_t lane = threadIdx.x % 64, wave = threadIdx.x / 64;
  const uint32_t lr = lane / T, t = lane % T;
  uint64_t* lrow = lds + (wave * RW + lr) * RSTR;
  double* trow = tw0 + (wave * RW + lr) * 16;
  auto idx = [](uint32_t p) { return rpad(p); };
  auto sync = [] { __builtin_amdgcn_wave_barrier(); };
  uint32_t r;
  {
    const TileRef tr = row_ref<S1_LOG, S2_LOG>(a, item, lr, t, r);
    uint64_t x[E];
    if constexpr (!FWD && KS) ks_prologue<T>(a, tr, x);  // ntt_inverse_ks: no input buffer
    else row_load<S2_LOG>(x, a.in + tr.in_off);
    if (!FWD && a.copy.out) row_copy<S2_LOG>(a, tr, x);  // workgroup-uniform branch
    const LimbCtx lc = limb_ctx(a, tr.row);
    uint64_t* dst = a.out + tr.off;
    [[maybe_unused]] EpiOperands eo;
    if (KIND == kKindF64 || (KIND == kKindAny && lc.f64)) {
      const double* A = a.row_a + ((size_t)tr.row * S1 + r) * 16;
      const double* Bt = a.row_b + (size_t)tr.row * S2;
      // raw factors: round 0 (e = t + 1 + T k < 2^ER0) and every later round's slots
      double b0[K0], a0[K0];
#pragma unroll
      for (int k = 0; k < K0; ++k) {
        const uint32_t e = t + 1 + T * k;
        const bool ok = e < (1u << ER0);
        b0[k] = ok ? Bt[e] : 0.0;
        a0[k] = ok ? A[31 - __builtin_clz(e)] : 0.0;
      }
      double bw[RN][E], aw[RN][E_LOG];
      static_for<RN>([&](auto rc) {
        constexpr int R = decltype(rc)::value;
        if constexpr (R > 0) {
          using Rd = Round<S2_LOG, R>;
          const uint32_t pt = Rd::p_thread(t);
#pragma unroll
          for (int gl = 0; gl < Rd::er; ++gl) {
            const int g = Rd::g0 + gl;
            aw[R][gl] = A[g];
#pragma unroll
            for (int key = 0; key < (1 << (gl + Rd::ex)); ++key) {
              const uint32_t p = pt | Rd::p_elem(key_elem<Rd::ex>(gl, key));
              bw[R][tw_slot<Rd::ex>(gl, key)] = Bt[(1u << g) + (p >> (S2_LOG - g))];
            }
          }
        }
      });
#pragma unroll
      for (int k = 0; k < K0; ++k) {
        const uint32_t e = t + 1 + T * k;
        if (e < (1u << ER0)) trow[e] = fmodmul(b0[k], a0[k], lc.qd, lc.qinv);
      }
      double v[E];
#pragma unroll
      for (int j = 0; j < E; ++j) v[j] = FWD ? as_f64(x[j]) : u52_to_f64(x[j]);
      sync();
      auto get_tw = [&](auto rc, double (&w)[E]) {
        constexpr int R = decltype(rc)::value;
        if constexpr (R == 0) {
#pragma unroll
          for (int s = 0; s < (1 << ER0) - 1; ++s) w[s] = trow[s + 1];
        } else {
          using Rd = Round<S2_LOG, R>;
#pragma unroll
          for (int gl = 0; gl < Rd::er; ++gl)
#pragma unroll
            for (int key = 0; key < (1 << (gl + Rd::ex)); ++key) {
              const int s = tw_slot<Rd::ex>(gl, key);
              w[s] = fmodmul(bw[R][s], aw[R][gl], lc.qd, lc.qinv);
            }
        }
      };
      if constexpr (FWD) {
        if constexpr (!EPI) PHX_STAMP(sslot, 1, true);
        static_for<RN>([&](auto rc) {
          constexpr int R = decltype(rc)::value;
          if constexpr (R > 0) relayout<S2_LOG, R - 1, R>(v, reinterpret_cast<double*>(lrow), idx, sync, t);
          double w[E];
          get_tw(rc, w);
          // the epilogue's operands behind the last twiddles: held through the last round only
          if constexpr (EPI && !KS && R == RN - 1) epilogue_load(a, tr, T, eo);
          ct_round_f64<S2_LOG, R, P::row_fwd.mask>(v, w, lc.qd, lc.qinv);
        });
        if constexpr (RN > 1) relayout<S2_LOG, RN - 1, 0>(v, reinterpret_cast<double*>(lrow), idx, sync, t);
        if constexpr (!EPI) PHX_STAMP(sslot, 2, false);
        if constexpr (KS) {
          uint64_t y[E];
#pragma unroll
          for (int j = 0; j < E; ++j) y[j] = f64_to_canonical(v[j], lc.qd, lc.qinv);
          ks_epilogue<T>(a, tr, y, lc.q, a.barrett[2 * tr.row], a.barrett[2 * tr.row + 1]);
        } else if constexpr (EPI) {
#pragma unroll
          for (int j = 0; j < E; ++j) epilogue_store(a, tr, j, T, eo, f64_to_canonical(v[j], lc.qd, lc.qinv), lc.q);
        } else {
#pragma unroll
          for (int j = 0; j < E; ++j) store_wt(dst + j * T, f64_to_canonical(v[j], lc.qd, lc.qinv));
          PHX_STAMP(sslot, 3, false);
          PHX_STAMP(sslot, 4, true);
        }
      } else {
        if constexpr (RN > 1) relayout<S2_LOG, 0, RN - 1>(v, reinterpret_cast<double*>(lrow), idx, sync, t);
        static_for<RN>([&](auto rc) {
          constexpr int R = RN - 1 - decltype(rc)::value;
          if constexpr (R < RN - 1) relayout<S2_LOG, R + 1, R>(v, reinterpret_cast<double*>(lrow), idx, sync, t);
          double w[E];
          get_tw(std::integral_constant<int, R>{}, w);
          gs_round_f64<S2_LOG, R, P::row_inv.mask, false>(v, w, lc.qd, lc.qinv, 0.0, 0.0);
        });
#pragma unroll
        for (int j = 0; j < E; ++j) store_wt(dst + j * T, as_bits(v[j]));  // exact-integer doubles for the column pass
      }
    } else {
      const uint32_t B = (1u << S1_LOG) + r;
      const uint64_t* tw = a.tw + (size_t)tr.row * a.n;
      const uint64_t* tws = a.tws + (size_t)tr.row * a.n;
      uint64_t(&v)[E] = x;
      // rounds after the first (whose twiddles are row-uniform: one broadcast line) read only
      // the Shoup quotients and derive w (w_from_shoup): half the row pass's twiddle bytes (the
      // (S1 + row)-indexed tables are ~2x the data; inverse -1.5 us, profiles/r03/ntt_experiments/twd_*.txt)
      auto get_tw = [&](auto rc, uint64_t (&w)[E], uint64_t (&ws)[E]) {
        constexpr int R = decltype(rc)::value;
        if constexpr (R == 0) {
          load_tw<S2_LOG, R>(w, tw, Round<S2_LOG, R>::p_thread(t), B);
          load_tw<S2_LOG, R>(ws, tws, Round<S2_LOG, R>::p_thread(t), B);
        } else {
          load_tw<S2_LOG, R>(ws, tws, Round<S2_LOG, R>::p_thread(t), B);
          w_from_shoup_round<S2_LOG, R>(w, ws, lc.q);
        }
      };
      if constexpr (FWD) {
        // LZ: the 16q lazy range; the input is the column pass's lazy output
        {
          if constexpr (!EPI) PHX_STAMP(sslot, 1, true);
          static_for<RN>([&](auto rc) {
            constexpr int R = decltype(rc)::value;
            if constexpr (R > 0) relayout<S2_LOG, R - 1, R>(v, lrow, idx, sync, t);
            uint64_t w[E], ws[E];
            get_tw(rc, w, ws);
            if constexpr (EPI && !KS && R == RN - 1) epilogue_load(a, tr, T, eo);  // behind the last twiddles
            if constexpr (LZ)
              ct_round_int16<S2_LOG, R, P::row_lz.mask>(v, w, ws, lc.q);
            else
              ct_round_int<S2_LOG, R>(v, w, ws, lc.q);
          });
          if constexpr (RN > 1) relayout<S2_LOG, RN - 1, 0>(v, lrow, idx, sync, t);
          [[maybe_unused]] const float rq = static_cast<float>(4294967296.0 / static_cast<double>(lc.q));
          auto canon = [&](uint64_t y) {
            if constexpr (LZ && P::row_lz.out > 8) return reduce16_est(y, lc.q, rq);
            else return reduce8(y, lc.q);
          };
          if constexpr (KS) {
            uint64_t y[E];
#pragma unroll
            for (int j = 0; j < E; ++j) y[j] = canon(v[j]);
            ks_epilogue<T>(a, tr, y, lc.q, a.barrett[2 * tr.row], a.barrett[2 * tr.row + 1]);
          } else if constexpr (EPI) {
#pragma unroll
            for (int j = 0; j < E; ++j) epilogue_store(a, tr, j, T, eo, canon(v[j]), lc.q);
          } else {
            PHX_STAMP(sslot, 2, false);
#pragma unroll
            for (int j = 0; j < E; ++j) store_wt(dst + j * T, canon(v[j]));
            PHX_STAMP(sslot, 3, false);
            PHX_STAMP(sslot, 4, true);
          }
        }
      } else {
        if constexpr (RN > 1) relayout<S2_LOG, 0, RN - 1>(v, lrow, idx, sync, t);
        static_for<RN>([&](auto rc) {
          constexpr int R = RN - 1 - decltype(rc)::value;
          if constexpr (R < RN - 1) relayout<S2_LOG, R + 1, R>(v, lrow, idx, sync, t);
          uint64_t w[E], ws[E];
          get_tw(std::integral_constant<int, R>{}, w, ws);
          if constexpr (LZ)
            gs_round_int8<S2_LOG, R, R == RN - 1 ? 4 : 8>(v, w, ws, lc.q);  // input < 4q, as gs_bfly4
          else
            gs_round_int<S2_LOG, R>(v, w, ws, lc.q);
        });
#pragma unroll
        for (int j = 0; j < E; ++j) store_wt(dst + j * T, v[j]);  // [0, 4q) ([0, 8q) LZ), column pass follows
      }
    }
  }
}

// The epilogue form holds its operands (EpiOperands) through the butterflies: two waves per SIMD
// give it the registers to do so without spilling (168 VGPRs at three waves spilled 47).
// KS: forward, the epilogue is the key-switch form (ks_epilogue; EPI must be set too); inverse, the
// input is the key-switch prologue (ks_prologue).
template <int S1_LOG, int S2_LOG, bool FWD, bool EPI = false, bool LZ = false, bool KS = false, bool IO = false>
__global__ __launch_bounds__(BLOCK, IO ? (KS ? (FWD ? kIoKsWaves : kIoKspWaves) : EPI ? kIoEpiWaves : kIoRowWaves)
                                      : KS ? (FWD ? kKsWaves : kKspWaves) : EPI ? kEpiWaves : kRowWaves)
void ntt_row(KArgs a) {
  using RS = RowShape<S1_LOG, S2_LOG>;
  __shared__ uint64_t lds[RS::LDS_WORDS];
  __shared__ double tw0[RS::TW0];
  const int wave = threadIdx.x / 64;
  const int blk = (KS || PHX_ROW_DEAL) ? ks_row_block(a, blockIdx.x, RS::WAVES, RS::GROUPS) : (int)blockIdx.x;
  const int item = __builtin_amdgcn_readfirstlane(blk * RS::WAVES + wave);
  if (item >= a.limbs * RS::GROUPS) return;  // no workgroup barrier in this kernel
#if PHX_NTT_STAMP
  const int sslot = kStampRow + blockIdx.x * RS::WAVES + wave;
#else
  const int sslot = 0;
#endif
  if constexpr (FWD && !EPI) PHX_STAMP(sslot, 0, false);
  if constexpr (IO) {
    row_item<S1_LOG, S2_LOG, FWD, EPI, LZ, KS, kKindInt>(a, item, lds, tw0, sslot);
  } else if constexpr (PHX_NTT_SPLIT) {  // one code path per limb kind, chosen before any load
    if (limb_is_f64(a, item / RS::GROUPS))
      row_item<S1_LOG, S2_LOG, FWD, EPI, LZ, KS, kKindF64>(a, item, lds, tw0, sslot);
    else
      row_item<S1_LOG, S2_LOG, FWD, EPI, LZ, KS, kKindInt>(a, item, lds, tw0, sslot);
  } else {
    row_item<S1_LOG, S2_LOG, FWD, EPI, LZ, KS, kKindAny>(a, item, lds, tw0, sslot);
  }
}
// ---------------------------------------------------------------------------------------
// 1-D path for small transforms, n = 2^8 .. 2^11 (the reference's radix-2 fnwt_1d / inwt_1d,
// src/ntt/ntt_1d.cu): one workgroup of n/2 threads per limb, the limb in LDS, one butterfly per
// thread and stage, the reference's in-place loop order and twiddle indices (tw[m + j]).  Integer
// Shoup butterflies for every prime; the prologue / epilogue / scale of the 2-D path are honoured
// so every launcher works at these degrees.
// ---------------------------------------------------------------------------------------
constexpr int kMaxLog1D = 11;

template <bool FWD>
__global__ __launch_bounds__(1024) void ntt_1d(KArgs a) {
  __shared__ uint64_t v[1 << kMaxLog1D];
  const int n = a.n, half = n >> 1;
  int poly, buf_limb, row;
  resolve_limb(a, blockIdx.x, poly, buf_limb, row);
  poly = __builtin_amdgcn_readfirstlane(poly);
  buf_limb = __builtin_amdgcn_readfirstlane(buf_limb);
  row = __builtin_amdgcn_readfirstlane(row);
  const uint64_t q = a.modulus[row], q2 = q << 1;
  const uint64_t* tw = a.tw + (size_t)row * n;
  const uint64_t* tws = a.tws + (size_t)row * n;
  const size_t e0 = (size_t)buf_limb * n;
  const uint32_t i = threadIdx.x;
  for (int k = i; k < n; k += half) {
    uint64_t x;
    if (FWD && a.bcast) x = barrett_reduce_64(a.bcast[poly * a.bcast_stride + k], q, a.barrett[2 * row + 1]);
    else x = a.in[a.map.in_off(poly) + e0 + k];
    v[k] = x;
  }
  __syncthreads();
  if constexpr (FWD) {
    for (int m = 1, t = half; m < n; m <<= 1, t >>= 1) {
      const int j = i / t, k = i % t, i1 = 2 * j * t + k;
      uint64_t x = v[i1], y = v[i1 + t];
      ct_bfly(x, y, tw[m + j], tws[m + j], q);
      v[i1] = x;
      v[i1 + t] = y;
      __syncthreads();
    }
  } else {
    for (int m = half, t = 1; m >= 1; m >>= 1, t <<= 1) {
      const int j = i / t, k = i % t, i1 = 2 * j * t + k;
      uint64_t x = v[i1], y = v[i1 + t];
      gs_bfly(x, y, tw[m + j], tws[m + j], q);
      v[i1] = x;
      v[i1 + t] = y;
      __syncthreads();
    }
  }
  uint64_t* out = a.out + a.map.out_off(poly) + e0;
  for (int k = i; k < n; k += half) {
    uint64_t y = v[k];
    if constexpr (FWD) {
      y = csub(csub(y, q2), q);
      if (a.epi.out) {
        uint64_t* o = a.epi.ks_out(poly) + e0 + k;
        uint64_t r = mul_shoup(sub_mod(a.epi.c[poly * a.epi.c_stride + e0 + k], y, q), a.epi.w[buf_limb],
                               a.epi.ws[buf_limb], q);
        if (a.epi.accumulate) r = add_mod(r, *o, q);
        *o = r;
        continue;
      }
    } else {
      y = mul_shoup(y, a.n_inv[row], a.n_inv_shoup[row], q);
      if (a.scale) y = mul_shoup(y, a.scale[buf_limb], a.scale_shoup[buf_limb], q);
    }
    out[k] = y;
  }
}


template <int S1_LOG, int S2_LOG>
hipError_t launch(const NttTables& tb, const uint64_t* in, uint64_t* out, const LimbMap& map, bool inverse,
                  const uint64_t* scale, const uint64_t* scale_shoup, hipStream_t stream,
                  const uint64_t* bcast = nullptr, size_t bcast_stride = 0, const NttEpilogue& epi = NttEpilogue{},
                  const BconvPrologue* bcv = nullptr, const NttCopy& copy = NttCopy{}) {
  const int per_poly = map.num_limbs - (map.skip_end - map.skip_begin);
  if (per_poly <= 0 || map.polys <= 0) return hipSuccess;
  const int limbs = per_poly * map.polys;
  KArgs a;
  a.in = in; a.out = out; a.modulus = tb.modulus;
  a.modulus_f = tb.modulus_f; a.modulus_inv = tb.modulus_inv;
  a.tw = inverse ? tb.itw : tb.tw;
  a.tws = inverse ? tb.itw_shoup : tb.tw_shoup;
  a.col = inverse ? tb.col_inv : tb.col_fwd;
  a.row_a = inverse ? tb.row_a_inv : tb.row_a_fwd;
  a.row_b = inverse ? tb.row_b_inv : tb.row_b_fwd;
  a.n_inv = tb.n_inv; a.n_inv_shoup = tb.n_inv_shoup;
  a.scale = scale; a.scale_shoup = scale_shoup;
  a.map = map; a.n = (int)tb.n; a.limbs = limbs; a.limbs_per_poly = per_poly;
  a.barrett = tb.barrett;
  a.bcast = bcast; a.bcast_stride = bcast_stride;
  a.epi = epi;
  if (bcv) a.bcv = *bcv;
  if (inverse) a.copy = copy;
  if (a.map.in_stride == 0) a.map.in_stride = (size_t)map.num_limbs * tb.n;
  if (a.map.out_stride == 0) a.map.out_stride = (size_t)map.num_limbs * tb.n;
  constexpr int S1 = 1 << S1_LOG, S2 = 1 << S2_LOG;
  constexpr int RW = cmin(64 / Sub<S2_LOG>::T, S1);
  const int col_tiles = limbs * (S2 / COLS);
  const int row_items = limbs * (S1 / RW);
  const int row_groups = (row_items + BLOCK / 64 - 1) / (BLOCK / 64);
  const dim3 grid_c(col_tiles), grid_r(row_groups);
  // column tiles of small transforms need fewer than BLOCK threads (rounded up to a wavefront)
  const dim3 block_c(std::max(64, COLS * Sub<S1_LOG>::T)), block_r(BLOCK);
  // integer-only instantiations (IO) for degrees >= 2^14 (the bootstrap's): the FP64 branch is
  // compiled out, so the kernels' registers are the integer path's alone
  constexpr bool kIO = PHX_NTT_IO && S1_LOG + S2_LOG >= 14;
  if (!inverse) {
    NttEpilogue epi_row = a.epi;
    a.epi = NttEpilogue{};  // the column pass stores its intermediate
    // one lazy range for the whole launch: both passes must agree on the intermediate's bound
    const bool lz = tb.lazy16;
    const bool io = kIO && lz && tb.int_only;
    if (bcv && io)
      hipLaunchKernelGGL((ntt_col<S1_LOG, S2_LOG, true, true, true, kIO>), grid_c, block_c, 0, stream, a);
    else if (bcv && lz)
      hipLaunchKernelGGL((ntt_col<S1_LOG, S2_LOG, true, true, true>), grid_c, block_c, 0, stream, a);
    else if (bcv)
      hipLaunchKernelGGL((ntt_col<S1_LOG, S2_LOG, true, true, false>), grid_c, block_c, 0, stream, a);
    else if (io)
      hipLaunchKernelGGL((ntt_col<S1_LOG, S2_LOG, true, false, true, kIO>), grid_c, block_c, 0, stream, a);
    else if (lz)
      hipLaunchKernelGGL((ntt_col<S1_LOG, S2_LOG, true, false, true>), grid_c, block_c, 0, stream, a);
    else
      hipLaunchKernelGGL((ntt_col<S1_LOG, S2_LOG, true, false, false>), grid_c, block_c, 0, stream, a);
    a.in = out;
    a.map.in_stride = a.map.out_stride;
    a.map.in_outer = a.map.out_outer;
    a.bcast = nullptr;  // the row pass reads the intermediate
    a.epi = epi_row;
    if (a.epi.out && a.epi.ks_beta > 0 && io)
      hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, true, true, true, true, kIO>), grid_r, block_r, 0, stream, a);
    else if (a.epi.out && a.epi.ks_beta > 0 && lz)
      hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, true, true, true, true>), grid_r, block_r, 0, stream, a);
    else if (a.epi.out && a.epi.ks_beta > 0)
      hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, true, true, false, true>), grid_r, block_r, 0, stream, a);
    else if (a.epi.out && io)
      hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, true, true, true, false, kIO>), grid_r, block_r, 0, stream, a);
    else if (a.epi.out && lz)
      hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, true, true, true>), grid_r, block_r, 0, stream, a);
    else if (a.epi.out)
      hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, true, true, false>), grid_r, block_r, 0, stream, a);
    else if (io)
      hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, true, false, true, false, kIO>), grid_r, block_r, 0, stream, a);
    else if (lz)
      hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, true, false, true>), grid_r, block_r, 0, stream, a);
    else
      hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, true, false, false>), grid_r, block_r, 0, stream, a);
  } else {
    // one lazy range for the whole launch, as forward
    const bool lz = tb.lazy16;
    const bool io = kIO && lz && tb.int_only;
    if (a.epi.ks_beta > 0 && io)
      hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, false, false, true, true, kIO>), grid_r, block_r, 0, stream, a);
    else if (a.epi.ks_beta > 0 && lz)
      hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, false, false, true, true>), grid_r, block_r, 0, stream, a);
    else if (a.epi.ks_beta > 0)
      hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, false, false, false, true>), grid_r, block_r, 0, stream, a);
    else if (io)
      hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, false, false, true, false, kIO>), grid_r, block_r, 0, stream, a);
    else if (lz)
      hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, false, false, true>), grid_r, block_r, 0, stream, a);
    else
      hipLaunchKernelGGL((ntt_row<S1_LOG, S2_LOG, false>), grid_r, block_r, 0, stream, a);
    a.in = out;
    a.map.in_stride = a.map.out_stride;
    a.map.in_outer = a.map.out_outer;
    a.copy = NttCopy{};  // the row pass made the copy
    a.epi = NttEpilogue{};  // ... and consumed the key-switch prologue
    if (io)
      hipLaunchKernelGGL((ntt_col<S1_LOG, S2_LOG, false, false, true, kIO>), grid_c, block_c, 0, stream, a);
    else if (lz)
      hipLaunchKernelGGL((ntt_col<S1_LOG, S2_LOG, false, false, true>), grid_c, block_c, 0, stream, a);
    else
      hipLaunchKernelGGL((ntt_col<S1_LOG, S2_LOG, false>), grid_c, block_c, 0, stream, a);
  }
  return hipGetLastError();
}

}  // namespace nttd
}  // namespace phx
