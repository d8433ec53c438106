// Micro-benchmark (tools only): does a streaming (software-pipelined) column pass beat the
// all-resident one?  Column pass of a forward FP64 NTT with the N = 64 x 1024 split (tiles of 16
// columns x 64 rows, one wave each; 44 limbs -> 2,816 tiles = 11 per CU), built from the engine's
// own round / relayout helpers (ntt.hip is included).  Timing only: the data is random residues
// of one 50-bit prime, transformed in place (values stay finite doubles).
//
//  resident : one wave per tile, the grid covers every tile (today's structure)
//  stream<D>: 256 workgroups x 4 waves; the 11 tiles of a workgroup are dealt to its waves
//             (3, 3, 3, 2), each wave loads D tiles ahead of the one it transforms
//  skeleton variants: the same data movement with the butterflies removed
#include "../phantom-fhe-boot_amd/csrc/ntt.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

namespace phx {
namespace {
constexpr int kS1 = 6, kS2 = 10, kN = 1 << 16, kL = 44, kCT = (1 << kS2) / 16, kTiles = kL * kCT;
using SB6 = Sub<kS1>;
using P610 = Plan<kS1, kS2>;
constexpr int kRN = SB6::ROUNDS;  // 2
constexpr int kLdsTile = (SB6::S + SB6::S / 16) * 16;

struct Ctx {
  double q, qinv;
  const double* tab;
};

template <bool COMPUTE>
__device__ __forceinline__ void tile_body(uint64_t (&x)[E], uint64_t* d, int tile, const Ctx& cx, uint64_t* L,
                                          uint32_t c, uint32_t t, const double (&w)[kRN][E]) {
  const int limb = tile / kCT;
  uint64_t* base = d + (size_t)limb * kN + (tile % kCT) * 16 + c;
  constexpr int RL = kRN - 1;
  const uint32_t pl = Round<kS1, RL>::p_thread(t);
  if constexpr (COMPUTE) {
    double v[E];
#pragma unroll
    for (int j = 0; j < E; ++j) v[j] = u52_to_f64(x[j] & 0x000FFFFFFFFFFFFFull);
    auto idx = [c](uint32_t p) { return cidx(p, c); };
    auto sync = [] { __builtin_amdgcn_wave_barrier(); };
    static_for<kRN>([&](auto rc) {
      constexpr int R = decltype(rc)::value;
      if constexpr (R > 0) relayout<kS1, R - 1, R>(v, reinterpret_cast<double*>(L), idx, sync, t);
      ct_round_f64<kS1, R, P610::col_fwd.mask>(v, w[R], cx.q, cx.qinv);
    });
#pragma unroll
    for (int j = 0; j < E; ++j) store_wt(base + (size_t)(pl | Round<kS1, RL>::p_elem(j)) * (1 << kS2), as_bits(v[j]) & 0x000FFFFFFFFFFFFFull);
  } else {
#pragma unroll
    for (int j = 0; j < E; ++j) store_wt(base + (size_t)(Round<kS1, 0>::p_thread(t) | Round<kS1, 0>::p_elem(j)) * (1 << kS2), x[j] + 1);
  }
}

__device__ __forceinline__ void tile_load(uint64_t (&x)[E], const uint64_t* d, int tile, uint32_t c, uint32_t t) {
  const int limb = tile / kCT;
  const uint64_t* base = d + (size_t)limb * kN + (tile % kCT) * 16 + c;
  const uint32_t pf = Round<kS1, 0>::p_thread(t);
#pragma unroll
  for (int j = 0; j < E; ++j) x[j] = __builtin_nontemporal_load(base + (size_t)(pf | Round<kS1, 0>::p_elem(j)) * (1 << kS2));
}

__device__ __forceinline__ void tw_load(double (&w)[kRN][E], const Ctx& cx, uint32_t t) {
  static_for<kRN>([&](auto rc) {
    constexpr int R = decltype(rc)::value;
    load_tw<kS1, R>(w[R], cx.tab, Round<kS1, R>::p_thread(t), 1);
  });
}

template <bool COMPUTE>
__global__ __launch_bounds__(64) void col_resident(uint64_t* d, Ctx cx) {
  __shared__ uint64_t lds[kLdsTile];
  const uint32_t lane = threadIdx.x, c = lane % 16, t = lane / 16;
  uint64_t x[E];
  tile_load(x, d, blockIdx.x, c, t);
  double w[kRN][E];
  if constexpr (COMPUTE) tw_load(w, cx, t);
  tile_body<COMPUTE>(x, d, blockIdx.x, cx, lds, c, t, w);
}

// D = tiles loaded ahead (1 or 2)
template <bool COMPUTE, int D>
__global__ __launch_bounds__(256, 1) void col_stream(uint64_t* d, Ctx cx) {
  __shared__ uint64_t lds[4 * kLdsTile];
  const uint32_t wave = threadIdx.x / 64, lane = threadIdx.x % 64, c = lane % 16, t = lane / 16;
  uint64_t* L = lds + wave * kLdsTile;
  const int base = blockIdx.x * 11 + wave;
  const int cnt = wave < 3 ? 3 : 2;  // tiles base, base + 4, base + 8 (wave 3: two)
  double w[kRN][E];
  uint64_t x[D + 1][E];
  tile_load(x[0], d, base, c, t);
  if constexpr (COMPUTE) tw_load(w, cx, t);
  if constexpr (D >= 2) tile_load(x[1], d, base + 4, c, t);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (k < cnt) {
      if (k + D < cnt) tile_load(x[(k + D) % (D + 1)], d, base + 4 * (k + D), c, t);
      tile_body<COMPUTE>(x[k % (D + 1)], d, base + 4 * k, cx, L, c, t, w);
    }
  }
}
}  // namespace
}  // namespace phx

using namespace phx;

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int ring = 15, reps = 60;
  const size_t tot = (size_t)kN * kL;
  const double q = 1125899906826241.0;  // a 50-bit NTT prime (2^50 - 2^17 + 1 form not required here)
  std::vector<uint64_t> h(tot);
  uint64_t s = 1;
  for (auto& v : h) { s = s * 6364136223846793005ull + 1442695040888963407ull; v = (s >> 14) % (uint64_t)q; }
  std::vector<uint64_t*> buf(ring);
  for (auto& b : buf) { CK(hipMalloc(&b, tot * 8)); CK(hipMemcpy(b, h.data(), tot * 8, hipMemcpyHostToDevice)); }
  std::vector<double> th(64);
  for (int i = 0; i < 64; ++i) th[i] = (double)((i * 7919 + 13) % 100000) - 50000.0;
  double* tab; CK(hipMalloc(&tab, 64 * 8)); CK(hipMemcpy(tab, th.data(), 64 * 8, hipMemcpyHostToDevice));
  Ctx cx{q, 1.0 / q, tab};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto time = [&](const char* name, auto launch) {
    for (int i = 0; i < 10; ++i) launch(buf[i % ring]);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch(buf[i % ring]);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1000 / reps;
    printf("%-28s stream-avg %7.2f us  %7.1f GB/s (16 B/coef)\n", name, us, tot * 16.0 / us / 1e3);
    return 0;
  };
  time("resident skeleton", [&](uint64_t* b) { col_resident<false><<<kTiles, 64>>>(b, cx); });
  time("resident compute", [&](uint64_t* b) { col_resident<true><<<kTiles, 64>>>(b, cx); });
  time("stream D1 skeleton", [&](uint64_t* b) { col_stream<false, 1><<<kTiles / 11, 256>>>(b, cx); });
  time("stream D1 compute", [&](uint64_t* b) { col_stream<true, 1><<<kTiles / 11, 256>>>(b, cx); });
  time("stream D2 skeleton", [&](uint64_t* b) { col_stream<false, 2><<<kTiles / 11, 256>>>(b, cx); });
  time("stream D2 compute", [&](uint64_t* b) { col_stream<true, 2><<<kTiles / 11, 256>>>(b, cx); });
  return 0;
}
