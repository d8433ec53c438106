// Micro-benchmark (tools only): what does a single-launch, two-phase NTT data movement cost on
// gfx950 compared with two launches?  Phase 1 moves column tiles (16 cols x 256 rows, the
// column-pass pattern), phase 2 row tiles, in place on [44][65536] u64 limbs; +1 stands in for
// the butterflies.  Buffer ring of 15 (> 256 MiB Infinity Cache) as in bench.py.
//
//  two-pass   : coltile kernel then rowtile kernel (today's structure)
//  fused<G,F> : one launch; G workgroups per limb, all co-resident; after phase 1 each workgroup
//               publishes its tiles and bumps the limb's counter; phase 2 waits for G arrivals.
//               F = 0: plain stores + agent release/acquire fences; F = 1: sc1 (write-through)
//               stores and sc1 loads (MI355X_MICROARCH.md §Workgroup dispatch, Valid forms).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int N = 1 << 16, L = 44, S1 = 256, S2 = 256;
constexpr size_t TOT = (size_t)N * L;

__device__ __forceinline__ uint64_t ld_sc1(const uint64_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_sc1(uint64_t* p, uint64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

template <int ST>  // 0 plain, 1 nt, 2 sc1
__device__ __forceinline__ void st(uint64_t* p, uint64_t v) {
  if constexpr (ST == 0) *p = v;
  else if constexpr (ST == 1) __builtin_nontemporal_store(v, p);
  else st_sc1(p, v);
}

template <int ST>
__global__ __launch_bounds__(256) void touch8(uint64_t* d, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) st<ST>(d + i, d[i] + 1);
}

// column tile: 16 cols x 256 rows; 256 threads: c = tid % 16, t = tid / 16, rows t + 16 j
template <int ST, bool SC1LD>
__device__ __forceinline__ void col_tile(uint64_t* d, int limb, int ct) {
  const int c = threadIdx.x % 16, t = threadIdx.x / 16;
  uint64_t* base = d + (size_t)limb * N + ct * 16 + c;
  uint64_t v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = SC1LD ? ld_sc1(base + (size_t)(t + 16 * j) * S2) : base[(size_t)(t + 16 * j) * S2];
#pragma unroll
  for (int j = 0; j < 16; ++j) st<ST>(base + (size_t)(t + 16 * j) * S2, v[j] + 1);
}
// row item: 4 rows per wave, lane t = lane % 16 holds t + 16 j
template <int ST, bool SC1LD>
__device__ __forceinline__ void row_item(uint64_t* d, int limb, int r4) {
  const int lane = threadIdx.x % 64, lr = lane / 16, t = lane % 16;
  uint64_t* base = d + (size_t)limb * N + (size_t)(r4 * 4 + lr) * S2 + t;
  uint64_t v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = SC1LD ? ld_sc1(base + 16 * j) : base[16 * j];
#pragma unroll
  for (int j = 0; j < 16; ++j) st<ST>(base + 16 * j, v[j] + 1);
}

template <int ST>
__global__ __launch_bounds__(256) void colpass(uint64_t* d) {
  const int tile = blockIdx.x;  // L * 16 tiles
  col_tile<ST, false>(d, tile / 16, tile % 16);
}
template <int ST>
__global__ __launch_bounds__(256) void rowpass(uint64_t* d) {
  const int item = blockIdx.x * 4 + threadIdx.x / 64;  // L * 64 items
  row_item<ST, false>(d, item / 64, item % 64);
}

// XCD-aware two-pass: block b: x = b % 8, j = b / 8, limb = x + 8 (j / 16), part = j % 16, so
// every workgroup touching limb i runs on the XCD of blocks = i (mod 8) (round-robin placement).
template <int ST>
__global__ __launch_bounds__(256) void colpass_x(uint64_t* d) {
  const int b = blockIdx.x, x = b % 8, j = b / 8, limb = x + 8 * (j / 16);
  if (limb >= L) return;
  col_tile<ST, false>(d, limb, j % 16);
}
template <int ST>
__global__ __launch_bounds__(256) void rowpass_x(uint64_t* d) {
  const int b = blockIdx.x, x = b % 8, j = b / 8, limb = x + 8 * (j / 16);
  if (limb >= L) return;
  row_item<ST, false>(d, limb, (j % 16) * 4 + threadIdx.x / 64);
}

// fused: grid = 8 * G * ceil(L / 8).  Block b: x = b % 8 (blocks sharing an XCD under round-robin
// placement, speed only), j = b / 8; limb = x + 8 (j / G), part = j % G.
template <int G, int F>
__global__ __launch_bounds__(256) void fused(uint64_t* d, unsigned* counters, unsigned epoch, unsigned* timeout) {
  const int b = blockIdx.x, x = b % 8, j = b / 8;
  const int limb = x + 8 * (j / G), part = j % G;
  if (limb >= L) return;
  constexpr int CT = 16 / G;  // column tiles per workgroup
  for (int k = 0; k < CT; ++k) {
    if (F == 1) col_tile<2, false>(d, limb, part * CT + k);
    else col_tile<0, false>(d, limb, part * CT + k);
  }
  // publish
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (F == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(counters + limb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = (epoch + 1) * G;
    unsigned spins = 0;
    while (__hip_atomic_load(counters + limb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 16)) { atomicAdd(timeout, 1u); break; }
    }
    if (F == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  constexpr int RI = 64 / G / 4;  // row items (4 rows) per wave
  const int w = threadIdx.x / 64;
  for (int k = 0; k < RI; ++k) {
    const int r4 = part * (64 / G) + w * RI + k;
    if (F == 1) row_item<0, true>(d, limb, r4);
    else row_item<0, false>(d, limb, r4);
  }
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int ring = 15, reps = 60;
  std::vector<uint64_t*> buf(ring);
  for (auto& b : buf) { CK(hipMalloc(&b, TOT * 8)); CK(hipMemset(b, 0, TOT * 8)); }
  unsigned *counters, *tmo;
  CK(hipMalloc(&counters, 64 * sizeof(unsigned))); CK(hipMemset(counters, 0, 64 * sizeof(unsigned)));
  CK(hipMalloc(&tmo, sizeof(unsigned))); CK(hipMemset(tmo, 0, sizeof(unsigned)));
  unsigned epoch = 0;
  auto time = [&](const char* name, auto launch) {
    CK(hipDeviceSynchronize());
    CK(hipMemset(counters, 0, 64 * sizeof(unsigned)));
    CK(hipDeviceSynchronize());
    epoch = 0;
    for (int i = 0; i < 10; ++i) launch(buf[i % ring]);
    CK(hipDeviceSynchronize());
    // (a) per-launch event timing, median
    std::vector<float> ts;
    for (int i = 0; i < reps; ++i) {
      CK(hipEventRecord(e0)); launch(buf[i % ring]); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms * 1000);
    }
    std::sort(ts.begin(), ts.end());
    // (b) back-to-back stream of launches, average
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch(buf[i % ring]);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1000 / reps;
    printf("%-30s median %7.2f us  stream-avg %7.2f us  %7.1f GB/s (16 B/coef, stream)\n", name, ts[ts.size() / 2], us,
           TOT * 16.0 / us / 1e3);
    return 0;
  };
  time("touch8 plain", [&](uint64_t* b) { touch8<0><<<2048, 256>>>(b, TOT); });
  time("touch8 nt", [&](uint64_t* b) { touch8<1><<<2048, 256>>>(b, TOT); });
  time("touch8 sc1", [&](uint64_t* b) { touch8<2><<<2048, 256>>>(b, TOT); });
  time("colpass plain", [&](uint64_t* b) { colpass<0><<<L * 16, 256>>>(b); });
  time("colpass sc1", [&](uint64_t* b) { colpass<2><<<L * 16, 256>>>(b); });
  time("rowpass plain", [&](uint64_t* b) { rowpass<0><<<L * 16, 256>>>(b); });
  time("rowpass nt", [&](uint64_t* b) { rowpass<1><<<L * 16, 256>>>(b); });
  time("two-pass plain", [&](uint64_t* b) { colpass<0><<<L * 16, 256>>>(b); rowpass<0><<<L * 16, 256>>>(b); });
  time("two-pass col sc1", [&](uint64_t* b) { colpass<2><<<L * 16, 256>>>(b); rowpass<0><<<L * 16, 256>>>(b); });
  time("two-pass both sc1", [&](uint64_t* b) { colpass<2><<<L * 16, 256>>>(b); rowpass<2><<<L * 16, 256>>>(b); });
  const int GX = 8 * 16 * ((L + 7) / 8);
  time("xcd two-pass plain/plain", [&](uint64_t* b) { colpass_x<0><<<GX, 256>>>(b); rowpass_x<0><<<GX, 256>>>(b); });
  time("xcd two-pass plain/sc1", [&](uint64_t* b) { colpass_x<0><<<GX, 256>>>(b); rowpass_x<2><<<GX, 256>>>(b); });
  time("xcd two-pass sc1/sc1", [&](uint64_t* b) { colpass_x<2><<<GX, 256>>>(b); rowpass_x<2><<<GX, 256>>>(b); });
  time("xcd two-pass nt/sc1", [&](uint64_t* b) { colpass_x<1><<<GX, 256>>>(b); rowpass_x<2><<<GX, 256>>>(b); });
  time("xcd rowpass sc1 alone", [&](uint64_t* b) { rowpass_x<2><<<GX, 256>>>(b); });
  time("xcd colpass plain alone", [&](uint64_t* b) { colpass_x<0><<<GX, 256>>>(b); });
  if (getenv("FUSED") == nullptr) return 0;
  auto fz = [&](auto kern, int G) {
    return [&, kern, G](uint64_t* b) { kern<<<8 * G * ((L + 7) / 8), 256>>>(b, counters, epoch++, tmo); };
  };
  time("fused G=4 fence", fz(fused<4, 0>, 4));
  time("fused G=4 sc1", fz(fused<4, 1>, 4));
  time("fused G=8 fence", fz(fused<8, 0>, 8));
  time("fused G=8 sc1", fz(fused<8, 1>, 8));
  time("fused G=16 fence", fz(fused<16, 0>, 16));
  time("fused G=16 sc1", fz(fused<16, 1>, 16));
  CK(hipDeviceSynchronize());
  unsigned h;
  CK(hipMemcpy(&h, tmo, sizeof h, hipMemcpyDeviceToHost));
  printf("spin timeouts: %u\n", h);
  return 0;
}
