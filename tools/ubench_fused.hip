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


// fusedq: one launch, per-XCD work queues.  A workgroup reads its XCC id, and takes tasks from
// that XCD's queue only, so every hand-off stays inside one XCD's L2: column tasks store their
// intermediate with plain stores (the line stays in the L2), row tasks load it with nt loads
// (L1 bypassed, served by the same L2) after the limb's counter shows all 16 column tiles.
// Queue of XCD x (limbs x, x+8, ...; m of them): C(0..D-1), then R(s-D), C(s) interleaved.
__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 7;
}
template <int D, int SL = 1>
__global__ __launch_bounds__(256) void fusedq(uint64_t* d, unsigned* ctr, unsigned* tmo) {
  // ctr[0..7] queue heads, ctr[8..8+L) limb counters, ctr[63] finish counter
  __shared__ int s_task;
  const unsigned x = xcc_id();
  if (threadIdx.x == 0) atomicAdd(tmo + 1 + x, 1u);  // workgroups seen per XCC id
  const int m = (L - (int)x + 7) / 8;
  const int ntask = 32 * m;
  for (int iter = 0; iter < 4096; ++iter) {
    if (threadIdx.x == 0) s_task = (int)__hip_atomic_fetch_add(ctr + 32 * x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int task = __builtin_amdgcn_readfirstlane(s_task);
    __syncthreads();
    if (task >= ntask) break;
    // decode: C(0..D-1); then R(s-D), C(s) for s in [D, m); then R(m-D..m-1)
    bool col; int li, part;
    if (task < 16 * D) { col = true; li = task / 16; part = task % 16; }
    else if (task - 16 * D < 32 * (m - D)) {
      const int u = task - 16 * D, s = u / 32 + D, r = u % 32;
      col = r >= 16; li = col ? s : s - D; part = r % 16;
    } else {
      const int v = task - 16 * D - 32 * (m - D);
      col = false; li = m - D + v / 16; part = v % 16;
    }
    const int limb = (int)x + 8 * li;
    if (col) {
      col_tile<0, false>(d, limb, part);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr + 32 * (8 + limb), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (threadIdx.x < 64) {  // wave 0 polls (wave-uniform loop)
        for (unsigned spins = 0;; ++spins) {
          const unsigned v = __builtin_amdgcn_readfirstlane(
              __hip_atomic_load(ctr + 32 * (8 + limb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
          if (v >= 16u) break;
          if (spins > (1u << 14)) { if (threadIdx.x == 0) atomicAdd(tmo, 1u); break; }
          __builtin_amdgcn_s_sleep(SL);
        }
      }
      __syncthreads();
      const int w = threadIdx.x / 64;
      const int lane = threadIdx.x % 64, lr = lane / 16, t = lane % 16;
      uint64_t* base = d + (size_t)limb * N + (size_t)((part * 4 + w) * 4 + lr) * S2 + t;
      uint64_t v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = __builtin_nontemporal_load(base + 16 * j);
#pragma unroll
      for (int j = 0; j < 16; ++j) st<2>(base + 16 * j, v[j] + 1);
    }
  }
  // last workgroup out resets the counters for the next launch
  if (threadIdx.x == 0) {
    const unsigned f = __hip_atomic_fetch_add(ctr + 32 * 60, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (f == gridDim.x - 1) {
      for (int i = 0; i < 60; ++i) __hip_atomic_store(ctr + 32 * i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 32 * 60, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// fusedx: one launch, every workgroup co-resident (grid = 8 * 16 * ceil(L / 8)), per-XCD ticket
// queues ordered column tasks first, then row tasks (a row task waits only on column tasks with
// smaller tickets, so any residency makes progress).  Column tasks store plain (the line stays
// dirty in this XCD's L2), row tasks poll the limb counter, then load the intermediate with sc1
// loads (L1 bypassed, same L2) and store the result with store flavour RS (0 plain, 2 sc1).
template <int RS>
__global__ __launch_bounds__(256) void fusedx(uint64_t* d, unsigned* ctr, unsigned* tmo) {
  __shared__ int s_task;
  const unsigned x = xcc_id();
  const int m = (L - (int)x + 7) / 8;
  const int ncol = 16 * m, ntask = 32 * m;
  for (int iter = 0; iter < 64; ++iter) {
    if (threadIdx.x == 0) s_task = (int)__hip_atomic_fetch_add(ctr + 32 * x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int task = __builtin_amdgcn_readfirstlane(s_task);
    __syncthreads();
    if (task >= ntask) break;
    if (task < ncol) {
      const int limb = (int)x + 8 * (task / 16);
      col_tile<0, false>(d, limb, task % 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr + 32 * (8 + limb), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const int u = task - ncol, limb = (int)x + 8 * (u / 16), part = u % 16;
      if (threadIdx.x < 64) {
        for (unsigned spins = 0;; ++spins) {
          const unsigned v = __builtin_amdgcn_readfirstlane(
              __hip_atomic_load(ctr + 32 * (8 + limb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
          if (v >= 16u) break;
          if (spins > (1u << 14)) { if (threadIdx.x == 0) atomicAdd(tmo, 1u); break; }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      __syncthreads();
      const int w = threadIdx.x / 64, lane = threadIdx.x % 64, lr = lane / 16, t = lane % 16;
      uint64_t* base = d + (size_t)limb * N + (size_t)((part * 4 + w) * 4 + lr) * S2 + t;
      uint64_t v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = ld_sc1(base + 16 * j);
#pragma unroll
      for (int j = 0; j < 16; ++j) st<RS>(base + 16 * j, v[j] + 1);
    }
  }
  if (threadIdx.x == 0) {
    const unsigned f = __hip_atomic_fetch_add(ctr + 32 * 60, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (f == gridDim.x - 1) {
      for (int i = 0; i < 60; ++i) __hip_atomic_store(ctr + 32 * i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 32 * 60, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
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
  CK(hipMalloc(&counters, 64 * 32 * sizeof(unsigned))); CK(hipMemset(counters, 0, 64 * 32 * sizeof(unsigned)));
  CK(hipMalloc(&tmo, sizeof(unsigned))); CK(hipMemset(tmo, 0, sizeof(unsigned)));
  unsigned epoch = 0;
  auto time = [&](const char* name, auto launch) {
    CK(hipDeviceSynchronize());
    CK(hipMemset(counters, 0, 64 * 32 * sizeof(unsigned)));
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
  if (getenv("FUSEDX")) {
    CK(hipMalloc(&tmo, 16 * sizeof(unsigned)));
    const int GX = 8 * 16 * ((L + 7) / 8);
    // correctness: one launch on zeros -> every element 2, no timeouts
    CK(hipMemset(counters, 0, 64 * 32 * sizeof(unsigned)));
    CK(hipMemset(tmo, 0, 16 * sizeof(unsigned)));
    for (int rs = 0; rs < 2; ++rs) {
      printf("fusedx check RS=%d launching\n", rs);
      CK(hipMemset(buf[0], 0, TOT * 8));
      CK(hipDeviceSynchronize());
      if (rs == 0) fusedx<0><<<GX, 256>>>(buf[0], counters, tmo);
      else fusedx<2><<<GX, 256>>>(buf[0], counters, tmo);
      CK(hipDeviceSynchronize());
      std::vector<uint64_t> h(TOT);
      CK(hipMemcpy(h.data(), buf[0], TOT * 8, hipMemcpyDeviceToHost));
      size_t bad = 0;
      for (size_t i = 0; i < TOT; ++i) bad += h[i] != 2;
      unsigned t;
      CK(hipMemcpy(&t, tmo, sizeof t, hipMemcpyDeviceToHost));
      printf("fusedx RS=%d check: %zu bad, timeouts %u\n", rs ? 2 : 0, bad, t);
      if (bad || t) return 1;
    }
    time("two-pass both sc1", [&](uint64_t* b) { colpass<2><<<L * 16, 256>>>(b); rowpass<2><<<L * 16, 256>>>(b); });
    time("fusedx plain/sc1ld/plain", [&](uint64_t* b) { fusedx<0><<<GX, 256>>>(b, counters, tmo); });
    time("fusedx plain/sc1ld/sc1", [&](uint64_t* b) { fusedx<2><<<GX, 256>>>(b, counters, tmo); });
    unsigned t;
    CK(hipMemcpy(&t, tmo, sizeof t, hipMemcpyDeviceToHost));
    printf("spin timeouts %u\n", t);
    return 0;
  }
  if (!getenv("FUSEDQ")) {
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
  }
  if (getenv("FUSEDQ")) {
    CK(hipMalloc(&tmo, 16 * sizeof(unsigned)));
    auto check = [&](int grid) -> int {
      CK(hipMemset(counters, 0, 64 * 32 * sizeof(unsigned)));
      CK(hipMemset(tmo, 0, 16 * sizeof(unsigned)));
      CK(hipMemset(buf[0], 0, TOT * 8));
      CK(hipDeviceSynchronize());
      hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
      CK(hipEventRecord(a));
      fusedq<1><<<grid, 256>>>(buf[0], counters, tmo);
      CK(hipEventRecord(z));
      CK(hipDeviceSynchronize());
      float ms; CK(hipEventElapsedTime(&ms, a, z));
      std::vector<uint64_t> h(TOT);
      CK(hipMemcpy(h.data(), buf[0], TOT * 8, hipMemcpyDeviceToHost));
      size_t bad = 0;
      for (size_t i = 0; i < TOT; ++i) bad += h[i] != 2;
      unsigned t[16], c[64];
      CK(hipMemcpy(t, tmo, sizeof t, hipMemcpyDeviceToHost));
      CK(hipMemcpy(c, counters, sizeof c, hipMemcpyDeviceToHost));
      printf("fusedq grid %d: %.3f ms, %zu bad, timeouts %u, per-xcc", grid, ms, bad, t[0]);
      for (int i = 0; i < 8; ++i) printf(" %u", t[1 + i]);
      printf(" | ctr0 %u\n", c[0]);
      return (bad || t[0]) ? 1 : 0;
    };
    if (check(256) || check(512)) return 1;
    for (int per : {1, 2}) {
      char nm[64];
#define FQ(DD, SLP) \
      snprintf(nm, sizeof nm, "fusedq D=%d sl=%d %d/CU", DD, SLP, per); \
      time(nm, [&, per](uint64_t* b) { fusedq<DD, SLP><<<256 * per, 256>>>(b, counters, tmo); });
      FQ(1, 1) FQ(2, 1) FQ(2, 8) FQ(3, 8) FQ(2, 32)
    }
    unsigned t;
    CK(hipMemcpy(&t, tmo, sizeof t, hipMemcpyDeviceToHost));
    printf("spin timeouts %u\n", t);
    return 0;
  }
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
