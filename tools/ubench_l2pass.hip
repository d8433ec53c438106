// Micro-benchmark (tools only): data movement of a single-launch two-phase NTT whose column-phase
// output stays in the XCD's L2.  [44][65536] u64 limbs, in place, "+1" stands in for each phase's
// butterflies, ring of 15 buffers (> 256 MiB Infinity Cache) as in bench.py.
//
// l2pass: 352 workgroups = 8 per limb.  A workgroup reads its XCD (HW_REG_XCC_ID) and takes ONE
// ticket from that XCD's counter: the XCD's limbs are x, x + 8, ...; ticket t -> limb t / 8, part
// t % 8.  Phase 1: two column tiles (32 columns x 256 rows, 64 KB) HBM -> +1 -> plain stores
// (the lines stay dirty in this XCD's L2).  Then every storing wave waits vmcnt(0), a workgroup
// barrier, one relaxed agent-scope add to the limb's counter.  Phase 2: poll until the limb's 8
// parts have arrived, then 32 whole rows (64 KB) with sc1 loads (L1 bypassed, this XCD's L2)
// -> +1 -> sc1 stores.  Producer and consumer are on one XCD by construction (the ticket pools
// are per XCD id), so the L2 holds the hand-off; a workgroup whose XCD pool is exhausted counts
// itself in `extra` and exits (the check reports it).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int N = 1 << 16, L = 44, S2 = 256, PARTS = 8;
constexpr size_t TOT = (size_t)N * L;

__device__ __forceinline__ uint64_t ld_sc1(const uint64_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_sc1(uint64_t* p, uint64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 7;
}

// ctr[32 * x]: XCD x ticket head; ctr[32 * (8 + l)]: limb l arrivals; ctr[32 * 60]: finished
// workgroups; ctr[32 * 61]: extra workgroups (XCD pool exhausted); ctr[32 * 62]: spin time-outs
template <int ST2>
__global__ __launch_bounds__(256) void l2pass(uint64_t* d, unsigned* ctr) {
  __shared__ int s_task;
  const unsigned x = xcc_id();
  if (threadIdx.x == 0) s_task = (int)__hip_atomic_fetch_add(ctr + 32 * x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int t = __builtin_amdgcn_readfirstlane(s_task);
  // XCD x: whole limbs x, x + 8, .., x + 32 (tickets 0..39) and half of limb 40 + x / 2 (tickets
  // 40..43: parts 4 (x % 2) ..): 44 tasks per XCD = 352 / 8 under round-robin placement.  A split
  // limb's hand-off crosses XCDs, so its phase 1 stores write through (sc1).
  if (t < 44) {
    const bool split = t >= 40;
    const int limb = split ? 40 + (int)x / 2 : (int)x + 8 * (t / PARTS);
    const int part = split ? (int)(x % 2) * 4 + (t - 40) : t % PARTS;
    uint64_t* base = d + (size_t)limb * N;
    // phase 1: columns [32 part, 32 part + 32) x 256 rows; thread: column c, rows r0 + 8 j
    {
      const int c = threadIdx.x % 32, r0 = threadIdx.x / 32;
      uint64_t v[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) v[j] = __builtin_nontemporal_load(base + (size_t)(r0 + 8 * j) * S2 + part * 32 + c);
      if (split) {
#pragma unroll
        for (int j = 0; j < 32; ++j) st_sc1(base + (size_t)(r0 + 8 * j) * S2 + part * 32 + c, v[j] + 1);
      } else {
#pragma unroll
        for (int j = 0; j < 32; ++j) base[(size_t)(r0 + 8 * j) * S2 + part * 32 + c] = v[j] + 1;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(ctr + 32 * (8 + limb), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (unsigned spins = 0;; ++spins) {
        if (__hip_atomic_load(ctr + 32 * (8 + limb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= PARTS) break;
        if (spins > (1u << 16)) { atomicAdd(ctr + 32 * 62, 1u); break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    // phase 2: rows [32 part, 32 part + 32); wave w: 8 rows, lane: 4 consecutive u64 per row chunk
    {
      const int w = threadIdx.x / 64, lane = threadIdx.x % 64;
      uint64_t v[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const int row = part * 32 + w * 8 + j / 4, col = (j % 4) * 64 + lane;
        v[j] = ld_sc1(base + (size_t)row * S2 + col);
      }
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const int row = part * 32 + w * 8 + j / 4, col = (j % 4) * 64 + lane;
        if (ST2) st_sc1(base + (size_t)row * S2 + col, v[j] + 1);
        else base[(size_t)row * S2 + col] = v[j] + 1;
      }
    }
  } else if (threadIdx.x == 0) {
    atomicAdd(ctr + 32 * 61, 1u);
  }
  if (threadIdx.x == 0) {
    const unsigned f = __hip_atomic_fetch_add(ctr + 32 * 60, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (f == gridDim.x - 1) {  // last workgroup out resets the counters for the next launch
      for (int i = 0; i < 60; ++i) __hip_atomic_store(ctr + 32 * i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 32 * 60, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// two-pass reference with the same tiles: column phase, then row phase (sc1 stores both)
__global__ __launch_bounds__(256) void colphase(uint64_t* d) {
  const int limb = blockIdx.x / PARTS, part = blockIdx.x % PARTS;
  uint64_t* base = d + (size_t)limb * N;
  const int c = threadIdx.x % 32, r0 = threadIdx.x / 32;
  uint64_t v[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) v[j] = __builtin_nontemporal_load(base + (size_t)(r0 + 8 * j) * S2 + part * 32 + c);
#pragma unroll
  for (int j = 0; j < 32; ++j) st_sc1(base + (size_t)(r0 + 8 * j) * S2 + part * 32 + c, v[j] + 1);
}
__global__ __launch_bounds__(256) void rowphase(uint64_t* d) {
  const int limb = blockIdx.x / PARTS, part = blockIdx.x % PARTS;
  uint64_t* base = d + (size_t)limb * N;
  const int w = threadIdx.x / 64, lane = threadIdx.x % 64;
  uint64_t v[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) v[j] = __builtin_nontemporal_load(base + (size_t)(part * 32 + w * 8 + j / 4) * S2 + (j % 4) * 64 + lane);
#pragma unroll
  for (int j = 0; j < 32; ++j) st_sc1(base + (size_t)(part * 32 + w * 8 + j / 4) * S2 + (j % 4) * 64 + lane, v[j] + 1);
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int ring = 15, reps = 60;
  std::vector<uint64_t*> buf(ring);
  for (auto& b : buf) { CK(hipMalloc(&b, TOT * 8)); CK(hipMemset(b, 0, TOT * 8)); }
  unsigned* ctr;
  CK(hipMalloc(&ctr, 64 * 32 * sizeof(unsigned)));
  CK(hipMemset(ctr, 0, 64 * 32 * sizeof(unsigned)));
  const int grid = L * PARTS;
  // correctness: one launch on zeros -> every element 2
  l2pass<1><<<grid, 256>>>(buf[0], ctr);
  CK(hipDeviceSynchronize());
  std::vector<uint64_t> h(TOT);
  CK(hipMemcpy(h.data(), buf[0], TOT * 8, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (auto v : h) bad += v != 2;
  unsigned c[64 * 32];
  CK(hipMemcpy(c, ctr, sizeof(c), hipMemcpyDeviceToHost));
  printf("l2pass check: %zu wrong elements, extra workgroups %u, spin time-outs %u\n", bad, c[32 * 61], c[32 * 62]);
  CK(hipMemset(ctr, 0, 64 * 32 * sizeof(unsigned)));
  CK(hipMemset(buf[0], 0, TOT * 8));
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
    printf("%-30s stream-avg %7.2f us  %7.1f GB/s (16 B/coef)\n", name, us, TOT * 16.0 / us / 1e3);
    return 0;
  };
  time("two-pass (same tiles, sc1)", [&](uint64_t* b) { colphase<<<grid, 256>>>(b); rowphase<<<grid, 256>>>(b); });
  time("l2pass sc1 final stores", [&](uint64_t* b) { l2pass<1><<<grid, 256>>>(b, ctr); });
  time("l2pass plain final stores", [&](uint64_t* b) { l2pass<0><<<grid, 256>>>(b, ctr); });
  CK(hipMemcpy(c, ctr, sizeof(c), hipMemcpyDeviceToHost));
  printf("after timing: extra workgroups %u, spin time-outs %u\n", c[32 * 61], c[32 * 62]);
  return 0;
}
