// Micro-test of the fused-NTT hand-off protocol (csrc/ntt.hip ntt_fused_fwd): workgroups take
// tickets; tickets < NCOL bump counter[t / 16] after a delay, later tickets poll counter[limb]
// (sc1 loads) until 16, bounded.  Reports lost updates / timeouts and the poll counts.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_counter tools/ubench_counter.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int NCOL = 704, NROW = 704, CT = 16;

// Every branch is wave-uniform (scalar): wave 0 does the counter work with all 64 lanes active
// (each lane adds 1, so counters move by 64 per workgroup); a lane-divergent `if (tid == 0)`
// around the atomics inside this barrier loop was structurized into an inner loop that never
// exits (ROCm 7.2 hipcc).
template <int SCOPE>
__global__ __launch_bounds__(256) void k_handoff(int* sync, int* out, int delay, int poll) {
  __shared__ int s_t;
  __shared__ uint64_t pad[4608];  // the fused kernel's LDS footprint
  int* done = sync + 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (;;) {
    if (wave == 0) {
      const int base = __builtin_amdgcn_readfirstlane(__hip_atomic_fetch_add(sync, 1, __ATOMIC_RELAXED, SCOPE));
      if (threadIdx.x == 0) s_t = base >> 6;
    }
    __syncthreads();
    const int k = __builtin_amdgcn_readfirstlane(s_t);
    __syncthreads();
    if (k >= NCOL + NROW) break;
    if (k < NCOL) {
      for (int i = 0; i < delay; ++i) __builtin_amdgcn_s_sleep(8);
      pad[threadIdx.x] = k;
      __syncthreads();
      if (wave == 0) __hip_atomic_fetch_add(done + k / CT, 1, __ATOMIC_RELAXED, SCOPE);
    } else {
      const int limb = (k - NCOL) / CT;
      if (wave == 0 && poll) {
        int spins = 0, v = 0;
        for (;;) {
          v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(done + limb, __ATOMIC_RELAXED, SCOPE));
          if (v >= CT * 64 || spins >= 2000) break;
          __builtin_amdgcn_s_sleep(1);
          ++spins;
        }
        if (threadIdx.x == 0) {
          out[2 * (k - NCOL)] = v / 64;
          out[2 * (k - NCOL) + 1] = spins;
        }
      }
      __syncthreads();
    }
  }
  if (wave == 0) {
    const int e = __builtin_amdgcn_readfirstlane(__hip_atomic_fetch_add(sync + 1, 1, __ATOMIC_RELAXED, SCOPE));
    if (e == ((int)gridDim.x - 1) * 64) {
      for (int l = threadIdx.x; l < NCOL / CT; l += 64) __hip_atomic_store(done + l, 0, __ATOMIC_RELAXED, SCOPE);
      if (threadIdx.x == 0) {
        __hip_atomic_store(sync + 1, 0, __ATOMIC_RELAXED, SCOPE);
        __hip_atomic_store(sync, 0, __ATOMIC_RELAXED, SCOPE);
      }
    }
  }
}

template <int SCOPE>
void run(const char* name, int grid, int delay, int reps, int poll = 1) {
  int *sync, *out;
  hipMalloc(&sync, 4096 * sizeof(int));
  hipMemset(sync, 0, 4096 * sizeof(int));
  hipMalloc(&out, 2 * NROW * sizeof(int));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::printf("%s: start\n", name);
  std::fflush(stdout);
  for (int r = 0; r < reps; ++r) {
    hipMemset(out, 0xff, 2 * NROW * sizeof(int));
    hipEventRecord(a, 0);
    hipLaunchKernelGGL(k_handoff<SCOPE>, dim3(grid), dim3(256), 0, 0, sync, out, delay, poll);
    hipEventRecord(b, 0);
    std::printf("%s: launched\n", name);
    std::fflush(stdout);
    hipDeviceSynchronize();
    std::printf("%s: synced\n", name);
    std::fflush(stdout);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    std::vector<int> h(2 * NROW), s(8);
    hipMemcpy(h.data(), out, h.size() * sizeof(int), hipMemcpyDeviceToHost);
    hipMemcpy(s.data(), sync, 8 * sizeof(int), hipMemcpyDeviceToHost);
    int bad = 0, tmo = 0, maxsp = 0;
    long sum = 0;
    for (int i = 0; i < NROW; ++i) {
      bad += h[2 * i] != CT;
      tmo += h[2 * i + 1] >= 2000;
      maxsp = std::max(maxsp, h[2 * i + 1]);
      sum += h[2 * i + 1];
    }
    std::printf("%s grid %d delay %d rep %d: %.3f ms, wrong %d, timeouts %d, max polls %d, mean polls %.1f, "
                "sync after [%d %d]\n",
                name, grid, delay, r, ms, bad, tmo, maxsp, (double)sum / NROW, s[0], s[1]);
    std::fflush(stdout);
  }
  hipFree(sync);
  hipFree(out);
}

// every workgroup adds 1 once and records the returned ticket: a coherent counter hands out
// 0 .. grid-1 exactly once each
template <int SCOPE>
__global__ void k_ticket(int* ctr, int* got) {
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, SCOPE);
    got[blockIdx.x] = t;
  }
}
template <int SCOPE>
void ticket_test(const char* name, int grid) {
  int *ctr, *got;
  hipMalloc(&ctr, 64);
  hipMemset(ctr, 0, 64);
  hipMalloc(&got, grid * sizeof(int));
  hipLaunchKernelGGL(k_ticket<SCOPE>, dim3(grid), dim3(64), 0, 0, ctr, got);
  hipDeviceSynchronize();
  std::vector<int> h(grid), seen(grid, 0);
  int c = 0;
  hipMemcpy(h.data(), got, grid * sizeof(int), hipMemcpyDeviceToHost);
  hipMemcpy(&c, ctr, sizeof(int), hipMemcpyDeviceToHost);
  int dup = 0, oob = 0;
  for (int v : h) {
    if (v < 0 || v >= grid) ++oob;
    else if (seen[v]++) ++dup;
  }
  std::printf("ticket %s grid %d: final %d, duplicates %d, out of range %d\n", name, grid, c, dup, oob);
  std::fflush(stdout);
  hipFree(ctr);
  hipFree(got);
}

int main(int argc, char** argv) {
  const int c = argc > 1 ? std::atoi(argv[1]) : 0;
  if (c == 0) ticket_test<__HIP_MEMORY_SCOPE_AGENT>("agent", 1408);
  if (c == 1) run<__HIP_MEMORY_SCOPE_AGENT>("agent-nopoll", 704, 4, 2, 0);
  if (c == 2) run<__HIP_MEMORY_SCOPE_AGENT>("agent", 64, 4, 2);
  if (c == 3) run<__HIP_MEMORY_SCOPE_AGENT>("agent", 704, 4, 2);
  if (c == 4) run<__HIP_MEMORY_SCOPE_SYSTEM>("system", 704, 4, 2);
  if (c == 5) run<__HIP_MEMORY_SCOPE_AGENT>("agent-1wg-nopoll", 1, 0, 1, 0);
  if (c == 6) run<__HIP_MEMORY_SCOPE_AGENT>("agent-8wg-nopoll", 8, 0, 1, 0);
  return 0;
}
