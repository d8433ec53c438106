// Micro-benchmark (tools only): issue rate of the multiply instructions the integer paths use
// (v_mad_u64_u32, v_mul_lo_u32, v_mul_hi_u32) against v_fma_f64, on every CU.  Each lane runs 8
// independent chains of K operations; the result is folded into one store so nothing is dead.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int K = 4096, CH = 8;

__global__ __launch_bounds__(256) void k_mad64(uint64_t* out, uint32_t s) {
  uint64_t acc[CH];
  const uint32_t b = blockIdx.x * 7 + s + 0x9e3779b9u;
  for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x * 0x85ebca6bull + c;
  for (int i = 0; i < K; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = static_cast<uint64_t>(static_cast<uint32_t>(acc[c])) * b + (acc[c] >> 32);
  }
  uint64_t r = 0;
  for (int c = 0; c < CH; ++c) r ^= acc[c];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_mullo(uint64_t* out, uint32_t s) {
  uint32_t acc[CH];
  const uint32_t b = blockIdx.x * 7 + s;
  for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x + c;
  for (int i = 0; i < K; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = acc[c] * (acc[c] | b);
  }
  uint64_t r = 0;
  for (int c = 0; c < CH; ++c) r ^= acc[c];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_mulhi(uint64_t* out, uint32_t s) {
  uint32_t acc[CH];
  const uint32_t b = blockIdx.x * 7 + s + 0x9e3779b9u;
  for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x * 0x85ebca6bu + c;
  for (int i = 0; i < K; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __umulhi(acc[c], b) | 1u;
  }
  uint64_t r = 0;
  for (int c = 0; c < CH; ++c) r ^= acc[c];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_fma64(uint64_t* out, uint32_t s) {
  double acc[CH];
  const double b = 1.0000001 + s * 1e-9, c0 = 1e-7;
  for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x + c;
  for (int i = 0; i < K; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_fma(acc[c], b, c0);
  }
  double r = 0;
  for (int c = 0; c < CH; ++c) r += acc[c];
  out[blockIdx.x * 256 + threadIdx.x] = __double_as_longlong(r);
}

__global__ __launch_bounds__(256) void k_add32(uint64_t* out, uint32_t s) {
  uint32_t acc[CH];
  const uint32_t b = blockIdx.x * 7 + s;
  for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x + c;
  for (int i = 0; i < K; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = (acc[c] + b) ^ (c + 1);
  }
  uint64_t r = 0;
  for (int c = 0; c < CH; ++c) r ^= acc[c];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
  const int blocks = 256 * 8;  // 8 workgroups (32 waves) per CU
  uint64_t* out;
  CK(hipMalloc(&out, (size_t)blocks * 256 * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, void (*k)(uint64_t*, uint32_t), double ops_per_iter) {
    k<<<blocks, 256>>>(out, 1);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) k<<<blocks, 256>>>(out, r);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double lane_ops = 5.0 * blocks * 256.0 * K * CH * ops_per_iter;
    // per CU per cycle at 2.4 GHz, in lane-operations (64 = one wave instruction per cycle)
    printf("%-8s %8.3f ms  %8.2f T lane-ops/s  %6.1f lane-ops/CU/cycle\n", name, ms / 5, lane_ops / (ms * 1e-3) / 1e12,
           lane_ops / (ms * 1e-3) / 256 / 2.4e9);
    return 0;
  };
  run("add32x2", k_add32, 2.0);
  run("mad64", k_mad64, 1.0);
  run("mullo+or", k_mullo, 2.0);
  run("mulhi+or", k_mulhi, 2.0);
  run("fma64", k_fma64, 1.0);
  return 0;
}
