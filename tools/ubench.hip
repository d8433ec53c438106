// Micro-benchmarks for gfx950: HBM copy bandwidth and 32/64-bit integer multiply
// throughput, used to size the NTT kernel design (see DESIGN.md "Arithmetic cost").
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void copy_kernel(const ulonglong2* __restrict__ in, ulonglong2* __restrict__ out, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) out[i] = in[i];
}

constexpr int CH = 8;  // independent chains per lane

__global__ void mul_lo_kernel(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a[CH];
  for (int c = 0; c < CH; ++c) a[c] = seed + threadIdx.x + c;
  uint32_t b = seed | 1;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = a[c] * b + 1u;  // v_mad_u32_u24? no: mul_lo + add
  uint32_t s = 0;
  for (int c = 0; c < CH; ++c) s ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void mul_hi_kernel(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a[CH];
  for (int c = 0; c < CH; ++c) a[c] = seed + threadIdx.x + c;
  uint32_t b = seed | 0x80000001u;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = __umulhi(a[c], b) ^ b;
  uint32_t s = 0;
  for (int c = 0; c < CH; ++c) s ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void mad64_kernel(uint64_t* out, int iters, uint32_t seed) {
  uint64_t a[CH];
  for (int c = 0; c < CH; ++c) a[c] = seed + threadIdx.x + c;
  uint32_t b = seed | 1;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = (uint64_t)(uint32_t)a[c] * b + (a[c] >> 32);
  uint64_t s = 0;
  for (int c = 0; c < CH; ++c) s ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void fma64_kernel(double* out, int iters, double seed) {
  double a[CH];
  for (int c = 0; c < CH; ++c) a[c] = seed + threadIdx.x + c;
  double b = 0.999999, d = 1e-7;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = fma(a[c], b, d);
  double s = 0;
  for (int c = 0; c < CH; ++c) s += a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__device__ __forceinline__ void ct_bfly(uint64_t& x, uint64_t& y, uint64_t w, uint64_t ws, uint64_t q) {
  uint64_t hi = __umul64hi(y, ws);
  uint64_t t = y * w - hi * q;
  uint64_t q2 = 2 * q;
  uint64_t tmp = x - q2;
  x = tmp + (tmp >> 63) * q2;
  y = x + q2 - t;
  x += t;
}

__global__ void bfly_kernel(uint64_t* out, int iters, uint64_t q, uint64_t w, uint64_t ws) {
  uint64_t v[8];
  for (int c = 0; c < 8; ++c) v[c] = (threadIdx.x * 977 + c * 131) % q;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 4; ++c) ct_bfly(v[c], v[c + 4], w, ws, q);
#pragma unroll
    for (int c = 0; c < 4; ++c) ct_bfly(v[2 * c], v[2 * c + 1], w, ws, q);
  }
  uint64_t s = 0;
  for (int c = 0; c < 8; ++c) s ^= v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float ms;
  // copy bandwidth
  for (size_t bytes : {size_t(256) << 20, size_t(1) << 30, size_t(2) << 30}) {
    size_t n = bytes / 16;
    ulonglong2 *a, *b; CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 1, bytes)); CK(hipMemset(b, 0, bytes));
    for (int grid : {2048, 8192}) {
      copy_kernel<<<grid, 256>>>(a, b, n);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int r = 0; r < 20; ++r) copy_kernel<<<grid, 256>>>(a, b, n);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("copy %zu MiB grid %d: %.3f ms/iter, %.1f GB/s (read+write)\n", bytes >> 20, grid, ms / 20,
             2.0 * bytes / (ms / 20 * 1e-3) / 1e9);
    }
    CK(hipFree(a)); CK(hipFree(b));
  }
  const int grid = 256 * 8, block = 256, iters = 4096;
  const double lanes = double(grid) * block;
  void* out; CK(hipMalloc(&out, grid * block * 8));
  auto report = [&](const char* name, double ops_per_iter_lane) {
    double t = ms * 1e-3;
    double ops = lanes * iters * ops_per_iter_lane;
    printf("%-10s %.3f ms  %.2f Tops/s  (%.2f lane-ops/clk/SIMD @2.4GHz)\n", name, ms, ops / t / 1e12,
           ops / t / (1024 * 2.4e9));
  };
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipEventRecord(e0)); mul_lo_kernel<<<grid, block>>>((uint32_t*)out, iters, 7); CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1)); if (rep) report("mul_lo+add", CH);
    CK(hipEventRecord(e0)); mul_hi_kernel<<<grid, block>>>((uint32_t*)out, iters, 7); CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1)); if (rep) report("mul_hi+xor", CH);
    CK(hipEventRecord(e0)); mad64_kernel<<<grid, block>>>((uint64_t*)out, iters, 7); CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1)); if (rep) report("mad_u64", CH);
    CK(hipEventRecord(e0)); fma64_kernel<<<grid, block>>>((double*)out, iters, 7.0); CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1)); if (rep) report("fma_f64", CH);
    CK(hipEventRecord(e0));
    bfly_kernel<<<grid, block>>>((uint64_t*)out, iters, 1125899904679937ull, 123456789012345ull, 2023ull);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1)); if (rep) report("ct_bfly", 8);
  }
  return 0;
}
