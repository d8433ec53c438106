// ubench_mfma: cycles per MFMA on gfx950 for the int8 forms the base conversion uses, against the
// bf16 form the guide quotes.  Each wave runs ITERS x 8 independent MFMAs (8 accumulators);
// time = the kernel's duration (hipEvent), reported as cycles per MFMA per SIMD at 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
constexpr int ITERS = 4096;

__global__ void k16(const v4i* in, v4i* out) {
  v4i a = in[threadIdx.x], b = in[threadIdx.x + 64];
  v4i acc[8] = {};
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[j], 0, 0, 0);
  v4i s = {};
  for (int j = 0; j < 8; ++j) s += acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k32(const v4i* in, v16i* out) {
  v4i a = in[threadIdx.x], b = in[threadIdx.x + 64];
  v16i acc[4] = {};
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[j], 0, 0, 0);
  v16i s = {};
  for (int j = 0; j < 4; ++j) s += acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void kbf(const v8bf* in, v4f* out) {
  v8bf a = in[threadIdx.x], b = in[threadIdx.x + 64];
  v4f acc[8] = {};
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
  v4f s = {};
  for (int j = 0; j < 8; ++j) s += acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename I, typename O>
void run(const char* name, void (*kern)(const I*, O*), const I* in, O* out, int waves_per_simd, int mfma_per_iter) {
  const int blocks = 256 * waves_per_simd, threads = 256;  // 4 waves per block, one block per CU per wave-per-SIMD
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, in, out);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, in, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double per_simd = (double)ITERS * mfma_per_iter * waves_per_simd;
  printf("%-26s waves/SIMD %d  %8.3f ms  %6.1f cycles per MFMA per SIMD\n", name, waves_per_simd, ms,
         ms * 1e-3 * 2.4e9 / per_simd);
}

int main() {
  void* in;
  void* out;
  hipMalloc(&in, 1 << 20);
  hipMemset(in, 1, 1 << 20);
  hipMalloc(&out, 64 << 20);
  for (int w = 1; w <= 4; w *= 2) {
    run("i32_16x16x64_i8", k16, (const v4i*)in, (v4i*)out, w, 8);
    run("i32_32x32x32_i8", k32, (const v4i*)in, (v16i*)out, w, 4);
    run("f32_16x16x32_bf16", kbf, (const v8bf*)in, (v4f*)out, w, 8);
  }
  return 0;
}
