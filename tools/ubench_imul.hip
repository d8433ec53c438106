// Issue cost of the integer instructions the 60-bit NTT butterflies are made of, on gfx950.
// Every wave runs `iters` x 16 independent instances of one instruction (8 accumulator chains,
// unrolled twice) between two s_memtime reads; cycles per instruction per wave and per SIMD
// (W waves resident per SIMD) are printed as one JSON line per (op, W).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_imul tools/ubench_imul.hip && /tmp/ubench_imul
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                              \
    }                                                                        \
  } while (0)

enum Op { MUL_LO, MUL_HI, MAD_U64, ADD_U32, LSHL_ADD_U64, ADD_CO_PAIR, BFI, FMA_F64, MUL_F64, NOPS };
static const char* kNames[NOPS] = {"v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_add_u32",
                                   "v_lshl_add_u64", "v_add_co_u32+v_addc_co_u32", "v_bfi_b32",
                                   "v_fma_f64", "v_mul_f64"};

template <int OP>
__device__ __forceinline__ void step(uint64_t& a, uint32_t b) {
  uint32_t lo = static_cast<uint32_t>(a), hi = static_cast<uint32_t>(a >> 32);
  if constexpr (OP == MUL_LO) {
    asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(lo) : "v"(b));
  } else if constexpr (OP == MUL_HI) {
    asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(lo) : "v"(b));
  } else if constexpr (OP == MAD_U64) {
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a) : "v"(lo), "v"(b) : "vcc");
    return;
  } else if constexpr (OP == ADD_U32) {
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(lo) : "v"(b));
  } else if constexpr (OP == LSHL_ADD_U64) {
    asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a) : "v"(static_cast<uint64_t>(b)));
    return;
  } else if constexpr (OP == ADD_CO_PAIR) {
    asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc"
                 : "+v"(lo), "+v"(hi) : "v"(b) : "vcc");
  } else if constexpr (OP == BFI) {
    asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(lo) : "v"(b), "v"(hi));
  } else if constexpr (OP == FMA_F64) {
    double d = __builtin_bit_cast(double, a);
    asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d) : "v"(static_cast<double>(b)));
    a = __builtin_bit_cast(uint64_t, d);
    return;
  } else if constexpr (OP == MUL_F64) {
    double d = __builtin_bit_cast(double, a);
    asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d) : "v"(static_cast<double>(b)));
    a = __builtin_bit_cast(uint64_t, d);
    return;
  }
  a = (static_cast<uint64_t>(hi) << 32) | lo;
}

// CH independent chains, 16 / CH dependent steps each per iteration (16 instructions)
template <int OP, int CH>
__global__ void __launch_bounds__(256) bench(uint64_t* sink, uint64_t* cycles, int iters, uint32_t seed) {
  uint64_t a[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) a[c] = (static_cast<uint64_t>(seed) << 32) + threadIdx.x * 8 + c + 1;
  const uint32_t b = seed | 1u;
  const uint64_t t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16 / CH; ++u) {
#pragma unroll
      for (int c = 0; c < CH; ++c) step<OP>(a[c], b);
    }
  }
  const uint64_t t1 = clock64();
  uint64_t x = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) x ^= a[c];
  const size_t gid = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  sink[gid] = x;
  if ((threadIdx.x & 63) == 0) cycles[gid / 64] = t1 - t0;
}

template <int OP, int CH = 8>
static int run(int waves_per_simd, int cus, int iters) {
  const int blocks = cus * waves_per_simd;  // 256 threads = one wave per SIMD per block
  const size_t threads = static_cast<size_t>(blocks) * 256;
  uint64_t *sink = nullptr, *cyc = nullptr;
  CHECK(hipMalloc(&sink, threads * 8));
  CHECK(hipMalloc(&cyc, threads / 64 * 8));
  hipLaunchKernelGGL((bench<OP, CH>), dim3(blocks), dim3(256), 0, nullptr, sink, cyc, iters, 0x9E3779B9u);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, nullptr));
  hipLaunchKernelGGL((bench<OP, CH>), dim3(blocks), dim3(256), 0, nullptr, sink, cyc, iters, 0x9E3779B9u);
  CHECK(hipEventRecord(e1, nullptr));
  CHECK(hipDeviceSynchronize());
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<uint64_t> h(threads / 64);
  CHECK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
  double mean = 0;
  for (uint64_t c : h) mean += static_cast<double>(c);
  mean /= h.size();
  const double per_wave = mean / (static_cast<double>(iters) * 16);
  std::printf("{\"op\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"cycles_per_instr_per_wave\": %.2f, "
              "\"cycles_per_instr_per_simd\": %.2f, \"kernel_ms\": %.3f}\n",
              kNames[OP], CH, waves_per_simd, per_wave, per_wave / waves_per_simd, ms);
  CHECK(hipFree(sink));
  CHECK(hipFree(cyc));
  return 0;
}

template <int OP>
static int sweep(int cus, int iters) {
  for (int w : {1, 2, 3, 4, 6, 8})
    if (run<OP>(w, cus, iters)) return 1;
  return 0;
}
// instruction-level parallelism inside one wave against waves per SIMD
template <int OP>
static int sweep_ilp(int cus, int iters) {
  for (int w : {1, 2, 4}) {
    if (run<OP, 1>(w, cus, iters) || run<OP, 2>(w, cus, iters) || run<OP, 4>(w, cus, iters)) return 1;
  }
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount, iters = 4096;
  int rc = 0;
  rc |= sweep<MUL_LO>(cus, iters);
  rc |= sweep<MUL_HI>(cus, iters);
  rc |= sweep<MAD_U64>(cus, iters);
  rc |= sweep<ADD_U32>(cus, iters);
  rc |= sweep<LSHL_ADD_U64>(cus, iters);
  rc |= sweep<ADD_CO_PAIR>(cus, iters);
  rc |= sweep<BFI>(cus, iters);
  rc |= sweep<FMA_F64>(cus, iters);
  rc |= sweep<MUL_F64>(cus, iters);
  rc |= sweep_ilp<MUL_LO>(cus, iters);
  rc |= sweep_ilp<MAD_U64>(cus, iters);
  rc |= sweep_ilp<ADD_U32>(cus, iters);
  return rc;
}
