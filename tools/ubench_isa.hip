// Per-instruction throughput on gfx950 (cycles per wave64 instruction per SIMD),
// measured with 8 independent register chains per lane, full occupancy.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(e)); return 1; } } while (0)

#define R8(X) X X X X X X X X
#define KERNEL(name, body, init)                                                   \
  __global__ void name(uint32_t* out, int iters) {                                 \
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = 12345, c = 777;            \
    uint64_t d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7; \
    double f0 = a0, f1 = a1, f2 = a2, f3 = a3, f4 = a4, f5 = a5, f6 = a6, f7 = a7, fb = 1.0000001; \
    init;                                                                          \
    for (int i = 0; i < iters; ++i) { R8(body) }                                   \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(d0 ^ d1 ^ d2 ^ d3 ^ d4 ^ d5 ^ d6 ^ d7) ^ (uint32_t)(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7); \
  }

#define OP32(ins) asm volatile(ins " %0, %0, %8\n" ins " %1, %1, %8\n" ins " %2, %2, %8\n" ins " %3, %3, %8\n" \
                                ins " %4, %4, %8\n" ins " %5, %5, %8\n" ins " %6, %6, %8\n" ins " %7, %7, %8\n" \
                                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
#define OPMAD(ins) asm volatile(ins " %0, s[0:1], %8, %9, %0\n" ins " %1, s[0:1], %8, %9, %1\n" ins " %2, s[0:1], %8, %9, %2\n" ins " %3, s[0:1], %8, %9, %3\n" \
                                ins " %4, s[0:1], %8, %9, %4\n" ins " %5, s[0:1], %8, %9, %5\n" ins " %6, s[0:1], %8, %9, %6\n" ins " %7, s[0:1], %8, %9, %7\n" \
                                : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7) : "v"(b), "v"(c) : "s0", "s1");
#define OPF64_3(ins) asm volatile(ins " %0, %0, %8, %8\n" ins " %1, %1, %8, %8\n" ins " %2, %2, %8, %8\n" ins " %3, %3, %8, %8\n" \
                                ins " %4, %4, %8, %8\n" ins " %5, %5, %8, %8\n" ins " %6, %6, %8, %8\n" ins " %7, %7, %8, %8\n" \
                                : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7) : "v"(fb));
#define OPF64_2(ins) asm volatile(ins " %0, %0, %8\n" ins " %1, %1, %8\n" ins " %2, %2, %8\n" ins " %3, %3, %8\n" \
                                ins " %4, %4, %8\n" ins " %5, %5, %8\n" ins " %6, %6, %8\n" ins " %7, %7, %8\n" \
                                : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7) : "v"(fb));
#define OPF64_1(ins) asm volatile(ins " %0, %0\n" ins " %1, %1\n" ins " %2, %2\n" ins " %3, %3\n" \
                                ins " %4, %4\n" ins " %5, %5\n" ins " %6, %6\n" ins " %7, %7\n" \
                                : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7));
#define OP64_2(ins) asm volatile(ins " %0, %0, 0, %8\n" ins " %1, %1, 0, %8\n" ins " %2, %2, 0, %8\n" ins " %3, %3, 0, %8\n" \
                                ins " %4, %4, 0, %8\n" ins " %5, %5, 0, %8\n" ins " %6, %6, 0, %8\n" ins " %7, %7, 0, %8\n" \
                                : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7) : "v"(d0));

KERNEL(k_mul_lo, OP32("v_mul_lo_u32"), )
KERNEL(k_mul_hi, OP32("v_mul_hi_u32"), )
KERNEL(k_mul_u24, OP32("v_mul_u32_u24"), )
KERNEL(k_mul_hi_u24, OP32("v_mul_hi_u32_u24"), )
KERNEL(k_add, OP32("v_add_u32"), )
KERNEL(k_xor, OP32("v_xor_b32"), )
KERNEL(k_mad64, OPMAD("v_mad_u64_u32"), )
KERNEL(k_lshl_add64, OP64_2("v_lshl_add_u64"), )
KERNEL(k_fma64, OPF64_3("v_fma_f64"), )
KERNEL(k_mul64, OPF64_2("v_mul_f64"), )
KERNEL(k_add64, OPF64_2("v_add_f64"), )
KERNEL(k_rnd64, OPF64_1("v_rndne_f64"), )
KERNEL(k_floor64, OPF64_1("v_floor_f64"), )

int main() {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int grid = 256 * 8, block = 256, iters = 2048;
  uint32_t* out; CK(hipMalloc(&out, grid * block * 4));
  struct { const char* n; void (*k)(uint32_t*, int); } ks[] = {
    {"v_mul_lo_u32", k_mul_lo}, {"v_mul_hi_u32", k_mul_hi}, {"v_mul_u32_u24", k_mul_u24},
    {"v_mul_hi_u32_u24", k_mul_hi_u24}, {"v_add_u32", k_add}, {"v_xor_b32", k_xor},
    {"v_mad_u64_u32", k_mad64}, {"v_lshl_add_u64", k_lshl_add64}, {"v_fma_f64", k_fma64},
    {"v_mul_f64", k_mul64}, {"v_add_f64", k_add64}, {"v_rndne_f64", k_rnd64}, {"v_floor_f64", k_floor64}};
  for (int rep = 0; rep < 2; ++rep)
    for (auto& k : ks) {
      float ms;
      CK(hipEventRecord(e0)); k.k<<<grid, block>>>(out, iters); CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
      double winstr = double(grid) * block / 64 * iters * 64;  // wave-instructions
      double cyc = ms * 1e-3 * 2.4e9 * 1024 / winstr;          // cycles per wave-instr per SIMD
      if (rep) printf("%-18s %.3f ms  %.2f cycles/wave-instr/SIMD\n", k.n, ms, cyc);
    }
  return 0;
}
