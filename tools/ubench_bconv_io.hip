// Data-movement skeletons of the matrix-core base conversion (csrc/rns.hip bconv_mfma_kernel), no
// arithmetic: what the C3 three-digit modup (3 jobs, 15 -> 45 limbs, N = 2^16) costs in reads and
// writes alone in the kernel's access pattern, against plain streaming of the same bytes (tools only).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_bconv_io.hip -o tools/bin_ubench_bconv_io
// Buffer rings larger than the 256 MiB Infinity Cache, as bench.py's C2 ring.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>
#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__);             \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

constexpr uint32_t N = 1u << 16, IB = 15, OB = 45, JOBS = 3, TILES = N / 16;
constexpr size_t IN_U64 = (size_t)JOBS * IB * N, OUT_U64 = (size_t)JOBS * OB * N;
constexpr int RING = 6;  // 6 x (23.6 + 70.8) MB = 566 MB
constexpr int kWaves = 8;
constexpr int kSc1 = 16;
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// the kernel's pattern: wave-owned 16-coefficient tiles, per lane (c = lane & 15, g = lane >> 4)
// loads of limbs 2g, 2g+1 (+8) at coefficient c, 4 x 8-byte stores per 16-row block (rows 4g + r)
// through a raw buffer with sc1; READ / WRITE select the halves
template <bool READ, bool WRITE>
__global__ __launch_bounds__(kWaves * 64) void skel8(const uint64_t* in, uint64_t* out, uint64_t* sink) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  const uint32_t job = blockIdx.y;
  const uint64_t* src = in + (size_t)job * IB * N;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(out + (size_t)job * OB * N, 0, (int)(OB * N * 8u), 0x00020000);
  uint64_t acc = 0;
  for (uint32_t tile = blockIdx.x * kWaves + wave; tile < TILES; tile += gridDim.x * kWaves) {
    uint64_t x[2][2];
    if (READ) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const uint32_t s = min(8 * t + 2 * g + u, IB - 1);
          x[t][u] = __builtin_nontemporal_load(src + (size_t)s * N + tile * 16 + c);
        }
      acc += x[0][0] ^ x[0][1] ^ x[1][0] ^ x[1][1];
    }
    if (WRITE) {
      const uint64_t v = acc + tile;
#pragma unroll
      for (int jb = 0; jb < 3; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t j = jb * 16 + 4 * g + r;
          const uint32_t off = j < OB ? j * N * 8u + (tile * 16 + c) * 8u : 0x80000000u;
          const v2u yv = {(uint32_t)v, (uint32_t)(v >> 32)};
          __builtin_amdgcn_raw_buffer_store_b64(yv, rs, off, 0, kSc1);
        }
    }
  }
  if (!WRITE && acc == 0x123456789ull) sink[0] = acc;
}

// 16-byte stores: 8 lanes per 128-byte row segment, 8 rows per instruction (the layout a lane
// exchange after the MFMA reassembly would give)
__global__ __launch_bounds__(kWaves * 64) void write16(uint64_t* out) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 7, g = lane >> 3;
  const uint32_t job = blockIdx.y;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(out + (size_t)job * OB * N, 0, (int)(OB * N * 8u), 0x00020000);
  for (uint32_t tile = blockIdx.x * kWaves + wave; tile < TILES; tile += gridDim.x * kWaves) {
#pragma unroll
    for (int jb = 0; jb < 6; ++jb) {
      const uint32_t j = jb * 8 + g;
      const uint32_t off = j < OB ? j * N * 8u + (tile * 16 + 2 * c) * 8u : 0x80000000u;
      const v4u yv = {tile, j, 1u, 2u};
      __builtin_amdgcn_raw_buffer_store_b128(yv, rs, off, 0, kSc1);
    }
  }
}

// plain streaming write of the same bytes, 16 B per lane, grid-stride
__global__ __launch_bounds__(256) void stream_write(uint64_t* out, size_t n2) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x)
    reinterpret_cast<ulonglong2*>(out)[i] = make_ulonglong2(i, i + 1);
}

int main() {
  int dev = 0, cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  std::vector<uint64_t*> in(RING), out(RING);
  uint64_t* sink;
  for (int i = 0; i < RING; ++i) {
    CK(hipMalloc(&in[i], IN_U64 * 8));
    CK(hipMalloc(&out[i], OUT_U64 * 8));
    CK(hipMemset(in[i], 1, IN_U64 * 8));
    CK(hipMemset(out[i], 0, OUT_U64 * 8));
  }
  CK(hipMalloc(&sink, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double in_mb = IN_U64 * 8 / 1e6, out_mb = OUT_U64 * 8 / 1e6;
  auto run = [&](const char* name, double mb, auto launch) -> int {
    for (int w = 0; w < 2 * RING; ++w) launch(w % RING);
    CK(hipDeviceSynchronize());
    const int iters = 20 * RING;
    float best = 1e9f, tot = 0.f;
    for (int it = 0; it < iters; ++it) {
      CK(hipEventRecord(e0, 0));
      launch(it % RING);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
      tot += ms;
    }
    const double us = 1e3 * tot / iters;
    printf("%-44s avg %7.2f us  min %7.2f us  %7.1f GB/s (%.1f MB)\n", name, us, 1e3 * best, mb * 1e3 / us, mb);
    return 0;
  };
  for (int wg_per_cu : {2, 4}) {
    const dim3 g(std::max(1, wg_per_cu * cus / (int)JOBS), 1, JOBS);
    char nm[96];
    snprintf(nm, sizeof nm, "skel read+write (%d WG/CU)", wg_per_cu);
    if (run(nm, in_mb + out_mb, [&](int r) { skel8<true, true><<<g, kWaves * 64>>>(in[r], out[r], sink); })) return 1;
    snprintf(nm, sizeof nm, "skel read only (%d WG/CU)", wg_per_cu);
    if (run(nm, in_mb, [&](int r) { skel8<true, false><<<g, kWaves * 64>>>(in[r], out[r], sink); })) return 1;
    snprintf(nm, sizeof nm, "skel write only, 8 B/lane (%d WG/CU)", wg_per_cu);
    if (run(nm, out_mb, [&](int r) { skel8<false, true><<<g, kWaves * 64>>>(in[r], out[r], sink); })) return 1;
    snprintf(nm, sizeof nm, "write only, 16 B/lane (%d WG/CU)", wg_per_cu);
    if (run(nm, out_mb, [&](int r) { write16<<<g, kWaves * 64>>>(out[r]); })) return 1;
  }
  if (run("stream write, 16 B/lane, grid-stride", out_mb,
          [&](int r) { stream_write<<<4 * cus, 256>>>(out[r], OUT_U64 / 2); }))
    return 1;
  return 0;
}
