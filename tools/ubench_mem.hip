// Memory-pattern micro-benchmarks for the NTT pass structure on gfx950 (tools only).
// Buffer ring of 15 x [44][65536] u64 (> 256 MiB Infinity Cache) as in bench.py.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr size_t N = 1 << 16, L = 44, TOT = N * L;

// in-place "touch" copy: x = x + 1, 16 B per lane, grid-stride
__global__ void touch16(uint64_t* d, size_t n2) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
    ulonglong2 v = reinterpret_cast<ulonglong2*>(d)[i];
    v.x += 1; v.y += 1;
    reinterpret_cast<ulonglong2*>(d)[i] = v;
  }
}
__global__ void touch8(uint64_t* d, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] += 1;
}
// column-tile pattern: tile = 16 cols x 256 rows (stride 256), 256 threads: c = tid%16, t = tid/16, rows t + 16 j
__global__ void coltile8(uint64_t* d) {
  const int tiles = L * 16;
  const int c = threadIdx.x % 16, t = threadIdx.x / 16;
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    uint64_t* base = d + (size_t)(tile / 16) * N + (tile % 16) * 16 + c;
    uint64_t v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = base[(size_t)(t + 16 * j) * 256];
#pragma unroll
    for (int j = 0; j < 16; ++j) base[(size_t)(t + 16 * j) * 256] = v[j] + 1;
  }
}
// same tile, 16 B per lane: 8 lanes per 16-col row segment, 32 row-threads x 8 rows
__global__ void coltile16(uint64_t* d) {
  const int tiles = L * 16;
  const int c = threadIdx.x % 8, t = threadIdx.x / 8;
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    uint64_t* base = d + (size_t)(tile / 16) * N + (tile % 16) * 16 + 2 * c;
    ulonglong2 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<ulonglong2*>(base + (size_t)(t + 32 * j) * 256);
#pragma unroll
    for (int j = 0; j < 8; ++j) { v[j].x += 1; v[j].y += 1; *reinterpret_cast<ulonglong2*>(base + (size_t)(t + 32 * j) * 256) = v[j]; }
  }
}
// wider column tile: 32 cols (256 B per row segment), 16 B per lane
__global__ void coltile32(uint64_t* d) {
  const int tiles = L * 8;
  const int c = threadIdx.x % 16, t = threadIdx.x / 16;
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    uint64_t* base = d + (size_t)(tile / 8) * N + (tile % 8) * 32 + 2 * c;
    ulonglong2 v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = *reinterpret_cast<ulonglong2*>(base + (size_t)(t + 16 * j) * 256);
#pragma unroll
    for (int j = 0; j < 16; ++j) { v[j].x += 1; v[j].y += 1; *reinterpret_cast<ulonglong2*>(base + (size_t)(t + 16 * j) * 256) = v[j]; }
  }
}
// row pattern 8 B: wave = 4 rows, lane t = lane % 16 holds t + 16 j
__global__ void rowtile8(uint64_t* d) {
  const int items = L * 64;
  const int lane = threadIdx.x % 64, w = threadIdx.x / 64, lr = lane / 16, t = lane % 16;
  for (int it = blockIdx.x * 4 + w; it < items; it += gridDim.x * 4) {
    uint64_t* base = d + (size_t)(it / 64) * N + (size_t)((it % 64) * 4 + lr) * 256 + t;
    uint64_t v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = base[16 * j];
#pragma unroll
    for (int j = 0; j < 16; ++j) base[16 * j] = v[j] + 1;
  }
}

int main() {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int ring = 15;
  std::vector<uint64_t*> buf(ring);
  for (auto& b : buf) { CK(hipMalloc(&b, TOT * 8)); CK(hipMemset(b, 0, TOT * 8)); }
  auto time = [&](const char* name, auto launch) {
    for (int i = 0; i < 10; ++i) launch(buf[i % ring]);
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int i = 0; i < 60; ++i) {
      CK(hipEventRecord(e0)); launch(buf[i % ring]); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms * 1000);
    }
    std::sort(ts.begin(), ts.end());
    double us = ts[ts.size() / 2];
    printf("%-28s %8.2f us  %7.1f GB/s (16 B/coef)\n", name, us, TOT * 16.0 / us / 1e3);
    return 0;
  };
  for (int g : {1024, 2048, 4096})
    { char nm[64]; snprintf(nm, 64, "touch16 grid%d", g); time(nm, [&](uint64_t* b) { touch16<<<g, 256>>>(b, TOT / 2); }); }
  time("touch8 grid2048", [&](uint64_t* b) { touch8<<<2048, 256>>>(b, TOT); });
  for (int g : {256, 512, 704})
    { char nm[64]; snprintf(nm, 64, "coltile8 grid%d", g); time(nm, [&](uint64_t* b) { coltile8<<<g, 256>>>(b); }); }
  for (int g : {256, 512, 704})
    { char nm[64]; snprintf(nm, 64, "coltile16 grid%d", g); time(nm, [&](uint64_t* b) { coltile16<<<g, 256>>>(b); }); }
  for (int g : {176, 352})
    { char nm[64]; snprintf(nm, 64, "coltile32 grid%d", g); time(nm, [&](uint64_t* b) { coltile32<<<g, 256>>>(b); }); }
  for (int g : {256, 512, 704})
    { char nm[64]; snprintf(nm, 64, "rowtile8 grid%d", g); time(nm, [&](uint64_t* b) { rowtile8<<<g, 256>>>(b); }); }
  // back-to-back pair on the same buffer (second pass MALL-warm)
  time("coltile16+touch16 pair", [&](uint64_t* b) { coltile16<<<512, 256>>>(b); touch16<<<2048, 256>>>(b, TOT / 2); });
  time("touch16+touch16 pair", [&](uint64_t* b) { touch16<<<2048, 256>>>(b, TOT / 2); touch16<<<2048, 256>>>(b, TOT / 2); });
  return 0;
}
