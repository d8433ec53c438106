// prng.h — the counter-based generator behind device-side sampling (ckks.hip) and the
// key-switch inner product's regeneration of a key's uniform half (rns.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace phx {

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// stream key of (seed, sid): hoisted out of per-element loops
__host__ __device__ __forceinline__ uint64_t rand_stream(uint64_t seed, uint64_t sid) {
  return mix64(seed ^ (sid * 0x9E3779B97F4A7C15ull));
}

// word w of element i of a stream
__host__ __device__ __forceinline__ uint64_t rand_word_k(uint64_t key, uint64_t i, uint32_t w) {
  return mix64(key + (i * 4 + w) * 0xD1B54A32D192ED03ull);
}

// counter-based generator: word w of element i of stream (seed, sid)
__host__ __device__ __forceinline__ uint64_t rand_word(uint64_t seed, uint64_t sid, uint64_t i, uint32_t w) {
  return rand_word_k(rand_stream(seed, sid), i, w);
}

}  // namespace phx
