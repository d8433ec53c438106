// salsa.h — the reference's Salsa20 seed expansion (src/prng.cu:17-140), used where bytes must
// interchange with the reference: the `a` polynomial of a symmetric ciphertext is the uniform
// expansion of its public 64-byte seed (encrypt_symmetric / save_symmetric / load_symmetric,
// include/ciphertext.h:227-318), so a seed-compressed ciphertext written by either engine loads
// in the other.  (Secret keys and errors come from ChaCha20, chacha.h: no file carries them.)
//
// The state is the reference's, not the Salsa20 stream cipher's: seed bytes 0..31 in words 0..7,
// the 64-bit nonce in words 8..9, seed bytes 32..55 in words 10..15, no constants and no block
// counter; the 20-round core is standard Salsa20 (the specification's example vector is checked
// in tests/test_capi.py).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace phx {

// the 64-byte seed as 16 little-endian words (only the first 14 enter the state)
struct SalsaSeed {
  uint32_t w[16];
};

__host__ __device__ __forceinline__ uint32_t salsa_rotl(uint32_t u, int c) { return (u << c) | (u >> (32 - c)); }

#define PHX_SALSA_QR(a, b, c, d) \
  b ^= salsa_rotl(a + d, 7);     \
  c ^= salsa_rotl(b + a, 9);     \
  d ^= salsa_rotl(c + b, 13);    \
  a ^= salsa_rotl(d + c, 18);

__host__ __device__ __forceinline__ void salsa20_core(const uint32_t in[16], uint32_t out[16]) {
  uint32_t x[16];
  for (int i = 0; i < 16; ++i) x[i] = in[i];
  for (int r = 0; r < 10; ++r) {
    PHX_SALSA_QR(x[0], x[4], x[8], x[12])
    PHX_SALSA_QR(x[5], x[9], x[13], x[1])
    PHX_SALSA_QR(x[10], x[14], x[2], x[6])
    PHX_SALSA_QR(x[15], x[3], x[7], x[11])
    PHX_SALSA_QR(x[0], x[1], x[2], x[3])
    PHX_SALSA_QR(x[5], x[6], x[7], x[4])
    PHX_SALSA_QR(x[10], x[11], x[8], x[9])
    PHX_SALSA_QR(x[15], x[12], x[13], x[14])
  }
  for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}
#undef PHX_SALSA_QR

// one block of the reference's salsa20_gpu(out, 64, nonce, seed, 64)
__host__ __device__ __forceinline__ void salsa20_block(const SalsaSeed& s, uint64_t nonce, uint32_t out[16]) {
  const uint32_t in[16] = {s.w[0], s.w[1], s.w[2],  s.w[3],  s.w[4],  s.w[5],  s.w[6],
                           s.w[7], static_cast<uint32_t>(nonce), static_cast<uint32_t>(nonce >> 32),
                           s.w[8], s.w[9], s.w[10], s.w[11], s.w[12], s.w[13]};
  salsa20_core(in, out);
}

inline SalsaSeed salsa_seed(const uint8_t* bytes) {
  SalsaSeed s;
  for (int i = 0; i < 16; ++i)
    s.w[i] = static_cast<uint32_t>(bytes[4 * i]) | (static_cast<uint32_t>(bytes[4 * i + 1]) << 8) |
             (static_cast<uint32_t>(bytes[4 * i + 2]) << 16) | (static_cast<uint32_t>(bytes[4 * i + 3]) << 24);
  return s;
}

}  // namespace phx
