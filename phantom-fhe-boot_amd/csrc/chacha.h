// chacha.h — the ChaCha20 block function (D. J. Bernstein; RFC 8439 section 2.3), the
// cryptographic generator behind every random draw of this library: the secret key, the error
// and the uniform polynomials of key generation and encryption.  The reference samples from a
// Salsa20-based generator seeded by std::random_device (include/prng.cuh:13-24, src/prng.cu);
// ChaCha20 is Salsa20's successor with the same 512-bit state and counter-based access, so a GPU
// thread computes the block it needs from (key, counter, nonce) with no shared state.
//
// State layout: 4 constant words, 8 key words, a 64-bit block counter (words 12-13) and a 64-bit
// nonce (words 14-15), Bernstein's original split.  RFC 8439's 32-bit counter / 96-bit nonce
// test vectors map onto it as counter = c | n0 << 32, nonce = n1 | n2 << 32.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace phx {

// 256-bit ChaCha20 key
struct ChaChaKey {
  uint32_t k[8];
};

__host__ __device__ __forceinline__ uint32_t chacha_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

#define PHX_CHACHA_QR(a, b, c, d) \
  a += b;                         \
  d ^= a;                         \
  d = chacha_rotl(d, 16);         \
  c += d;                         \
  b ^= c;                         \
  b = chacha_rotl(b, 12);         \
  a += b;                         \
  d ^= a;                         \
  d = chacha_rotl(d, 8);          \
  c += d;                         \
  b ^= c;                         \
  b = chacha_rotl(b, 7);

// out[16] = ChaCha20(key, counter, nonce): 64 bytes of keystream
__host__ __device__ __forceinline__ void chacha20_block(const ChaChaKey& key, uint64_t counter, uint64_t nonce,
                                                        uint32_t out[16]) {
  const uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,  // "expand 32-byte k"
                           key.k[0],    key.k[1],    key.k[2],    key.k[3],
                           key.k[4],    key.k[5],    key.k[6],    key.k[7],
                           static_cast<uint32_t>(counter), static_cast<uint32_t>(counter >> 32),
                           static_cast<uint32_t>(nonce),   static_cast<uint32_t>(nonce >> 32)};
  uint32_t x[16];
  for (int i = 0; i < 16; ++i) x[i] = in[i];
  for (int r = 0; r < 10; ++r) {  // 10 double rounds = 20 rounds
    PHX_CHACHA_QR(x[0], x[4], x[8], x[12])
    PHX_CHACHA_QR(x[1], x[5], x[9], x[13])
    PHX_CHACHA_QR(x[2], x[6], x[10], x[14])
    PHX_CHACHA_QR(x[3], x[7], x[11], x[15])
    PHX_CHACHA_QR(x[0], x[5], x[10], x[15])
    PHX_CHACHA_QR(x[1], x[6], x[11], x[12])
    PHX_CHACHA_QR(x[2], x[7], x[8], x[13])
    PHX_CHACHA_QR(x[3], x[4], x[9], x[14])
  }
  for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}

#undef PHX_CHACHA_QR

// word i (< 8) of a block as 64-bit little-endian values
__host__ __device__ __forceinline__ uint64_t chacha_word64(const uint32_t b[16], int i) {
  return static_cast<uint64_t>(b[2 * i]) | (static_cast<uint64_t>(b[2 * i + 1]) << 32);
}

}  // namespace phx
