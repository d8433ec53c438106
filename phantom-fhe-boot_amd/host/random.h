// random.h — entropy and keyed random streams for key generation and encryption.
//
// The reference seeds a Salsa20 generator from std::random_device for every key and every
// encryption (include/prng.cuh:13-24, src/secretkey.cu random_bytes).  Here:
//   * os_entropy() reads the operating system's CSPRNG (getrandom(2));
//   * a RandomStream is a 256-bit ChaCha20 key plus a draw counter: draw k of the stream is the
//     ChaCha20 keystream under nonce k, so no two draws of one stream share keystream, and
//     device kernels compute their blocks from (key, counter = block index, nonce = draw).
// Streams are seeded from os_entropy() by default.  Fixed seeds exist only for reproducible
// tests (RandomStream::for_testing); no object exposes a stream key.
#pragma once

#include <cstddef>
#include <cstdint>

#include "../csrc/chacha.h"

namespace phantom {

// fills `out` with `bytes` bytes from the operating system's CSPRNG; throws on failure
void os_entropy(void* out, size_t bytes);

class RandomStream {
 public:
  // a fresh stream keyed from os_entropy()
  RandomStream();
  // a reproducible stream for tests: the key is derived from `seed` through ChaCha20 under a
  // fixed label, so it is not the seed itself but anyone who knows the seed knows the stream
  static RandomStream for_testing(uint64_t seed);
  // a stream keyed by a caller-held 256-bit secret (e.g. one the key owner drew from the OS and
  // shares with the replicas that must regenerate identical keys)
  static RandomStream from_key(const phx::ChaChaKey& k) { return RandomStream(k); }
  // a child stream keyed by 32 bytes of this stream's output (itself one draw)
  RandomStream derive();

  const phx::ChaChaKey& key() const { return key_; }
  // the nonce of the next draw; each call consumes one
  uint64_t next_draw() { return draws_++; }
  // `count` 64-bit words of one draw, computed on the host
  void host_words(uint64_t* out, size_t count);

 private:
  explicit RandomStream(const phx::ChaChaKey& k) : key_(k) {}
  phx::ChaChaKey key_{};
  uint64_t draws_ = 0;
};

}  // namespace phantom
