#include "random.h"

#include <sys/random.h>

#include <cerrno>
#include <cstring>
#include <stdexcept>

namespace phantom {

void os_entropy(void* out, size_t bytes) {
  auto* p = static_cast<unsigned char*>(out);
  while (bytes) {
    const ssize_t r = getrandom(p, bytes, 0);
    if (r < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("getrandom failed: ") + std::strerror(errno));
    }
    p += r;
    bytes -= static_cast<size_t>(r);
  }
}

RandomStream::RandomStream() { os_entropy(key_.k, sizeof(key_.k)); }

RandomStream RandomStream::for_testing(uint64_t seed) {
  // key = first half of ChaCha20(label key, counter 0, nonce seed)
  phx::ChaChaKey label{{0x74736574u, 0x796c6e6fu, 0x6465732du, 0x78696665u, 0u, 0u, 0u, 0u}};  // "testonly-sedfixe"
  uint32_t b[16];
  phx::chacha20_block(label, 0, seed, b);
  phx::ChaChaKey k;
  for (int i = 0; i < 8; ++i) k.k[i] = b[i];
  return RandomStream(k);
}

RandomStream RandomStream::derive() {
  uint32_t b[16];
  phx::chacha20_block(key_, 0, next_draw(), b);
  phx::ChaChaKey k;
  for (int i = 0; i < 8; ++i) k.k[i] = b[i];
  return RandomStream(k);
}

void RandomStream::host_words(uint64_t* out, size_t count) {
  const uint64_t nonce = next_draw();
  uint32_t b[16];
  for (size_t i = 0; i < count; ++i) {
    if (i % 8 == 0) phx::chacha20_block(key_, i / 8, nonce, b);
    out[i] = phx::chacha_word64(b, static_cast<int>(i % 8));
  }
}

}  // namespace phantom
