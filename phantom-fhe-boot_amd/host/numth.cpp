#include "numth.h"

namespace phantom::arith {

uint64_t pow_mod(uint64_t a, uint64_t e, uint64_t q) {
  uint64_t r = 1 % q;
  a %= q;
  while (e) {
    if (e & 1) r = mul_mod(r, a, q);
    a = mul_mod(a, a, q);
    e >>= 1;
  }
  return r;
}

bool try_invert_mod(uint64_t a, uint64_t q, uint64_t& out) {
  __int128 r0 = q, r1 = a % q, s0 = 0, s1 = 1;
  while (r1 != 0) {
    __int128 k = r0 / r1, t;
    t = r0 - k * r1; r0 = r1; r1 = t;
    t = s0 - k * s1; s0 = s1; s1 = t;
  }
  if (r0 != 1) return false;
  if (s0 < 0) s0 += q;
  out = static_cast<uint64_t>(s0);
  return true;
}

uint64_t inv_mod(uint64_t a, uint64_t q) {
  uint64_t r;
  if (!try_invert_mod(a, q, r)) throw std::invalid_argument("value is not invertible modulo q");
  return r;
}

// Deterministic Miller-Rabin: the 7-base set below is exact for every 64-bit input, so it
// accepts exactly the primes the reference's randomized test accepts.
bool is_prime(uint64_t v) {
  if (v < 2) return false;
  for (uint64_t p : {2ull, 3ull, 5ull, 7ull, 11ull, 13ull, 17ull, 19ull, 23ull, 29ull, 31ull, 37ull}) {
    if (v == p) return true;
    if (v % p == 0) return false;
  }
  uint64_t d = v - 1;
  int s = 0;
  while (!(d & 1)) { d >>= 1; ++s; }
  for (uint64_t a : {2ull, 325ull, 9375ull, 28178ull, 450775ull, 9780504ull, 1795265022ull}) {
    a %= v;
    if (!a) continue;
    uint64_t x = pow_mod(a, d, v);
    if (x == 1 || x == v - 1) continue;
    bool witness = true;
    for (int i = 1; i < s && witness; ++i) {
      x = mul_mod(x, x, v);
      if (x == v - 1) witness = false;
    }
    if (witness) return false;
  }
  return true;
}

void barrett_ratio(uint64_t q, uint64_t out[2]) {
  const u128 all = ~static_cast<u128>(0);
  u128 quo = all / q;
  if (all - quo * q + 1 == q) ++quo;  // 2^128 divisible case (never for odd q > 1)
  out[0] = static_cast<uint64_t>(quo);
  out[1] = static_cast<uint64_t>(quo >> 64);
}

int significant_bits(uint64_t v) {
  int b = 0;
  while (v) { ++b; v >>= 1; }
  return b;
}

int log2_exact(uint64_t n) {
  if (n == 0 || (n & (n - 1))) return -1;
  int l = 0;
  while ((1ull << l) < n) ++l;
  return l;
}

uint32_t reverse_bits(uint32_t x, int bits) {
  uint32_t r = 0;
  for (int i = 0; i < bits; ++i) { r = (r << 1) | (x & 1); x >>= 1; }
  return r;
}

uint64_t minimal_primitive_root(uint64_t degree, uint64_t q) {
  if ((q - 1) % degree) throw std::invalid_argument("modulus does not support the NTT degree");
  const uint64_t cofactor = (q - 1) / degree;
  uint64_t root = 0;
  for (uint64_t g = 2; g < q && !root; ++g) {
    uint64_t c = pow_mod(g, cofactor, q);
    if (pow_mod(c, degree >> 1, q) == q - 1) root = c;
  }
  if (!root) throw std::invalid_argument("no primitive root");
  // all primitive roots are root^(odd); keep the smallest one
  const uint64_t step = mul_mod(root, root, q);
  uint64_t cur = root, best = root;
  for (uint64_t i = 0; i < degree / 2; ++i) {
    if (cur < best) best = cur;
    cur = mul_mod(cur, step, q);
  }
  return best;
}

std::vector<uint64_t> get_primes(size_t n, int bit_size, size_t count) {
  std::vector<uint64_t> out;
  const uint64_t factor = 2 * static_cast<uint64_t>(n);
  uint64_t value = (1ull << bit_size) - factor + 1;
  const uint64_t lower = 1ull << (bit_size - 1);
  while (out.size() < count && value > lower) {
    if (is_prime(value)) out.push_back(value);
    value -= factor;
  }
  if (out.size() < count) throw std::logic_error("failed to find enough qualifying primes");
  return out;
}

}  // namespace phantom::arith
