#include "modulus.h"

#include <algorithm>
#include <map>

#include "numth.h"

namespace phantom::arith {

void Modulus::set_value(uint64_t value) {
  if (value == 0) {
    *this = Modulus();
    return;
  }
  if ((value >> MOD_BIT_COUNT_MAX) != 0 || value == 1)
    throw std::invalid_argument("value can be at most 61-bit and cannot be 1");
  value_ = value;
  bit_count_ = significant_bits(value);
  barrett_ratio(value, const_ratio_);
  const u128 two128_minus = ~static_cast<u128>(0);
  const u128 quo = (static_cast<u128>(const_ratio_[1]) << 64) | const_ratio_[0];
  // remainder of 2^128 / q (const_ratio_[2] in the reference)
  const_ratio_[2] = static_cast<uint64_t>(two128_minus - quo * value + 1);
  is_prime_ = arith::is_prime(value);
}

std::vector<Modulus> CoeffModulus::Create(size_t n, const std::vector<int>& bit_sizes) {
  if (n > POLY_MOD_DEGREE_MAX || n < POLY_MOD_DEGREE_MIN || log2_exact(n) < 0)
    throw std::invalid_argument("poly_modulus_degree is invalid");
  if (bit_sizes.size() > COEFF_MOD_COUNT_MAX) throw std::invalid_argument("bit_sizes is invalid");
  for (int b : bit_sizes)
    if (b < USER_MOD_BIT_COUNT_MIN || b > USER_MOD_BIT_COUNT_MAX) throw std::invalid_argument("bit_sizes is invalid");
  std::map<int, size_t> count;
  for (int b : bit_sizes) ++count[b];
  std::map<int, std::vector<uint64_t>> primes;
  for (auto& [b, c] : count) primes[b] = get_primes(n, b, c);
  std::vector<Modulus> out;
  out.reserve(bit_sizes.size());
  for (int b : bit_sizes) {
    out.emplace_back(primes[b].back());
    primes[b].pop_back();
  }
  return out;
}

}  // namespace phantom::arith
