// modulus.h — Modulus and CoeffModulus, mirroring the reference's
// include/host/modulus.h / src/host/modulus.cu:15-111 (same names, same semantics).
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <vector>

namespace phantom::arith {

constexpr int MOD_BIT_COUNT_MAX = 61;
constexpr int USER_MOD_BIT_COUNT_MIN = 2;
constexpr int USER_MOD_BIT_COUNT_MAX = 60;
constexpr size_t COEFF_MOD_COUNT_MAX = 64;       // include/host/defines.h:19
constexpr size_t POLY_MOD_DEGREE_MIN = 2;
constexpr size_t POLY_MOD_DEGREE_MAX = 131072;   // include/host/defines.h:23

class Modulus {
 public:
  Modulus() = default;
  explicit Modulus(uint64_t value) { set_value(value); }
  void set_value(uint64_t value);
  uint64_t value() const { return value_; }
  int bit_count() const { return bit_count_; }
  const uint64_t* const_ratio() const { return const_ratio_; }  // floor(2^128/q) {lo, hi}, remainder
  bool is_prime() const { return is_prime_; }
  bool is_zero() const { return value_ == 0; }
  bool operator==(const Modulus& o) const { return value_ == o.value_; }

 private:
  uint64_t value_ = 0;
  uint64_t const_ratio_[3] = {0, 0, 0};
  int bit_count_ = 0;
  bool is_prime_ = false;
};

class CoeffModulus {
 public:
  // CoeffModulus::Create (src/host/modulus.cu:80-111): per bit size, NTT-friendly primes
  // found largest-first and handed out from the back.
  static std::vector<Modulus> Create(size_t poly_modulus_degree, const std::vector<int>& bit_sizes);
};

}  // namespace phantom::arith
