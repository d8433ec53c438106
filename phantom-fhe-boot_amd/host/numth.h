// numth.h — host-side number theory for parameter and table generation.
//
// Behaviour follows the reference's host layer (src/host/numth.cu, src/host/modulus.cu,
// src/host/ntt.cu); the implementation is this engine's own (exact 128-bit integers,
// deterministic primality testing).
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <vector>

namespace phantom::arith {

using u128 = unsigned __int128;

inline uint64_t mul_mod(uint64_t a, uint64_t b, uint64_t q) { return static_cast<uint64_t>((u128)a * b % q); }
uint64_t pow_mod(uint64_t a, uint64_t e, uint64_t q);
// returns false when a has no inverse mod q (try_invert_uint_mod)
bool try_invert_mod(uint64_t a, uint64_t q, uint64_t& out);
uint64_t inv_mod(uint64_t a, uint64_t q);
bool is_prime(uint64_t v);
// floor(w * 2^64 / q) (compute_shoup, include/host/uintarithsmallmod.h:119-124)
inline uint64_t shoup(uint64_t w, uint64_t q) { return static_cast<uint64_t>(((u128)w << 64) / q); }
// floor(2^128 / q) as {lo, hi} (Modulus::set_value, src/host/modulus.cu:15-48)
void barrett_ratio(uint64_t q, uint64_t out[2]);
int significant_bits(uint64_t v);
int log2_exact(uint64_t n);  // -1 if n is not a power of two
uint32_t reverse_bits(uint32_t x, int bits);
// try_minimal_primitive_root (src/host/numth.cu:309-332)
uint64_t minimal_primitive_root(uint64_t degree, uint64_t q);
// get_primes (src/host/numth.cu:207-233)
std::vector<uint64_t> get_primes(size_t n, int bit_size, size_t count);

}  // namespace phantom::arith
