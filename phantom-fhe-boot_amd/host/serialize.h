// serialize.h — byte formats of the reference's save/load, so ciphertexts, plaintexts, secret
// keys and key-switching keys move between the reference and this engine (and between ranks).
//   ciphertext (include/ciphertext.h:184-201): chain_index, size, poly_modulus_degree,
//     coeff_modulus_size (size_t each), scale (double), correction_factor (uint64_t),
//     noiseScaleDeg (size_t), is_ntt_form, is_asymmetric (bool, 1 byte each), then
//     size * coeff_modulus_size * poly_modulus_degree uint64_t words;
//   plaintext (include/plaintext.h:90-103): chain_index, poly_modulus_degree,
//     coeff_modulus_size (size_t), scale (double), then the words;
//   secret key (include/secretkey.h:405-418): sk_max_power, poly_modulus_degree,
//     coeff_modulus_size (size_t), then the words;
//   key-switching key (PhantomRelinKey::save, include/secretkey.h:130-141): dnum (size_t), then
//     dnum public keys, each a ciphertext of 2 polynomials over the key level (chain index 0);
//   Galois key (include/secretkey.h:195-205): count (size_t), then that many relin keys.
// Fields are written one by one in native (little-endian) byte order with no padding, as
// std::ostream::write of each member does in the reference.
#pragma once

#include <cstdint>
#include <istream>
#include <ostream>
#include <vector>

namespace phantom::ser {

struct CiphertextHeader {
  uint64_t chain_index = 0, size = 0, poly_modulus_degree = 0, coeff_modulus_size = 0;
  double scale = 1.0;
  uint64_t correction_factor = 1, noise_scale_deg = 1;
  bool is_ntt_form = true, is_asymmetric = false;
  // size * coeff_modulus_size * poly_modulus_degree; throws std::runtime_error on overflow
  uint64_t words() const;
};
constexpr size_t kCiphertextHeaderBytes = 4 * 8 + 8 + 8 + 8 + 1 + 1;  // 58

struct PlaintextHeader {
  uint64_t chain_index = 0, poly_modulus_degree = 0, coeff_modulus_size = 0;
  double scale = 1.0;
  uint64_t words() const;
};
constexpr size_t kPlaintextHeaderBytes = 3 * 8 + 8;  // 32

// a * b * c, std::runtime_error if the product does not fit 64 bits
uint64_t checked_words(uint64_t a, uint64_t b, uint64_t c);

void write_ciphertext(std::ostream& os, const CiphertextHeader& h, const uint64_t* data);
void write_ciphertext_header(std::ostream& os, const CiphertextHeader& h);
// throws std::runtime_error on a short or inconsistent stream.  The payload is read in bounded
// chunks, so a header that claims more words than the stream holds fails after reading what is
// there instead of allocating what it claims.
void read_ciphertext(std::istream& is, CiphertextHeader& h, std::vector<uint64_t>& data);
void read_ciphertext_header(std::istream& is, CiphertextHeader& h);
void write_plaintext(std::ostream& os, const PlaintextHeader& h, const uint64_t* data);
void read_plaintext(std::istream& is, PlaintextHeader& h, std::vector<uint64_t>& data);
// key-switching key (PhantomRelinKey::save, include/secretkey.h:130-141): dnum, then every digit
// as a 2-polynomial key-level ciphertext (chain 0, size_QP limbs, scale 1, NTT form); digits[i]
// points at [2][size_QP][n] host words
void write_kswitch_key(std::ostream& os, uint64_t n, uint64_t size_QP, const std::vector<const uint64_t*>& digits);
// the inverse; throws std::runtime_error / std::invalid_argument on a malformed or mismatched stream
void read_kswitch_key(std::istream& is, uint64_t n, uint64_t size_QP, std::vector<std::vector<uint64_t>>& digits);
void write_u64(std::ostream& os, uint64_t v);
uint64_t read_u64(std::istream& is);
void write_secret_key(std::ostream& os, uint64_t max_power, uint64_t n, uint64_t limbs, const uint64_t* data);
void read_secret_key(std::istream& is, uint64_t& max_power, uint64_t& n, uint64_t& limbs, std::vector<uint64_t>& data);

}  // namespace phantom::ser
