#include "serialize.h"

#include <stdexcept>

namespace phantom::ser {

namespace {
template <typename T>
void put(std::ostream& os, const T& v) {
  os.write(reinterpret_cast<const char*>(&v), sizeof(T));
}
template <typename T>
void get(std::istream& is, T& v) {
  is.read(reinterpret_cast<char*>(&v), sizeof(T));
  if (!is) throw std::runtime_error("serialized object truncated");
}
void put_words(std::ostream& os, const uint64_t* p, uint64_t n) {
  os.write(reinterpret_cast<const char*>(p), static_cast<std::streamsize>(n * sizeof(uint64_t)));
}
void get_words(std::istream& is, std::vector<uint64_t>& v, uint64_t n) {
  // a corrupt header must not trigger a huge allocation: 2^36 words = 512 GiB is beyond any
  // object of the supported parameter sets
  if (n > (uint64_t(1) << 36)) throw std::runtime_error("serialized object too large");
  v.resize(n);
  is.read(reinterpret_cast<char*>(v.data()), static_cast<std::streamsize>(n * sizeof(uint64_t)));
  if (!is) throw std::runtime_error("serialized object truncated");
}
}  // namespace

void write_ciphertext(std::ostream& os, const CiphertextHeader& h, const uint64_t* data) {
  put(os, h.chain_index);
  put(os, h.size);
  put(os, h.poly_modulus_degree);
  put(os, h.coeff_modulus_size);
  put(os, h.scale);
  put(os, h.correction_factor);
  put(os, h.noise_scale_deg);
  put(os, h.is_ntt_form);
  put(os, h.is_asymmetric);
  put_words(os, data, h.words());
}

void read_ciphertext(std::istream& is, CiphertextHeader& h, std::vector<uint64_t>& data) {
  get(is, h.chain_index);
  get(is, h.size);
  get(is, h.poly_modulus_degree);
  get(is, h.coeff_modulus_size);
  get(is, h.scale);
  get(is, h.correction_factor);
  get(is, h.noise_scale_deg);
  get(is, h.is_ntt_form);
  get(is, h.is_asymmetric);
  get_words(is, data, h.words());
}

void write_plaintext(std::ostream& os, const PlaintextHeader& h, const uint64_t* data) {
  put(os, h.chain_index);
  put(os, h.poly_modulus_degree);
  put(os, h.coeff_modulus_size);
  put(os, h.scale);
  put_words(os, data, h.words());
}

void read_plaintext(std::istream& is, PlaintextHeader& h, std::vector<uint64_t>& data) {
  get(is, h.chain_index);
  get(is, h.poly_modulus_degree);
  get(is, h.coeff_modulus_size);
  get(is, h.scale);
  get_words(is, data, h.words());
}

void write_secret_key(std::ostream& os, uint64_t max_power, uint64_t n, uint64_t limbs, const uint64_t* data) {
  put(os, max_power);
  put(os, n);
  put(os, limbs);
  put_words(os, data, max_power * n * limbs);
}

void read_secret_key(std::istream& is, uint64_t& max_power, uint64_t& n, uint64_t& limbs, std::vector<uint64_t>& data) {
  get(is, max_power);
  get(is, n);
  get(is, limbs);
  get_words(is, data, max_power * n * limbs);
}

}  // namespace phantom::ser
