#include "serialize.h"

#include <algorithm>
#include <limits>
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
// a bool is one byte on the wire; any byte value other than 0/1 is rejected (reading it into a
// bool object directly would be undefined behaviour)
void get(std::istream& is, bool& v) {
  uint8_t b = 0;
  get(is, b);
  if (b > 1) throw std::runtime_error("serialized object has an invalid flag byte");
  v = b != 0;
}
void put_words(std::ostream& os, const uint64_t* p, uint64_t n) {
  os.write(reinterpret_cast<const char*>(p), static_cast<std::streamsize>(n * sizeof(uint64_t)));
}
void get_words(std::istream& is, std::vector<uint64_t>& v, uint64_t n) {
  // 2^36 words = 512 GiB is beyond any object of the supported parameter sets
  if (n > (uint64_t(1) << 36)) throw std::runtime_error("serialized object too large");
  // grow with the data actually read: a corrupt or hostile header cannot make this allocate
  // more than about twice the bytes the stream really holds
  constexpr uint64_t kChunk = uint64_t(1) << 20;
  v.clear();
  uint64_t done = 0;
  while (done < n) {
    const uint64_t c = std::min(kChunk, n - done);
    v.resize(done + c);
    is.read(reinterpret_cast<char*>(v.data() + done), static_cast<std::streamsize>(c * sizeof(uint64_t)));
    if (!is) throw std::runtime_error("serialized object truncated");
    done += c;
  }
}
}  // namespace

uint64_t checked_words(uint64_t a, uint64_t b, uint64_t c) {
  uint64_t ab = 0, abc = 0;
  if (__builtin_mul_overflow(a, b, &ab) || __builtin_mul_overflow(ab, c, &abc) ||
      abc > (std::numeric_limits<uint64_t>::max() / sizeof(uint64_t)))
    throw std::runtime_error("serialized object size overflows");
  return abc;
}

uint64_t CiphertextHeader::words() const { return checked_words(size, coeff_modulus_size, poly_modulus_degree); }
uint64_t PlaintextHeader::words() const { return checked_words(1, coeff_modulus_size, poly_modulus_degree); }

void write_ciphertext(std::ostream& os, const CiphertextHeader& h, const uint64_t* data) {
  write_ciphertext_header(os, h);
  put_words(os, data, h.words());
}

void write_ciphertext_header(std::ostream& os, const CiphertextHeader& h) {
  put(os, h.chain_index);
  put(os, h.size);
  put(os, h.poly_modulus_degree);
  put(os, h.coeff_modulus_size);
  put(os, h.scale);
  put(os, h.correction_factor);
  put(os, h.noise_scale_deg);
  put(os, h.is_ntt_form);
  put(os, h.is_asymmetric);
}

void read_ciphertext(std::istream& is, CiphertextHeader& h, std::vector<uint64_t>& data) {
  read_ciphertext_header(is, h);
  get_words(is, data, h.words());
}

void read_ciphertext_header(std::istream& is, CiphertextHeader& h) {
  get(is, h.chain_index);
  get(is, h.size);
  get(is, h.poly_modulus_degree);
  get(is, h.coeff_modulus_size);
  get(is, h.scale);
  get(is, h.correction_factor);
  get(is, h.noise_scale_deg);
  get(is, h.is_ntt_form);
  get(is, h.is_asymmetric);
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

void write_u64(std::ostream& os, uint64_t v) { put(os, v); }

uint64_t read_u64(std::istream& is) {
  uint64_t v = 0;
  get(is, v);
  return v;
}

void write_kswitch_key(std::ostream& os, uint64_t n, uint64_t size_QP, const std::vector<const uint64_t*>& digits) {
  put(os, static_cast<uint64_t>(digits.size()));
  for (const uint64_t* d : digits) {
    CiphertextHeader h;
    h.chain_index = 0;
    h.size = 2;
    h.poly_modulus_degree = n;
    h.coeff_modulus_size = size_QP;
    write_ciphertext(os, h, d);
  }
}

void read_kswitch_key(std::istream& is, uint64_t n, uint64_t size_QP, std::vector<std::vector<uint64_t>>& digits) {
  uint64_t dnum = 0;
  get(is, dnum);
  if (dnum > 64) throw std::runtime_error("bad key-switching key stream");
  digits.assign(dnum, {});
  for (auto& d : digits) {
    CiphertextHeader h;
    read_ciphertext(is, h, d);
    if (h.chain_index != 0 || h.size != 2 || h.poly_modulus_degree != n || h.coeff_modulus_size != size_QP)
      throw std::invalid_argument("key-switching key does not match the context");
  }
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
  get_words(is, data, checked_words(max_power, n, limbs));
}

}  // namespace phantom::ser
