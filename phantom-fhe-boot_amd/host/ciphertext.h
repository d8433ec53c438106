// ciphertext.h — PhantomCiphertext / PhantomPlaintext (include/ciphertext.h, include/plaintext.h):
// device-resident RNS polynomials in the reference's layout data[(poly * L + limb) * n + k].
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <istream>
#include <ostream>
#include <utility>
#include <vector>

#include "buffer.h"
#include "context.h"

namespace phantom {

class PhantomCiphertext {
 public:
  static constexpr size_t kSeedBytes = 64;  // prng_seed_byte_count (include/host/globals.h:20-21)
  PhantomCiphertext() = default;
  PhantomCiphertext(PhantomCiphertext&& o) noexcept { *this = std::move(o); }
  // moves leave the source empty (sizes zeroed with the buffer)
  PhantomCiphertext& operator=(PhantomCiphertext&& o) noexcept {
    if (this != &o) {
      chain_index_ = o.chain_index_;
      size_ = o.size_;
      n_ = o.n_;
      L_ = o.L_;
      scale_ = o.scale_;
      correction_factor_ = o.correction_factor_;
      noise_scale_deg_ = o.noise_scale_deg_;
      is_ntt_form_ = o.is_ntt_form_;
      is_asymmetric_ = o.is_asymmetric_;
      seed_ = std::move(o.seed_);
      seed_fp_ = std::move(o.seed_fp_);
      data_ = std::move(o.data_);
      sf_ = std::move(o.sf_);
      sf_big_ = std::move(o.sf_big_);
      o.size_ = o.L_ = o.n_ = 0;
    }
    return *this;
  }
  // deep device copy (the reference copies through cuda_auto_ptr, cuda_wrapper.cuh:94-104)
  PhantomCiphertext(const PhantomCiphertext& o) { copy_from(o); }
  PhantomCiphertext& operator=(const PhantomCiphertext& o) {
    if (this != &o) copy_from(o);
    return *this;
  }

  // ciphertext.h:50-80: reallocate for (chain_index, size); keeps the leading old data.  A
  // shrink that fits the current buffer keeps it (no copy).
  void resize(const PhantomContext& ctx, size_t chain_index, size_t size, hipStream_t s, bool copy_old = true);
  void resize(size_t size, size_t coeff_modulus_size, size_t n, hipStream_t s, bool copy_old = true);

  uint64_t* data() const { return data_.get(); }
  size_t chain_index() const { return chain_index_; }
  size_t size() const { return size_; }
  size_t poly_modulus_degree() const { return n_; }
  size_t coeff_modulus_size() const { return L_; }
  double scale() const { return scale_; }
  bool is_ntt_form() const { return is_ntt_form_; }
  uint64_t correction_factor() const { return correction_factor_; }
  size_t GetNoiseScaleDeg() const { return noise_scale_deg_; }

  void set_scale(double s) { scale_ = s; }
  void set_chain_index(size_t c) { chain_index_ = c; }
  void set_ntt_form(bool b) { is_ntt_form_ = b; }
  void SetNoiseScaleDeg(size_t d) { noise_scale_deg_ = d; }
  void set_correction_factor(uint64_t c) { correction_factor_ = c; }

  // save / load in the reference's byte format (include/ciphertext.h:184-225, host/serialize.h).
  // load takes the context for the stream it allocates on (the reference uses
  // cudaStreamPerThread); the loaded ciphertext keeps the saved chain index and sizes.
  void save(std::ostream& os) const;
  void load(const PhantomContext& ctx, std::istream& is);
  bool is_asymmetric() const { return is_asymmetric_; }
  // Seed-compressed symmetric ciphertexts (include/ciphertext.h:227-318): c0 and the 64-byte
  // seed of c1 = a instead of c1 itself.  encrypt_symmetric draws `a` from a fresh public seed
  // that the ciphertext keeps; load_symmetric regenerates c1 from it (ChaCha20 keystream, so the
  // bytes of c1 differ from the reference's Salsa20 expansion of the same seed).  Same errors as
  // the reference: asymmetric ciphertexts, size != 2, and (load) a chain below the first data
  // level throw std::runtime_error.  The seed describes c1 only while c1 is its expansion:
  // resize() drops it, and set_seed records a fingerprint of c1 (words sampled from every limb)
  // that save_symmetric re-reads, so a ciphertext whose c1 an in-place operation rewrote (rotate,
  // relinearize, add of a ciphertext, multiply_plain) throws instead of writing a stale seed;
  // operations that leave c1 alone (add_plain, sub_plain) keep the seed valid.
  void save_symmetric(std::ostream& os) const;
  void load_symmetric(const PhantomContext& ctx, std::istream& is);
  const std::vector<uint8_t>& seed() const { return seed_; }
  // c1 must already hold the seed's expansion (synchronises stream `s`)
  void set_seed(std::vector<uint8_t> seed, hipStream_t s);
  // hand the buffer to stream `s` (DeviceBuffer::set_stream): after a concurrent section, for a
  // result made on a side stream that the joining stream uses from now on
  void retag(hipStream_t s) { data_.set_stream(s); }
  void set_asymmetric(bool b) { is_asymmetric_ = b; }

  // PreComputeScale (include/ciphertext.h:320-367): the FLEXIBLEAUTO scaling factor of every level,
  // sf[0] = q_last, sf[k] = sf[k-1]^2 / q_(size_Q - k), and their squares ("big" factors)
  void PreComputeScale(const PhantomContext& ctx, double scale);
  std::vector<double>& getScalingFactorsReal() { return sf_; }
  std::vector<double>& getScalingFactorsRealBig() { return sf_big_; }

  // host transfer helpers (the reference's save/load staging, ciphertext.h:184-225)
  std::vector<uint64_t> to_host(hipStream_t s) const;
  void from_host(const PhantomContext& ctx, size_t chain_index, size_t size, const std::vector<uint64_t>& v,
                 hipStream_t s);

 private:
  void copy_from(const PhantomCiphertext& o);
  std::vector<uint64_t> c1_fingerprint(hipStream_t s) const;
  size_t chain_index_ = 0, size_ = 0, n_ = 0, L_ = 0;
  double scale_ = 1.0;
  uint64_t correction_factor_ = 1;
  size_t noise_scale_deg_ = 1;
  bool is_ntt_form_ = true;
  bool is_asymmetric_ = false;
  std::vector<uint8_t> seed_;  // prng_seed_byte_count (64) bytes after encrypt_symmetric, else empty
  std::vector<uint64_t> seed_fp_;  // c1_fingerprint() when seed_ was set
  DeviceBuffer<uint64_t> data_;
  std::vector<double> sf_, sf_big_;
};

namespace ser {
struct CiphertextHeader;
}
// throws std::invalid_argument unless a serialized header fits the context: degree, chain index,
// size 2 or 3 and the chain's limb count (everything a kernel will index by)
void check_ciphertext_header(const PhantomContext& ctx, const ser::CiphertextHeader& h);

class PhantomPlaintext {
 public:
  PhantomPlaintext() = default;
  PhantomPlaintext(PhantomPlaintext&&) noexcept = default;
  PhantomPlaintext& operator=(PhantomPlaintext&&) noexcept = default;
  // deep device copy (on this thread's stream, else the source's)
  PhantomPlaintext(const PhantomPlaintext& o) { copy_from(o); }
  PhantomPlaintext& operator=(const PhantomPlaintext& o) {
    if (this != &o) copy_from(o);
    return *this;
  }
  uint64_t* data() const { return data_.get(); }
  size_t chain_index() const { return chain_index_; }
  size_t coeff_modulus_size() const { return L_; }
  size_t poly_modulus_degree() const { return n_; }
  double scale() const { return scale_; }
  bool is_ntt_form() const { return true; }
  void set_scale(double s) { scale_ = s; }
  void set_chain_index(size_t c) { chain_index_ = c; }
  size_t GetNoiseScaleDeg() const { return noise_scale_deg_; }
  void SetNoiseScaleDeg(size_t d) { noise_scale_deg_ = d; }
  void resize(const PhantomContext& ctx, size_t chain_index, hipStream_t s);
  // `limbs` limbs tagged with `chain_index` (extended-basis plaintexts: Ql of the chain + P)
  void resize_ext(const PhantomContext& ctx, size_t chain_index, size_t limbs, hipStream_t s);
  void from_host(const PhantomContext& ctx, size_t chain_index, const std::vector<uint64_t>& v, hipStream_t s);
  // save / load in the reference's byte format (include/plaintext.h:90-122)
  void save(std::ostream& os, hipStream_t s) const;
  void load(const PhantomContext& ctx, std::istream& is);

 private:
  void copy_from(const PhantomPlaintext& o);
  size_t chain_index_ = 0, n_ = 0, L_ = 0;
  size_t noise_scale_deg_ = 1;
  double scale_ = 1.0;
  DeviceBuffer<uint64_t> data_;
};

}  // namespace phantom
