#include "ciphertext.h"

#include <algorithm>
#include <stdexcept>

#include "../csrc/ntt.h"
#include "hip_check.h"
#include "keys.h"
#include "serialize.h"

namespace phantom {

void PhantomCiphertext::resize(const PhantomContext& ctx, size_t chain_index, size_t size, hipStream_t s,
                               bool copy_old) {
  const auto& cd = ctx.get_context_data(chain_index);
  resize(size, cd.coeff_modulus_size(), ctx.poly_degree(), s, copy_old);
  chain_index_ = chain_index;
}

void PhantomCiphertext::resize(size_t size, size_t L, size_t n, hipStream_t s, bool copy_old) {
  const size_t old_count = size_ * L_ * n_, new_count = size * L * n;
  if (new_count == 0) {
    data_.release();
  } else if (data_ && new_count <= data_.size()) {
    // fits the current buffer: the leading data stays where it is (relinearize's 3 -> 2)
  } else if (new_count != old_count || !data_) {  // a moved-from ciphertext keeps its sizes
    DeviceBuffer<uint64_t> fresh(new_count, s);
    if (copy_old && data_ && old_count) {
      const size_t c = std::min(old_count, new_count);
      PHX_CHECK(hipMemcpyAsync(fresh.get(), data_.get(), c * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
    }
    data_ = std::move(fresh);
  }
  size_ = size;
  L_ = L;
  n_ = n;
  seed_.clear();  // a reshaped ciphertext is no longer the expansion of an encryption seed
  seed_fp_.clear();
}

// 8 words of every limb of c1, at coefficient positions k * n / 8
std::vector<uint64_t> PhantomCiphertext::c1_fingerprint(hipStream_t s) const {
  constexpr size_t kPerLimb = 8;
  std::vector<uint64_t> fp(kPerLimb * L_);
  if (size_ < 2 || !data_ || n_ < kPerLimb) return fp;
  const size_t stride = n_ / kPerLimb;
  PHX_CHECK(hipMemcpy2DAsync(fp.data(), sizeof(uint64_t), data_.get() + L_ * n_, stride * sizeof(uint64_t),
                             sizeof(uint64_t), fp.size(), hipMemcpyDeviceToHost, s));
  PHX_CHECK(hipStreamSynchronize(s));
  return fp;
}

void PhantomCiphertext::set_seed(std::vector<uint8_t> seed, hipStream_t s) {
  seed_ = std::move(seed);
  seed_fp_ = c1_fingerprint(s);
}

void PhantomCiphertext::save(std::ostream& os) const {
  ser::CiphertextHeader h;
  h.chain_index = chain_index_;
  h.size = size_;
  h.poly_modulus_degree = n_;
  h.coeff_modulus_size = L_;
  h.scale = scale_;
  h.correction_factor = correction_factor_;
  h.noise_scale_deg = noise_scale_deg_;
  h.is_ntt_form = is_ntt_form_;
  h.is_asymmetric = is_asymmetric_;
  const hipStream_t s = StreamScope::current() ? StreamScope::current() : data_.stream();
  const std::vector<uint64_t> v = to_host(s);
  ser::write_ciphertext(os, h, v.data());
}

void check_ciphertext_header(const PhantomContext& ctx, const ser::CiphertextHeader& h) {
  if (h.poly_modulus_degree != ctx.poly_degree()) throw std::invalid_argument("ciphertext degree mismatch");
  if (h.chain_index >= ctx.total_parm_size()) throw std::invalid_argument("ciphertext chain index out of range");
  if (h.size < 2 || h.size > 3) throw std::invalid_argument("ciphertext size must be 2 or 3");
  if (h.coeff_modulus_size != ctx.get_context_data(h.chain_index).coeff_modulus_size())
    throw std::invalid_argument("ciphertext limb count does not match its chain index");
}

void PhantomCiphertext::load(const PhantomContext& ctx, std::istream& is) {
  ser::CiphertextHeader h;
  std::vector<uint64_t> v;
  ser::read_ciphertext(is, h, v);
  check_ciphertext_header(ctx, h);
  resize(h.size, h.coeff_modulus_size, h.poly_modulus_degree, ctx.stream(), false);
  if (!v.empty()) {
    PHX_CHECK(hipMemcpyAsync(data_.get(), v.data(), v.size() * sizeof(uint64_t), hipMemcpyHostToDevice, ctx.stream()));
    PHX_CHECK(hipStreamSynchronize(ctx.stream()));
  }
  chain_index_ = h.chain_index;
  scale_ = h.scale;
  correction_factor_ = h.correction_factor;
  noise_scale_deg_ = h.noise_scale_deg;
  is_ntt_form_ = h.is_ntt_form;
  is_asymmetric_ = h.is_asymmetric;
}

void PhantomCiphertext::save_symmetric(std::ostream& os) const {
  if (is_asymmetric_) throw std::runtime_error("Asymmetric ciphertext does not have seed.");
  if (size_ != 2) throw std::runtime_error("This method is only for 2-polynomial ciphertext.");
  if (seed_.size() != kSeedBytes) throw std::runtime_error("ciphertext was not made by encrypt_symmetric");
  const hipStream_t s = StreamScope::current() ? StreamScope::current() : data_.stream();
  if (c1_fingerprint(s) != seed_fp_)
    throw std::runtime_error("ciphertext c1 was modified after encrypt_symmetric; its seed no longer describes it");
  ser::CiphertextHeader h;
  h.chain_index = chain_index_;
  h.size = size_;
  h.poly_modulus_degree = n_;
  h.coeff_modulus_size = L_;
  h.scale = scale_;
  h.correction_factor = correction_factor_;
  h.noise_scale_deg = noise_scale_deg_;
  h.is_ntt_form = is_ntt_form_;
  h.is_asymmetric = is_asymmetric_;
  std::vector<uint64_t> c0(L_ * n_);
  PHX_CHECK(hipMemcpyAsync(c0.data(), data_.get(), c0.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  PHX_CHECK(hipStreamSynchronize(s));
  ser::write_ciphertext_header(os, h);
  os.write(reinterpret_cast<const char*>(c0.data()), static_cast<std::streamsize>(c0.size() * sizeof(uint64_t)));
  os.write(reinterpret_cast<const char*>(seed_.data()), static_cast<std::streamsize>(seed_.size()));
  if (!os) throw std::runtime_error("ciphertext write failed");
}

void PhantomCiphertext::load_symmetric(const PhantomContext& ctx, std::istream& is) {
  ser::CiphertextHeader h;
  ser::read_ciphertext_header(is, h);
  if (h.is_asymmetric) throw std::runtime_error("Asymmetric ciphertext does not have seed.");
  if (h.size != 2) throw std::runtime_error("This method is only for 2-polynomial ciphertext.");
  check_ciphertext_header(ctx, h);
  if (h.coeff_modulus_size != ctx.get_context_data(1).coeff_modulus_size())
    throw std::runtime_error("Only support ciphertext without modulus switching.");
  const size_t words = h.coeff_modulus_size * h.poly_modulus_degree;
  std::vector<uint64_t> c0(words);
  std::vector<uint8_t> seed(kSeedBytes);
  is.read(reinterpret_cast<char*>(c0.data()), static_cast<std::streamsize>(words * sizeof(uint64_t)));
  is.read(reinterpret_cast<char*>(seed.data()), static_cast<std::streamsize>(seed.size()));
  if (!is) throw std::runtime_error("truncated seed-compressed ciphertext");
  const hipStream_t s = ctx.stream();
  resize(2, h.coeff_modulus_size, h.poly_modulus_degree, s, false);
  PHX_CHECK(hipMemcpyAsync(data_.get(), c0.data(), words * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  sample_uniform_seeded(ctx, seed.data(), data_.get() + words, h.coeff_modulus_size);
  if (!h.is_ntt_form)
    hip_ok(phx::ntt_inverse(ctx.gpu_rns_tables(), data_.get() + words, data_.get() + words,
                            phx::LimbMap::contiguous(static_cast<int>(h.coeff_modulus_size), 0), nullptr, nullptr, s),
           "c1 INTT");
  PHX_CHECK(hipStreamSynchronize(s));
  chain_index_ = h.chain_index;
  scale_ = h.scale;
  correction_factor_ = h.correction_factor;
  noise_scale_deg_ = h.noise_scale_deg;
  is_ntt_form_ = h.is_ntt_form;
  is_asymmetric_ = false;
  set_seed(std::move(seed), s);
}

void PhantomPlaintext::save(std::ostream& os, hipStream_t s) const {
  ser::PlaintextHeader h;
  h.chain_index = chain_index_;
  h.poly_modulus_degree = n_;
  h.coeff_modulus_size = L_;
  h.scale = scale_;
  std::vector<uint64_t> v(h.words());
  if (!v.empty()) {
    PHX_CHECK(hipMemcpyAsync(v.data(), data_.get(), v.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    PHX_CHECK(hipStreamSynchronize(s));
  }
  ser::write_plaintext(os, h, v.data());
}

void PhantomPlaintext::load(const PhantomContext& ctx, std::istream& is) {
  ser::PlaintextHeader h;
  std::vector<uint64_t> v;
  ser::read_plaintext(is, h, v);
  if (h.poly_modulus_degree != ctx.poly_degree()) throw std::invalid_argument("plaintext degree mismatch");
  if (h.chain_index >= ctx.total_parm_size()) throw std::invalid_argument("plaintext chain index out of range");
  // a chain's Ql limbs, or Ql u P for an extended-basis plaintext
  const size_t ql = ctx.get_context_data(h.chain_index).coeff_modulus_size();
  if (h.coeff_modulus_size != ql && h.coeff_modulus_size != ql + ctx.size_P())
    throw std::invalid_argument("plaintext limb count does not match its chain index");
  chain_index_ = h.chain_index;
  n_ = h.poly_modulus_degree;
  L_ = h.coeff_modulus_size;
  scale_ = h.scale;
  data_.allocate(v.size(), ctx.stream());
  if (!v.empty()) {
    PHX_CHECK(hipMemcpyAsync(data_.get(), v.data(), v.size() * sizeof(uint64_t), hipMemcpyHostToDevice, ctx.stream()));
    PHX_CHECK(hipStreamSynchronize(ctx.stream()));
  }
}

void PhantomCiphertext::PreComputeScale(const PhantomContext& ctx, double scale) {
  const size_t sizeQ = ctx.size_Q();
  const auto& m = ctx.key_moduli();
  sf_.assign(sizeQ, 0.0);
  if (sizeQ == 1) {
    sf_[0] = scale;
  } else {
    sf_[0] = static_cast<double>(m[sizeQ - 1]);
    for (size_t k = 1; k < sizeQ; ++k) {
      sf_[k] = sf_[k - 1] * sf_[k - 1] / static_cast<double>(m[sizeQ - k]);
      const double ratio = sf_[k] / sf_[0];
      if (ratio <= 0.5 || ratio >= 2.0)
        throw std::invalid_argument("FLEXIBLEAUTO cannot support this number of levels in this parameter setting");
    }
  }
  sf_big_.assign(sizeQ > 0 ? sizeQ - 1 : 0, 0.0);
  for (size_t k = 0; k < sf_big_.size(); ++k) sf_big_[k] = sf_[k] * sf_[k];
}

void PhantomCiphertext::copy_from(const PhantomCiphertext& o) {
  chain_index_ = o.chain_index_;
  size_ = o.size_;
  n_ = o.n_;
  L_ = o.L_;
  scale_ = o.scale_;
  correction_factor_ = o.correction_factor_;
  noise_scale_deg_ = o.noise_scale_deg_;
  is_ntt_form_ = o.is_ntt_form_;
  is_asymmetric_ = o.is_asymmetric_;
  seed_ = o.seed_;
  seed_fp_ = o.seed_fp_;
  sf_ = o.sf_;
  sf_big_ = o.sf_big_;
  const size_t count = size_ * L_ * n_;
  // the copy runs on this thread's stream (a StreamScope's), else on the source's stream
  hipStream_t s = StreamScope::current() ? StreamScope::current() : o.data_.stream();
  data_.allocate(count, s);
  if (count) PHX_CHECK(hipMemcpyAsync(data_.get(), o.data_.get(), count * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
}

std::vector<uint64_t> PhantomCiphertext::to_host(hipStream_t s) const {
  std::vector<uint64_t> v(size_ * L_ * n_);
  if (!v.empty()) {
    PHX_CHECK(hipMemcpyAsync(v.data(), data_.get(), v.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    PHX_CHECK(hipStreamSynchronize(s));
  }
  return v;
}

void PhantomCiphertext::from_host(const PhantomContext& ctx, size_t chain_index, size_t size,
                                  const std::vector<uint64_t>& v, hipStream_t s) {
  resize(ctx, chain_index, size, s, false);
  if (v.size() != size_ * L_ * n_) throw std::invalid_argument("ciphertext data size mismatch");
  PHX_CHECK(hipMemcpyAsync(data_.get(), v.data(), v.size() * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  PHX_CHECK(hipStreamSynchronize(s));
}

void PhantomPlaintext::copy_from(const PhantomPlaintext& o) {
  chain_index_ = o.chain_index_;
  n_ = o.n_;
  L_ = o.L_;
  noise_scale_deg_ = o.noise_scale_deg_;
  scale_ = o.scale_;
  const size_t count = L_ * n_;
  hipStream_t s = StreamScope::current() ? StreamScope::current() : o.data_.stream();
  data_.allocate(count, s);
  if (count) PHX_CHECK(hipMemcpyAsync(data_.get(), o.data_.get(), count * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
}

void PhantomPlaintext::resize(const PhantomContext& ctx, size_t chain_index, hipStream_t s) {
  const auto& cd = ctx.get_context_data(chain_index);
  chain_index_ = chain_index;
  L_ = cd.coeff_modulus_size();
  n_ = ctx.poly_degree();
  data_.allocate(L_ * n_, s);
}

void PhantomPlaintext::resize_ext(const PhantomContext& ctx, size_t chain_index, size_t limbs, hipStream_t s) {
  chain_index_ = chain_index;
  L_ = limbs;
  n_ = ctx.poly_degree();
  data_.allocate(L_ * n_, s);
}

void PhantomPlaintext::from_host(const PhantomContext& ctx, size_t chain_index, const std::vector<uint64_t>& v,
                                 hipStream_t s) {
  resize(ctx, chain_index, s);
  if (v.size() != L_ * n_) throw std::invalid_argument("plaintext data size mismatch");
  PHX_CHECK(hipMemcpyAsync(data_.get(), v.data(), v.size() * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  PHX_CHECK(hipStreamSynchronize(s));
}

}  // namespace phantom
