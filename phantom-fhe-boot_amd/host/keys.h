// keys.h — PhantomSecretKey / PhantomRelinKey / PhantomGaloisKey (include/secretkey.h).
//
// Key generation and encryption are the test harness, not the accelerated path:
// randomness comes from a caller-supplied seed (std::mt19937_64) instead of the reference's
// std::random_device-seeded Salsa20, so keys and ciphertexts are reproducible.  Key formats
// match the reference: a key-switching key is dnum digits of [2][size_QP][n] NTT-form
// polynomials (b_i, a_i) with b_i = -(a_i s + e_i) + P * s' on digit i's primes
// (src/secretkey.cu:362-406, multiply_temp_mod_and_add_rns_poly).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <istream>
#include <map>
#include <memory>
#include <ostream>
#include <vector>

#include "buffer.h"
#include "../csrc/rns.h"
#include "ciphertext.h"
#include "context.h"

namespace phantom {

class PhantomSecretKey;

// a set of key-switching digits plus the device pointer array the inner product reads
class PhantomKSwitchKey {
 public:
  size_t dnum() const { return digits_.size(); }
  const uint64_t* const* public_keys_ptr() const { return ptrs_.get(); }
  const uint64_t* digit(size_t i) const { return digits_.at(i).get(); }
  void adopt(std::vector<DeviceBuffer<uint64_t>>&& digits, hipStream_t s);
  // PhantomRelinKey::save / load (include/secretkey.h:130-157): dnum, then every digit as a
  // 2-polynomial key-level ciphertext (chain index 0, size_QP limbs, NTT form)
  void save(const PhantomContext& ctx, std::ostream& os) const;
  void load(const PhantomContext& ctx, std::istream& is);
  // Per-digit (seed, stream) of the uniform half when this library sampled it: the inner
  // product then regenerates that half instead of reading it (phx::KsSeeds).  Null for loaded
  // or adopted keys, and when PHX_KS_REGEN=0.
  const phx::KsSeeds* seeds() const;
  void set_seeds(const phx::KsSeeds& s) { seeds_ = s; has_seeds_ = true; }

 private:
  std::vector<DeviceBuffer<uint64_t>> digits_;
  DeviceBuffer<uint64_t*> ptrs_;
  phx::KsSeeds seeds_;
  bool has_seeds_ = false;
};

class PhantomRelinKey : public PhantomKSwitchKey {};

class PhantomGaloisKey {
 public:
  const PhantomKSwitchKey& get(uint32_t galois_elt) const;
  bool has(uint32_t galois_elt) const { return keys_.count(galois_elt) != 0; }
  void set(uint32_t galois_elt, PhantomKSwitchKey&& k) { keys_[galois_elt] = std::move(k); }
  // PhantomGaloisKey::save / load (include/secretkey.h:195-220): the number of keys, then each
  // as a relin key.  The reference indexes keys by position in its galois_elts list; here the
  // element itself is the key, so the count is followed by the elements (uint32_t each, in
  // ascending order) after the keys
  void save(const PhantomContext& ctx, std::ostream& os) const;
  void load(const PhantomContext& ctx, std::istream& is);

 private:
  std::map<uint32_t, PhantomKSwitchKey> keys_;
};

class PhantomSecretKey {
 public:
  PhantomSecretKey(const PhantomContext& ctx, uint64_t seed);
  // save / load (include/secretkey.h:405-440): sk_max_power (1), n, size_QP, then s in NTT
  // form.  A loaded key samples its later randomness from `seed`.
  void save(const PhantomContext& ctx, std::ostream& os) const;
  static PhantomSecretKey load(const PhantomContext& ctx, std::istream& is, uint64_t seed);
  // s in NTT form over the full Q u P chain, [size_QP][n]
  const uint64_t* secret_key_array() const { return s_.get(); }
  const std::vector<int8_t>& coefficients() const { return coeffs_; }

  PhantomRelinKey gen_relinkey(const PhantomContext& ctx);
  PhantomGaloisKey create_galois_keys(const PhantomContext& ctx, const std::vector<uint32_t>& galois_elts);
  // keys for hoisted rotations (the reference's PhantomGaloisKeyFused): the key for element k
  // switches from s to s(X^(k^-1)), so the automorphism can be applied after the inner product
  // of the shared modup digits (EvalFastRotationExt, src/evaluate.cu:3656-3748)
  PhantomGaloisKey create_galois_keys_fused(const PhantomContext& ctx, const std::vector<uint32_t>& galois_elts);

  // symmetric encryption of an NTT-form plaintext at `chain_index` (src/secretkey.cu:576-644)
  void encrypt_symmetric(const PhantomContext& ctx, const PhantomPlaintext& plain, PhantomCiphertext& out);
  // decryption c0 + c1 s (+ c2 s^2) in NTT form (ckks_decrypt, src/secretkey.cu:646-682)
  void decrypt(const PhantomContext& ctx, const PhantomCiphertext& ct, PhantomPlaintext& out);

  // kswitch key for new_key (NTT form over QP) -> enc_key (default s) (generate_one_kswitch_key)
  PhantomKSwitchKey make_kswitch_key(const PhantomContext& ctx, const uint64_t* new_key,
                                     const uint64_t* enc_key = nullptr);

 private:
  PhantomSecretKey() = default;
  void sample_uniform(const PhantomContext& ctx, uint64_t* dst, size_t L);
  void sample_error(const PhantomContext& ctx, uint64_t* dst, size_t L);  // NTT form
  uint64_t next();
  uint64_t seed_state_ = 0;
  uint64_t draws_ = 0;  // counter of device sampling draws
  std::vector<int8_t> coeffs_;
  DeviceBuffer<uint64_t> s_, s2_;
};

// galois element for a slot rotation by `step` (FindAutomorphismIndex2nComplex, src/util.cu:908-935)
uint32_t galois_elt_from_step(int step, size_t n);

}  // namespace phantom
