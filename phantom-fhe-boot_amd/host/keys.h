// keys.h — PhantomSecretKey / PhantomPublicKey / PhantomRelinKey / PhantomGaloisKey
// (include/secretkey.h).
//
// Key generation and encryption are the harness around the accelerated path, but
// they are real cryptography: every draw comes from a ChaCha20 stream (host/random.h) keyed from
// the operating system's CSPRNG, as the reference seeds Salsa20 from std::random_device
// (include/prng.cuh:13-24).  Reproducible keys exist only through the explicitly named
// PhantomSecretKey::for_testing.  Key formats match the reference:
//   * public key: (-(a s + e), a) at the key level Q u P, NTT form (gen_publickey,
//     src/secretkey.cu:493-504);
//   * key-switching key: dnum digits of [2][size_QP][n] NTT-form polynomials (b_i, a_i) with
//     b_i = -(a_i s + e_i) + P * s' on digit i's primes (src/secretkey.cu:362-406).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <istream>
#include <map>
#include <memory>
#include <ostream>
#include <vector>

#include "buffer.h"
#include "ciphertext.h"
#include "context.h"
#include "random.h"

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

 private:
  std::vector<DeviceBuffer<uint64_t>> digits_;
  DeviceBuffer<uint64_t*> ptrs_;
};

class PhantomRelinKey : public PhantomKSwitchKey {};

class PhantomGaloisKey {
 public:
  const PhantomKSwitchKey& get(uint32_t galois_elt) const;
  bool has(uint32_t galois_elt) const { return keys_.count(galois_elt) != 0; }
  void set(uint32_t galois_elt, PhantomKSwitchKey&& k) { keys_[galois_elt] = std::move(k); }
  // move every key of `other` in (replacing keys of the same element)
  void merge(PhantomGaloisKey&& other) {
    for (auto& kv : other.keys_) keys_[kv.first] = std::move(kv.second);
    other.keys_.clear();
  }
  // PhantomGaloisKey::save / load (include/secretkey.h:195-220), the reference's bytes: the
  // number of keys, then each as a relin key, in the order of the context's Galois element list
  // (PhantomContext::key_galois_elts, the reference's key_galois_tool_ order), which is how the
  // reference indexes them.  save throws std::invalid_argument if a key of that list is missing;
  // load requires the stream's count to be the list's length.
  void save(const PhantomContext& ctx, std::ostream& os) const;
  void load(const PhantomContext& ctx, std::istream& is);
  // any key set (e.g. the fused bootstrap keys, which the reference never serializes): the same
  // records followed by the elements (uint32_t each, ascending)
  void save_with_elements(const PhantomContext& ctx, std::ostream& os) const;
  void load_with_elements(const PhantomContext& ctx, std::istream& is);
  size_t size() const { return keys_.size(); }

 private:
  std::map<uint32_t, PhantomKSwitchKey> keys_;
};

// PhantomPublicKey (include/secretkey.h:17-101)
class PhantomPublicKey {
 public:
  PhantomPublicKey() = default;
  PhantomPublicKey(const PhantomPublicKey&) = delete;
  PhantomPublicKey& operator=(const PhantomPublicKey&) = delete;
  PhantomPublicKey(PhantomPublicKey&&) = default;
  PhantomPublicKey& operator=(PhantomPublicKey&&) = default;

  // encrypt_asymmetric (src/secretkey.cu:130-185): (pk0 u + e0, pk1 u + e1) over Q u P with u
  // ternary and e0, e1 centered binomial, divided by P (moddown) to Q, dropped to the
  // plaintext's level, then m added to c0.  The ciphertext takes the plaintext's scale.
  void encrypt_asymmetric(const PhantomContext& ctx, const PhantomPlaintext& plain, PhantomCiphertext& out);
  PhantomCiphertext encrypt_asymmetric(const PhantomContext& ctx, const PhantomPlaintext& plain) {
    PhantomCiphertext c;
    encrypt_asymmetric(ctx, plain, c);
    return c;
  }
  // encrypt_zero_asymmetric (include/secretkey.h:78-84): an encryption of 0 at chain index 1
  PhantomCiphertext encrypt_zero_asymmetric(const PhantomContext& ctx);

  // save / load (include/secretkey.h:86-101): the key-level ciphertext pk_.  A loaded key
  // encrypts with a fresh entropy-seeded stream.
  void save(std::ostream& os) const;
  void load(const PhantomContext& ctx, std::istream& is);
  const PhantomCiphertext& key() const { return pk_; }

 private:
  friend class PhantomSecretKey;
  void encrypt_zero_raw(const PhantomContext& ctx, PhantomCiphertext& out, size_t chain_index);
  PhantomCiphertext pk_;
  RandomStream rng_;
};

class PhantomSecretKey {
 public:
  // PhantomSecretKey(context) (src/secretkey.cu:470-491): ternary s from a fresh entropy-seeded
  // ChaCha20 stream
  explicit PhantomSecretKey(const PhantomContext& ctx);
  // reproducible key for tests only: every draw (s, errors, uniform halves) follows from `seed`
  static PhantomSecretKey for_testing(const PhantomContext& ctx, uint64_t seed);
  // key material (s, public key, relin / Galois keys) derived from a 256-bit secret seed: replicas
  // of one key owner (the ranks of a multi-GPU job) regenerate identical keys from a shared seed
  // instead of moving them.  Encryptions still draw from fresh OS entropy, so two replicas' k-th
  // encryptions share no randomness.
  static PhantomSecretKey from_seed(const PhantomContext& ctx, const uint8_t seed[32]);
  PhantomSecretKey(PhantomSecretKey&&) = default;
  PhantomSecretKey& operator=(PhantomSecretKey&&) = default;

  // save / load (include/secretkey.h:405-440): sk_max_power (1), n, size_QP, then s in NTT
  // form.  A loaded key draws its later randomness from a fresh entropy-seeded stream.
  void save(const PhantomContext& ctx, std::ostream& os) const;
  static PhantomSecretKey load(const PhantomContext& ctx, std::istream& is);
  // s in NTT form over the full Q u P chain, [size_QP][n]
  const uint64_t* secret_key_array() const { return s_.get(); }
  const std::vector<int8_t>& coefficients() const { return coeffs_; }

  // gen_publickey (src/secretkey.cu:493-504): a symmetric encryption of zero at the key level
  PhantomPublicKey gen_publickey(const PhantomContext& ctx) const;
  PhantomRelinKey gen_relinkey(const PhantomContext& ctx);
  PhantomGaloisKey create_galois_keys(const PhantomContext& ctx, const std::vector<uint32_t>& galois_elts);
  // create_galois_keys(context) (src/secretkey.cu:532-572): keys for the context's Galois element
  // list (PhantomContext::key_galois_elts)
  PhantomGaloisKey create_galois_keys(const PhantomContext& ctx);
  // keys for hoisted rotations (the reference's PhantomGaloisKeyFused): the key for element k
  // switches from s to s(X^(k^-1)), so the automorphism can be applied after the inner product
  // of the shared modup digits (EvalFastRotationExt, src/evaluate.cu:3656-3748)
  PhantomGaloisKey create_galois_keys_fused(const PhantomContext& ctx, const std::vector<uint32_t>& galois_elts);
  // EvalRotateKeyGen / EvalAtIndexKeyGen (include/secretkey.h:453-457, src/secretkey.cu:956-1022):
  // fused keys for the slot rotations in `index_list` plus the conjugation key
  PhantomGaloisKey EvalRotateKeyGen(const PhantomContext& ctx, const std::vector<int32_t>& index_list);
  PhantomGaloisKey EvalAtIndexKeyGen(const PhantomContext& ctx, const std::vector<int32_t>& index_list) {
    return EvalRotateKeyGen(ctx, index_list);
  }

  // symmetric encryption of an NTT-form plaintext at its chain index (src/secretkey.cu:576-644)
  void encrypt_symmetric(const PhantomContext& ctx, const PhantomPlaintext& plain, PhantomCiphertext& out) const;
  PhantomCiphertext encrypt_symmetric(const PhantomContext& ctx, const PhantomPlaintext& plain) const {
    PhantomCiphertext c;
    encrypt_symmetric(ctx, plain, c);
    return c;
  }
  // decryption c0 + c1 s (+ c2 s^2) in NTT form (ckks_decrypt, src/secretkey.cu:646-682, 806-830)
  void decrypt(const PhantomContext& ctx, const PhantomCiphertext& ct, PhantomPlaintext& out) const;
  PhantomPlaintext decrypt(const PhantomContext& ctx, const PhantomCiphertext& ct) const {
    PhantomPlaintext p;
    decrypt(ctx, ct, p);
    return p;
  }

  // kswitch key for new_key (NTT form over QP) -> enc_key (default s) (generate_one_kswitch_key)
  PhantomKSwitchKey make_kswitch_key(const PhantomContext& ctx, const uint64_t* new_key,
                                     const uint64_t* enc_key = nullptr);

 private:
  PhantomSecretKey(const PhantomContext& ctx, RandomStream rng, bool reproducible_encryption);
  PhantomSecretKey() = default;
  void init_powers(const PhantomContext& ctx);
  // symmetric encryption of zero over the first L limbs of Q u P under enc_key (default s):
  // (-(a s + e), a), NTT form
  // a_seed: take a from sample_uniform_seeded(a_seed) instead of this key's stream
  void encrypt_zero_raw(const PhantomContext& ctx, RandomStream& rng, uint64_t* c0, uint64_t* c1, size_t L,
                        const uint64_t* enc_key = nullptr, const uint8_t* a_seed = nullptr) const;
  // rng_: key material; enc_rng_: encryption draws (OS entropy unless for_testing)
  mutable RandomStream rng_, enc_rng_;
  bool reproducible_ = false;
  std::vector<int8_t> coeffs_;
  DeviceBuffer<uint64_t> s_, s2_;
};

// the reference's name for the fused (hoisted-rotation) key set (include/secretkey.h:226-262)
using PhantomGaloisKeyFused = PhantomGaloisKey;

// galois element for a slot rotation by `step` (FindAutomorphismIndex2nComplex, src/util.cu:908-935)
uint32_t galois_elt_from_step(int step, size_t n);

// draws of a ChaCha20 stream into device polynomials over the first L limbs of Q u P
// (the reference's sample_uniform_poly / sample_error_poly / sample_ternary_poly, src/prng.cu)
void sample_uniform_poly(const PhantomContext& ctx, RandomStream& rng, uint64_t* dst, size_t L);
// uniform `a` of a seed-compressed symmetric ciphertext from its public 64-byte seed: the
// reference's Salsa20 expansion (sample_uniform_poly, src/prng.cu:164-197; csrc/salsa.h), so the
// compressed form interchanges with the reference's save_symmetric / load_symmetric
void sample_uniform_seeded(const PhantomContext& ctx, const uint8_t* seed, uint64_t* dst, size_t L);
// centered-binomial error, returned in NTT form
void sample_error_poly_ntt(const PhantomContext& ctx, RandomStream& rng, uint64_t* dst, size_t L);
// ternary polynomial, returned in NTT form
void sample_ternary_poly_ntt(const PhantomContext& ctx, RandomStream& rng, uint64_t* dst, size_t L);

}  // namespace phantom
