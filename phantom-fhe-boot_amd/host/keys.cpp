#include "keys.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../csrc/ckks.h"
#include "../csrc/ntt.h"
#include "../csrc/rns.h"
#include "evaluate.h"
#include "numth.h"
#include "serialize.h"

namespace phantom {

void PhantomKSwitchKey::adopt(std::vector<DeviceBuffer<uint64_t>>&& digits, hipStream_t s) {
  digits_ = std::move(digits);
  std::vector<uint64_t*> p;
  for (auto& d : digits_) p.push_back(d.get());
  ptrs_.upload(p, s);
}

void PhantomKSwitchKey::save(const PhantomContext& ctx, std::ostream& os) const {
  const uint64_t n = ctx.poly_degree(), QP = ctx.size_QP();
  std::vector<std::vector<uint64_t>> h(digits_.size(), std::vector<uint64_t>(2 * QP * n));
  std::vector<const uint64_t*> ptrs;
  for (size_t i = 0; i < digits_.size(); ++i) {
    PHX_CHECK(hipMemcpyAsync(h[i].data(), digits_[i].get(), h[i].size() * sizeof(uint64_t), hipMemcpyDeviceToHost,
                             ctx.stream()));
    ptrs.push_back(h[i].data());
  }
  PHX_CHECK(hipStreamSynchronize(ctx.stream()));
  ser::write_kswitch_key(os, n, QP, ptrs);
}

void PhantomKSwitchKey::load(const PhantomContext& ctx, std::istream& is) {
  std::vector<std::vector<uint64_t>> v;
  ser::read_kswitch_key(is, ctx.poly_degree(), ctx.size_QP(), v);
  std::vector<DeviceBuffer<uint64_t>> digits;
  for (const auto& d : v) {
    DeviceBuffer<uint64_t> b;
    b.upload(d, ctx.stream());
    digits.push_back(std::move(b));
  }
  adopt(std::move(digits), ctx.stream());
}

void PhantomGaloisKey::save(const PhantomContext& ctx, std::ostream& os) const {
  // the reference's layout: keys in the order of the context's Galois element list, no elements.
  // Exactly that key set: a missing key or an extra one (which this layout cannot name) throws.
  const std::vector<uint32_t> elts = ctx.key_galois_elts();
  for (uint32_t e : elts)
    if (!has(e))
      throw std::invalid_argument("PhantomGaloisKey lacks the key of Galois element " + std::to_string(e) +
                                  " of the context's list (save_with_elements writes any key set)");
  for (const auto& kv : keys_)
    if (std::find(elts.begin(), elts.end(), kv.first) == elts.end())
      throw std::invalid_argument("PhantomGaloisKey holds the key of Galois element " + std::to_string(kv.first) +
                                  ", outside the context's list, which save() cannot name (use save_with_elements)");
  ser::write_u64(os, elts.size());
  for (uint32_t e : elts) keys_.at(e).save(ctx, os);
}

void PhantomGaloisKey::load(const PhantomContext& ctx, std::istream& is) {
  const std::vector<uint32_t> elts = ctx.key_galois_elts();
  // Files of this engine's earlier builds (round 3 and before) wrote the keys in ascending element
  // order followed by that element list (the save_with_elements layout): one key per distinct
  // element (the default list repeats 5^(N/2) = 5^(-N/2)).  Their trailing list is the context's
  // distinct elements, sorted: bind by it and consume it, instead of binding the keys to the
  // context order (which would attach them to the wrong elements).
  std::vector<uint32_t> distinct = elts;
  std::sort(distinct.begin(), distinct.end());
  distinct.erase(std::unique(distinct.begin(), distinct.end()), distinct.end());
  const uint64_t count = ser::read_u64(is);
  if (count != elts.size() && count != distinct.size())
    throw std::invalid_argument("Galois key count " + std::to_string(count) +
                                " does not match the context's Galois element list (" + std::to_string(elts.size()) + ")");
  std::vector<PhantomKSwitchKey> read(count);
  for (auto& k : read) k.load(ctx, is);
  std::vector<uint32_t> bind = elts;
  bool legacy = false;
  const std::istream::pos_type pos = is.tellg();
  if (pos != std::istream::pos_type(-1) && count == distinct.size()) {
    std::vector<uint32_t> trail(count);
    is.read(reinterpret_cast<char*>(trail.data()), static_cast<std::streamsize>(count * sizeof(uint32_t)));
    legacy = is && trail == distinct && (count != elts.size() || distinct != elts);
    if (legacy) {
      bind = trail;
    } else {
      is.clear();
      is.seekg(pos);  // the reference layout: what follows belongs to the next reader
    }
  }
  if (!legacy && count != elts.size())
    throw std::invalid_argument("Galois key count " + std::to_string(count) +
                                " does not match the context's Galois element list (" + std::to_string(elts.size()) + ")");
  std::map<uint32_t, PhantomKSwitchKey> keys;
  for (size_t i = 0; i < read.size(); ++i) keys[bind[i]] = std::move(read[i]);
  keys_ = std::move(keys);
}

void PhantomGaloisKey::save_with_elements(const PhantomContext& ctx, std::ostream& os) const {
  ser::write_u64(os, keys_.size());
  for (const auto& kv : keys_) kv.second.save(ctx, os);
  for (const auto& kv : keys_) os.write(reinterpret_cast<const char*>(&kv.first), sizeof(uint32_t));
}

void PhantomGaloisKey::load_with_elements(const PhantomContext& ctx, std::istream& is) {
  const uint64_t count = ser::read_u64(is);
  if (count > (uint64_t(1) << 20)) throw std::runtime_error("bad Galois key stream");
  std::vector<PhantomKSwitchKey> ks(count);
  for (auto& k : ks) k.load(ctx, is);
  keys_.clear();
  for (auto& k : ks) {
    uint32_t elt = 0;
    is.read(reinterpret_cast<char*>(&elt), sizeof(elt));
    if (!is) throw std::runtime_error("Galois key stream truncated");
    keys_[elt] = std::move(k);
  }
}

void PhantomSecretKey::save(const PhantomContext& ctx, std::ostream& os) const {
  const uint64_t n = ctx.poly_degree(), QP = ctx.size_QP();
  std::vector<uint64_t> h(QP * n);
  PHX_CHECK(hipMemcpyAsync(h.data(), s_.get(), h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx.stream()));
  PHX_CHECK(hipStreamSynchronize(ctx.stream()));
  ser::write_secret_key(os, 1, n, QP, h.data());
}

PhantomSecretKey PhantomSecretKey::load(const PhantomContext& ctx, std::istream& is) {
  uint64_t power = 0, n = 0, limbs = 0;
  std::vector<uint64_t> v;
  ser::read_secret_key(is, power, n, limbs, v);
  if (power < 1 || n != ctx.poly_degree() || limbs != ctx.size_QP())
    throw std::invalid_argument("secret key does not match the context");
  v.resize(n * limbs);  // s itself; higher powers are recomputed
  PhantomSecretKey k;  // fresh entropy-seeded streams
  hipStream_t s = ctx.stream();
  k.s_.upload(v, s);
  k.init_powers(ctx);
  // ternary coefficients from limb 0 in coefficient form
  DeviceBuffer<uint64_t> c(n, s);
  hip_ok(phx::ntt_inverse(ctx.gpu_rns_tables(), k.s_.get(), c.get(), phx::LimbMap::contiguous(1, 0), nullptr, nullptr, s),
         "sk INTT");
  const std::vector<uint64_t> h = c.download(s);
  const uint64_t q0 = ctx.key_moduli()[0];
  k.coeffs_.resize(n);
  for (size_t i = 0; i < n; ++i) {
    if (h[i] > 1 && h[i] != q0 - 1) throw std::invalid_argument("loaded secret key is not ternary");
    k.coeffs_[i] = h[i] == 0 ? 0 : (h[i] == 1 ? 1 : -1);
  }
  return k;
}

const PhantomKSwitchKey& PhantomGaloisKey::get(uint32_t elt) const {
  auto it = keys_.find(elt);
  if (it == keys_.end()) throw std::invalid_argument("Galois key not present");
  return it->second;
}

uint32_t galois_elt_from_step(int step, size_t n) {
  const uint32_t m = static_cast<uint32_t>(2 * n);
  if (step == 0) return m - 1;
  const bool sign = step < 0;
  uint32_t pos = static_cast<uint32_t>(std::abs(step));
  if (pos >= (n >> 1)) throw std::invalid_argument("step count too large");
  const uint32_t e = sign ? static_cast<uint32_t>(n >> 1) - pos : pos;
  uint64_t g = 1;
  for (uint32_t i = 0; i < e; ++i) g = (g * 5) & (m - 1);
  return static_cast<uint32_t>(g);
}

static std::vector<uint64_t> signed_to_rns(const std::vector<int64_t>& c, const std::vector<uint64_t>& mods) {
  const size_t n = c.size();
  std::vector<uint64_t> out(mods.size() * n);
  for (size_t l = 0; l < mods.size(); ++l)
    for (size_t k = 0; k < n; ++k) {
      const int64_t v = c[k];
      out[l * n + k] = v >= 0 ? static_cast<uint64_t>(v) % mods[l] : mods[l] - (static_cast<uint64_t>(-v) % mods[l]);
      if (out[l * n + k] == mods[l]) out[l * n + k] = 0;
    }
  return out;
}

void sample_uniform_poly(const PhantomContext& ctx, RandomStream& rng, uint64_t* dst, size_t L) {
  hip_ok(phx::sample_uniform(dst, ctx.mod_QP().q, ctx.mod_QP().barrett, ctx.poly_degree(), L, rng.key(),
                             rng.next_draw(), ctx.stream()),
         "sample uniform");
}

void sample_uniform_seeded(const PhantomContext& ctx, const uint8_t* seed, uint64_t* dst, size_t L) {
  hip_ok(phx::sample_uniform_seeded(dst, ctx.mod_QP().q, ctx.mod_QP().barrett, ctx.poly_degree(), L,
                                    phx::salsa_seed(seed), ctx.stream()),
         "sample uniform (seeded)");
}

void sample_error_poly_ntt(const PhantomContext& ctx, RandomStream& rng, uint64_t* dst, size_t L) {
  hip_ok(phx::sample_cbd(dst, ctx.mod_QP().q, ctx.poly_degree(), L, rng.key(), rng.next_draw(), ctx.stream()),
         "sample e");
  hip_ok(phx::ntt_forward(ctx.gpu_rns_tables(), dst, dst, phx::LimbMap::contiguous((int)L, 0), ctx.stream()), "e NTT");
}

void sample_ternary_poly_ntt(const PhantomContext& ctx, RandomStream& rng, uint64_t* dst, size_t L) {
  hip_ok(phx::sample_ternary(dst, ctx.mod_QP().q, ctx.poly_degree(), L, rng.key(), rng.next_draw(), ctx.stream()),
         "sample u");
  hip_ok(phx::ntt_forward(ctx.gpu_rns_tables(), dst, dst, phx::LimbMap::contiguous((int)L, 0), ctx.stream()), "u NTT");
}

PhantomSecretKey::PhantomSecretKey(const PhantomContext& ctx) : PhantomSecretKey(ctx, RandomStream(), false) {}

PhantomSecretKey PhantomSecretKey::for_testing(const PhantomContext& ctx, uint64_t seed) {
  return PhantomSecretKey(ctx, RandomStream::for_testing(seed), true);
}

PhantomSecretKey PhantomSecretKey::from_seed(const PhantomContext& ctx, const uint8_t seed[32]) {
  phx::ChaChaKey k;
  std::memcpy(k.k, seed, sizeof(k.k));
  // the seed fixes the key material only; encryptions draw from fresh OS entropy so that replicas
  // of one key owner never share an (a, e) pair
  return PhantomSecretKey(ctx, RandomStream::from_key(k), false);
}

PhantomSecretKey::PhantomSecretKey(const PhantomContext& ctx, RandomStream rng, bool reproducible_encryption)
    : rng_(rng), reproducible_(reproducible_encryption) {
  const size_t n = ctx.poly_degree();
  // ternary s (sample_ternary_poly): one 64-bit keystream word per coefficient, mod 3
  std::vector<uint64_t> w(n);
  rng_.host_words(w.data(), n);
  coeffs_.resize(n);
  std::vector<int64_t> c(n);
  for (size_t k = 0; k < n; ++k) {
    coeffs_[k] = static_cast<int8_t>(static_cast<int>(w[k] % 3) - 1);
    c[k] = coeffs_[k];
  }
  s_.upload(signed_to_rns(c, ctx.key_moduli()), ctx.stream());
  hip_ok(phx::ntt_forward(ctx.gpu_rns_tables(), s_.get(), s_.get(), phx::LimbMap::contiguous((int)ctx.size_QP(), 0),
                          ctx.stream()),
         "sk NTT");
  init_powers(ctx);
  // for_testing: encryptions follow from the seed too (a child of the key stream); otherwise they
  // come from a stream keyed from the OS CSPRNG, independent of the key seed
  enc_rng_ = reproducible_ ? rng_.derive() : RandomStream();
}

void PhantomSecretKey::init_powers(const PhantomContext& ctx) {
  const size_t n = ctx.poly_degree(), L = ctx.size_QP();
  hipStream_t s = ctx.stream();
  s2_.allocate(L * n, s);
  hip_ok(phx::poly_mul(s_.get(), s_.get(), s2_.get(), ctx.mod_QP(), n, L, s), "sk^2");
  PHX_CHECK(hipStreamSynchronize(s));
}

void PhantomSecretKey::encrypt_zero_raw(const PhantomContext& ctx, RandomStream& rng, uint64_t* c0, uint64_t* c1,
                                        size_t L, const uint64_t* enc_key, const uint8_t* a_seed) const {
  const size_t n = ctx.poly_degree();
  hipStream_t s = ctx.stream();
  DeviceBuffer<uint64_t> e(L * n, s);
  if (a_seed)
    sample_uniform_seeded(ctx, a_seed, c1, L);
  else
    sample_uniform_poly(ctx, rng, c1, L);  // uniform in NTT form is uniform
  sample_error_poly_ntt(ctx, rng, e.get(), L);
  const phx::ModView m = ctx.mod_QP();
  hip_ok(phx::poly_mul_add(c1, enc_key ? enc_key : s_.get(), e.get(), c0, m, n, L, s), "a*s+e");
  hip_ok(phx::poly_negate(c0, c0, m, n, L, s), "-(a*s+e)");
}

PhantomKSwitchKey PhantomSecretKey::make_kswitch_key(const PhantomContext& ctx, const uint64_t* new_key,
                                                    const uint64_t* enc_key) {
  if (!enc_key) enc_key = s_.get();
  const size_t n = ctx.poly_degree(), QP = ctx.size_QP(), Q = ctx.size_Q(), alpha = ctx.size_P();
  hipStream_t s = ctx.stream();
  const size_t dnum = (Q + alpha - 1) / alpha;
  const RnsTool& rt = ctx.get_context_data(1).gpu_rns_tool();
  std::vector<DeviceBuffer<uint64_t>> digits;
  DeviceBuffer<uint64_t> tmp(QP * n, s);
  const phx::ModView mqp = ctx.mod_QP();
  for (size_t d = 0; d < dnum; ++d) {
    DeviceBuffer<uint64_t> key(2 * QP * n, s);
    uint64_t* b = key.get();
    uint64_t* a = key.get() + QP * n;
    encrypt_zero_raw(ctx, rng_, b, a, QP, enc_key);
    // + P * new_key on this digit's primes (multiply_temp_mod_and_add_rns_poly)
    const size_t l0 = d * alpha, l1 = std::min(Q, l0 + alpha);
    phx::ModView sub{mqp.q + l0, mqp.barrett + 2 * l0};
    hip_ok(phx::poly_mul_scalar(new_key + l0 * n, rt.bigP_mod_q() + l0, rt.bigP_mod_q_shoup() + l0, tmp.get(), sub, n,
                                l1 - l0, s),
           "P*s'");
    hip_ok(phx::poly_add(b + l0 * n, tmp.get(), b + l0 * n, sub, n, l1 - l0, s), "b += P*s'");
    digits.push_back(std::move(key));
  }
  PhantomKSwitchKey k;
  k.adopt(std::move(digits), s);
  PHX_CHECK(hipStreamSynchronize(s));
  return k;
}

PhantomRelinKey PhantomSecretKey::gen_relinkey(const PhantomContext& ctx) {
  PhantomKSwitchKey k = make_kswitch_key(ctx, s2_.get());
  PhantomRelinKey r;
  static_cast<PhantomKSwitchKey&>(r) = std::move(k);
  return r;
}

PhantomGaloisKey PhantomSecretKey::create_galois_keys(const PhantomContext& ctx, const std::vector<uint32_t>& elts) {
  const size_t n = ctx.poly_degree(), QP = ctx.size_QP();
  hipStream_t s = ctx.stream();
  PhantomGaloisKey gk;
  // s(X^k) in NTT form = permutation of NTT(s)
  std::vector<uint32_t> perm(n);
  const int logn = arith::log2_exact(n);
  DeviceBuffer<uint32_t> d_perm;
  DeviceBuffer<uint64_t> rot(QP * n, s);
  for (uint32_t k : elts) {
    for (uint32_t j = 0; j < n; ++j) {
      const uint64_t idx = ((2ull * j + 1) * k) % (2ull * n);
      perm[arith::reverse_bits(j, logn)] = arith::reverse_bits(static_cast<uint32_t>(idx >> 1), logn);
    }
    d_perm.upload(perm, s);
    hip_ok(phx::galois_ntt(s_.get(), rot.get(), d_perm.get(), n, QP, s), "rotate sk");
    gk.set(k, make_kswitch_key(ctx, rot.get()));
  }
  return gk;
}

PhantomGaloisKey PhantomSecretKey::create_galois_keys(const PhantomContext& ctx) {
  return create_galois_keys(ctx, ctx.key_galois_elts());
}

PhantomGaloisKey PhantomSecretKey::EvalRotateKeyGen(const PhantomContext& ctx, const std::vector<int32_t>& index_list) {
  const size_t n = ctx.poly_degree();
  std::vector<uint32_t> elts;
  for (int32_t i : index_list) {
    // FindAutomorphismIndex2nComplex (src/util.cu:908-935)
    const int64_t slots = static_cast<int64_t>(n / 2);
    int64_t r = i % slots;
    if (r < 0) r += slots;
    uint64_t g = 1;
    for (int64_t e = 0; e < r; ++e) g = g * 5 % (2 * n);
    elts.push_back(static_cast<uint32_t>(g));
  }
  elts.push_back(static_cast<uint32_t>(2 * n - 1));
  std::sort(elts.begin(), elts.end());
  elts.erase(std::unique(elts.begin(), elts.end()), elts.end());
  return create_galois_keys_fused(ctx, elts);
}

PhantomGaloisKey PhantomSecretKey::create_galois_keys_fused(const PhantomContext& ctx,
                                                           const std::vector<uint32_t>& elts) {
  const size_t n = ctx.poly_degree(), QP = ctx.size_QP();
  hipStream_t s = ctx.stream();
  PhantomGaloisKey gk;
  const int logn = arith::log2_exact(n);
  const uint64_t m = 2 * n;
  std::vector<uint32_t> perm(n);
  DeviceBuffer<uint32_t> d_perm;
  DeviceBuffer<uint64_t> rot(QP * n, s);
  for (uint32_t k : elts) {
    // encryption secret s(X^(k^-1)): the hoisted rotation applies X -> X^k after the key switch
    const uint32_t kinv = static_cast<uint32_t>(arith::inv_mod(k, m));
    for (uint32_t j = 0; j < n; ++j) {
      const uint64_t idx = ((2ull * j + 1) * kinv) % m;
      perm[arith::reverse_bits(j, logn)] = arith::reverse_bits(static_cast<uint32_t>(idx >> 1), logn);
    }
    d_perm.upload(perm, s);
    hip_ok(phx::galois_ntt(s_.get(), rot.get(), d_perm.get(), n, QP, s), "rotate sk");
    gk.set(k, make_kswitch_key(ctx, s_.get(), rot.get()));
  }
  return gk;
}

void PhantomSecretKey::encrypt_symmetric(const PhantomContext& ctx, const PhantomPlaintext& plain,
                                         PhantomCiphertext& out) const {
  const size_t n = ctx.poly_degree(), ci = plain.chain_index();
  if (ci < 1 || ci >= ctx.total_parm_size()) throw std::invalid_argument("invalid plaintext chain index");
  const size_t L = ctx.get_context_data(ci).coeff_modulus_size();
  hipStream_t s = ctx.stream();
  out.resize(ctx, ci, 2, s, false);
  out.set_ntt_form(true);
  out.set_scale(plain.scale());
  out.set_correction_factor(1);
  out.SetNoiseScaleDeg(1);
  out.set_asymmetric(false);
  // a public seed for a (save_symmetric writes it instead of c1): one draw of this key's stream
  std::vector<uint8_t> seed(PhantomCiphertext::kSeedBytes);
  enc_rng_.host_words(reinterpret_cast<uint64_t*>(seed.data()), seed.size() / sizeof(uint64_t));
  encrypt_zero_raw(ctx, enc_rng_, out.data(), out.data() + L * n, L, nullptr, seed.data());
  hip_ok(phx::poly_add(out.data(), plain.data(), out.data(), ctx.mod_QP(), n, L, s), "m - (a s + e)");
  out.set_seed(std::move(seed), s);  // synchronises s
}

void PhantomSecretKey::decrypt(const PhantomContext& ctx, const PhantomCiphertext& ct, PhantomPlaintext& out) const {
  const size_t n = ctx.poly_degree(), L = ct.coeff_modulus_size();
  if (ct.size() < 2 || ct.size() > 3) throw std::invalid_argument("unsupported ciphertext size");
  hipStream_t s = ctx.stream();
  out.resize(ctx, ct.chain_index(), s);
  out.set_scale(ct.scale());
  const phx::ModView m = ctx.mod_QP();
  // out = c0 + c1 s (+ c2 s^2)
  hip_ok(phx::poly_mul_add(ct.data() + L * n, s_.get(), ct.data(), out.data(), m, n, L, s), "c0 + c1 s");
  if (ct.size() == 3)
    hip_ok(phx::poly_mul_add(ct.data() + 2 * L * n, s2_.get(), out.data(), out.data(), m, n, L, s), "+ c2 s^2");
  PHX_CHECK(hipStreamSynchronize(s));
}

PhantomPublicKey PhantomSecretKey::gen_publickey(const PhantomContext& ctx) const {
  PhantomPublicKey pk;
  const size_t n = ctx.poly_degree(), QP = ctx.size_QP();
  pk.pk_.resize(ctx, 0, 2, ctx.stream(), false);
  pk.pk_.set_ntt_form(true);
  encrypt_zero_raw(ctx, rng_, pk.pk_.data(), pk.pk_.data() + QP * n, QP);  // key material
  // the encryptor's own stream: fresh entropy, or derived for reproducible tests
  pk.rng_ = reproducible_ ? enc_rng_.derive() : RandomStream();
  PHX_CHECK(hipStreamSynchronize(ctx.stream()));
  return pk;
}

void PhantomPublicKey::encrypt_zero_raw(const PhantomContext& ctx, PhantomCiphertext& out, size_t ci) {
  if (pk_.size() != 2 || pk_.coeff_modulus_size() != ctx.size_QP())
    throw std::invalid_argument("PhantomPublicKey has not been generated");
  if (ci < 1 || ci >= ctx.total_parm_size()) throw std::invalid_argument("invalid chain index");
  const size_t n = ctx.poly_degree(), QP = ctx.size_QP();
  hipStream_t s = ctx.stream();
  const phx::ModView m = ctx.mod_QP();
  // (c0, c1) = (pk0 u + e0, pk1 u + e1) over Q u P (encrypt_zero_asymmetric_internal_internal,
  // src/secretkey.cu:12-86)
  DeviceBuffer<uint64_t> u(QP * n, s), e(QP * n, s), cx(2 * QP * n, s);
  sample_ternary_poly_ntt(ctx, rng_, u.get(), QP);
  for (size_t i = 0; i < 2; ++i) {
    sample_error_poly_ntt(ctx, rng_, e.get(), QP);
    hip_ok(phx::poly_mul_add(u.get(), pk_.data() + i * QP * n, e.get(), cx.get() + i * QP * n, m, n, QP, s), "pk u + e");
  }
  // divide by P: the moddown of encrypt_zero_asymmetric_internal (src/secretkey.cu:113-121)
  PhantomCiphertext z;
  z.resize(ctx, 1, 2, s, false);
  ctx.get_context_data(1).gpu_rns_tool().moddown_add(z.data(), cx.get(), false, ctx.gpu_rns_tables(), s, 2);
  z.set_ntt_form(true);
  // the reference moves between levels by modulus switching; dropping the leading limbs keeps an
  // encryption of zero (its noise is far below the dropped primes)
  out = ci > 1 ? mod_switch_to(ctx, z, ci) : std::move(z);
  out.set_scale(1.0);
  out.set_correction_factor(1);
  out.SetNoiseScaleDeg(1);
  out.set_asymmetric(true);
}

PhantomCiphertext PhantomPublicKey::encrypt_zero_asymmetric(const PhantomContext& ctx) {
  PhantomCiphertext c;
  encrypt_zero_raw(ctx, c, 1);
  PHX_CHECK(hipStreamSynchronize(ctx.stream()));
  return c;
}

void PhantomPublicKey::encrypt_asymmetric(const PhantomContext& ctx, const PhantomPlaintext& plain,
                                          PhantomCiphertext& out) {
  encrypt_zero_raw(ctx, out, plain.chain_index());
  if (out.coeff_modulus_size() != plain.coeff_modulus_size())
    throw std::invalid_argument("plaintext does not match its chain index");
  // c0 = c0 + plaintext
  hip_ok(phx::poly_add(out.data(), plain.data(), out.data(), ctx.mod_QP(), ctx.poly_degree(), out.coeff_modulus_size(),
                       ctx.stream()),
         "c0 + m");
  out.set_scale(plain.scale());
  PHX_CHECK(hipStreamSynchronize(ctx.stream()));
}

void PhantomPublicKey::save(std::ostream& os) const {
  if (pk_.size() != 2) throw std::invalid_argument("PhantomPublicKey has not been generated");
  pk_.save(os);
}

void PhantomPublicKey::load(const PhantomContext& ctx, std::istream& is) {
  PhantomCiphertext k;
  k.load(ctx, is);
  if (k.size() != 2 || k.chain_index() != 0 || k.coeff_modulus_size() != ctx.size_QP())
    throw std::invalid_argument("public key does not match the context");
  pk_ = std::move(k);
  rng_ = RandomStream();
}

}  // namespace phantom
