#include "keys.h"

#include <cstdlib>

#include <cmath>
#include <random>
#include <stdexcept>

#include "../csrc/ckks.h"
#include "../csrc/ntt.h"
#include "../csrc/rns.h"
#include "numth.h"
#include "serialize.h"

namespace phantom {

static void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw hip_error(e, what);
}

const phx::KsSeeds* PhantomKSwitchKey::seeds() const {
  static const bool regen = [] {
    const char* e = std::getenv("PHX_KS_REGEN");
    return !(e && e[0] == '0');
  }();
  return (has_seeds_ && regen) ? &seeds_ : nullptr;
}

void PhantomKSwitchKey::adopt(std::vector<DeviceBuffer<uint64_t>>&& digits, hipStream_t s) {
  has_seeds_ = false;
  digits_ = std::move(digits);
  std::vector<uint64_t*> p;
  for (auto& d : digits_) p.push_back(d.get());
  ptrs_.upload(p, s);
}

void PhantomKSwitchKey::save(const PhantomContext& ctx, std::ostream& os) const {
  const uint64_t dnum = digits_.size(), n = ctx.poly_degree(), QP = ctx.size_QP();
  os.write(reinterpret_cast<const char*>(&dnum), sizeof(dnum));
  std::vector<uint64_t> h(2 * QP * n);
  for (const auto& d : digits_) {
    PHX_CHECK(hipMemcpyAsync(h.data(), d.get(), h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx.stream()));
    PHX_CHECK(hipStreamSynchronize(ctx.stream()));
    ser::CiphertextHeader hd;
    hd.chain_index = 0;
    hd.size = 2;
    hd.poly_modulus_degree = n;
    hd.coeff_modulus_size = QP;
    ser::write_ciphertext(os, hd, h.data());
  }
}

void PhantomKSwitchKey::load(const PhantomContext& ctx, std::istream& is) {
  uint64_t dnum = 0;
  is.read(reinterpret_cast<char*>(&dnum), sizeof(dnum));
  if (!is || dnum > 64) throw std::runtime_error("bad key-switching key stream");
  const uint64_t n = ctx.poly_degree(), QP = ctx.size_QP();
  std::vector<DeviceBuffer<uint64_t>> digits;
  for (uint64_t i = 0; i < dnum; ++i) {
    ser::CiphertextHeader hd;
    std::vector<uint64_t> v;
    ser::read_ciphertext(is, hd, v);
    if (hd.size != 2 || hd.poly_modulus_degree != n || hd.coeff_modulus_size != QP)
      throw std::invalid_argument("key-switching key does not match the context");
    DeviceBuffer<uint64_t> d;
    d.upload(v, ctx.stream());
    digits.push_back(std::move(d));
  }
  adopt(std::move(digits), ctx.stream());
}

void PhantomGaloisKey::save(const PhantomContext& ctx, std::ostream& os) const {
  const uint64_t count = keys_.size();
  os.write(reinterpret_cast<const char*>(&count), sizeof(count));
  for (const auto& kv : keys_) kv.second.save(ctx, os);
  for (const auto& kv : keys_) os.write(reinterpret_cast<const char*>(&kv.first), sizeof(uint32_t));
}

void PhantomGaloisKey::load(const PhantomContext& ctx, std::istream& is) {
  uint64_t count = 0;
  is.read(reinterpret_cast<char*>(&count), sizeof(count));
  if (!is || count > (uint64_t(1) << 20)) throw std::runtime_error("bad Galois key stream");
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

PhantomSecretKey PhantomSecretKey::load(const PhantomContext& ctx, std::istream& is, uint64_t seed) {
  uint64_t power = 0, n = 0, limbs = 0;
  std::vector<uint64_t> v;
  ser::read_secret_key(is, power, n, limbs, v);
  if (power < 1 || n != ctx.poly_degree() || limbs != ctx.size_QP())
    throw std::invalid_argument("secret key does not match the context");
  v.resize(n * limbs);  // s itself; higher powers are recomputed
  PhantomSecretKey k;
  k.seed_state_ = seed;
  hipStream_t s = ctx.stream();
  k.s_.upload(v, s);
  k.s2_.allocate(limbs * n, s);
  hip_ok(phx::poly_mul(k.s_.get(), k.s_.get(), k.s2_.get(), ctx.mod_QP(), n, limbs, s), "sk^2");
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

uint64_t PhantomSecretKey::next() {
  // splitmix64 stream over the seed
  uint64_t z = (seed_state_ += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
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

PhantomSecretKey::PhantomSecretKey(const PhantomContext& ctx, uint64_t seed) : seed_state_(seed) {
  const size_t n = ctx.poly_degree(), L = ctx.size_QP();
  hipStream_t s = ctx.stream();
  coeffs_.resize(n);
  std::vector<int64_t> c(n);
  for (size_t k = 0; k < n; ++k) {
    coeffs_[k] = static_cast<int8_t>(static_cast<int>(next() % 3) - 1);  // ternary (sample_ternary_poly)
    c[k] = coeffs_[k];
  }
  s_.upload(signed_to_rns(c, ctx.key_moduli()), s);
  hip_ok(phx::ntt_forward(ctx.gpu_rns_tables(), s_.get(), s_.get(), phx::LimbMap::contiguous((int)L, 0), s), "sk NTT");
  s2_.allocate(L * n, s);
  hip_ok(phx::poly_mul(s_.get(), s_.get(), s2_.get(), ctx.mod_QP(), n, L, s), "sk^2");
  PHX_CHECK(hipStreamSynchronize(s));
}

// Randomness comes from device-side counter-based generators keyed by (seed, draw counter), so
// key generation for hundreds of rotation keys stays on the GPU (the reference samples on the
// GPU as well: src/prng.cu, sample_uniform_poly / sample_error_poly in src/secretkey.cu).
void PhantomSecretKey::sample_uniform(const PhantomContext& ctx, uint64_t* dst, size_t L) {
  hip_ok(phx::sample_uniform(dst, ctx.mod_QP().q, ctx.mod_QP().barrett, ctx.poly_degree(), L, seed_state_, draws_++,
                             ctx.stream()),
         "sample uniform");
}

void PhantomSecretKey::sample_error(const PhantomContext& ctx, uint64_t* dst, size_t L) {
  // centered binomial, sigma ~ 3.2 (sample_error_poly uses a CBD as well), then NTT
  hip_ok(phx::sample_cbd(dst, ctx.mod_QP().q, ctx.poly_degree(), L, seed_state_, draws_++, ctx.stream()), "sample e");
  hip_ok(phx::ntt_forward(ctx.gpu_rns_tables(), dst, dst, phx::LimbMap::contiguous((int)L, 0), ctx.stream()), "e NTT");
}

PhantomKSwitchKey PhantomSecretKey::make_kswitch_key(const PhantomContext& ctx, const uint64_t* new_key,
                                                    const uint64_t* enc_key) {
  if (!enc_key) enc_key = s_.get();
  const size_t n = ctx.poly_degree(), QP = ctx.size_QP(), Q = ctx.size_Q(), alpha = ctx.size_P();
  hipStream_t s = ctx.stream();
  const size_t dnum = (Q + alpha - 1) / alpha;
  const RnsTool& rt = ctx.get_context_data(1).gpu_rns_tool();
  phx::KsSeeds seeds;
  std::vector<DeviceBuffer<uint64_t>> digits;
  DeviceBuffer<uint64_t> e(QP * n, s), tmp(QP * n, s);
  const phx::ModView mqp = ctx.mod_QP();
  for (size_t d = 0; d < dnum; ++d) {
    DeviceBuffer<uint64_t> key(2 * QP * n, s);
    uint64_t* b = key.get();
    uint64_t* a = key.get() + QP * n;
    if (d < static_cast<size_t>(phx::kMaxKsDigits)) {
      seeds.seed[d] = seed_state_;  // the stream sample_uniform draws from next
      seeds.sid[d] = draws_;
    }
    sample_uniform(ctx, a, QP);   // uniform in NTT form is uniform
    sample_error(ctx, e.get(), QP);
    hip_ok(phx::poly_mul_add(a, enc_key, e.get(), tmp.get(), mqp, n, QP, s), "a*s+e");
    hip_ok(phx::poly_negate(tmp.get(), b, mqp, n, QP, s), "-(a*s+e)");
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
  if (dnum <= static_cast<size_t>(phx::kMaxKsDigits)) k.set_seeds(seeds);
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
                                         PhantomCiphertext& out) {
  const size_t n = ctx.poly_degree(), ci = plain.chain_index();
  const size_t L = ctx.get_context_data(ci).coeff_modulus_size();
  hipStream_t s = ctx.stream();
  out.resize(ctx, ci, 2, s, false);
  out.set_ntt_form(true);
  out.set_scale(plain.scale());
  uint64_t* c0 = out.data();
  uint64_t* c1 = out.data() + L * n;
  DeviceBuffer<uint64_t> e(L * n, s), t(L * n, s);
  sample_uniform(ctx, c1, L);
  sample_error(ctx, e.get(), L);
  const phx::ModView m = ctx.mod_QP();
  hip_ok(phx::poly_mul_add(c1, s_.get(), e.get(), t.get(), m, n, L, s), "a*s+e");
  hip_ok(phx::poly_sub(plain.data(), t.get(), c0, m, n, L, s), "m-(a*s+e)");
  PHX_CHECK(hipStreamSynchronize(s));
}

void PhantomSecretKey::decrypt(const PhantomContext& ctx, const PhantomCiphertext& ct, PhantomPlaintext& out) {
  const size_t n = ctx.poly_degree(), L = ct.coeff_modulus_size();
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

}  // namespace phantom
