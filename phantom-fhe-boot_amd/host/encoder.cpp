#include "encoder.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <thread>

#include "../csrc/ntt.h"
#include "hip_check.h"
#include "numth.h"

namespace phantom {

using namespace arith;

PhantomCKKSEncoder::PhantomCKKSEncoder(const PhantomContext& ctx) : PhantomCKKSEncoder(ctx.poly_degree()) {}

PhantomCKKSEncoder::PhantomCKKSEncoder(size_t n) {
  n_ = n;
  logn_ = log2_exact(n_);
  if (logn_ < 2) throw std::invalid_argument("poly_modulus_degree too small");
  const size_t m = 2 * n_;
  zeta_pows_.resize(m);
  for (size_t j = 0; j < m; ++j) {
    const double a = 2.0 * M_PI * static_cast<double>(j) / static_cast<double>(m);
    zeta_pows_[j] = {std::cos(a), std::sin(a)};
  }
  slot_index_.resize(n_ / 2);
  uint64_t p = 1;
  for (size_t j = 0; j < n_ / 2; ++j) {
    slot_index_[j] = static_cast<uint32_t>((p - 1) / 2);
    p = (p * 5) % m;
  }
  brev_.resize(n_);
  for (size_t i = 0; i < n_; ++i) brev_[i] = reverse_bits(static_cast<uint32_t>(i), logn_);
}

// in-place size-n DFT: forward a[k] <- sum_s a[s] w^(sk), inverse with w^-1 (no 1/n), w = zeta^2
void PhantomCKKSEncoder::fft(std::vector<std::complex<double>>& a, bool inverse) const {
  const size_t n = n_;
  for (size_t i = 0; i < n; ++i)
    if (i < brev_[i]) std::swap(a[i], a[brev_[i]]);
  for (size_t len = 2; len <= n; len <<= 1) {
    const size_t step = 2 * n / len;  // w_len = zeta^(2n/len)
    for (size_t i = 0; i < n; i += len)
      for (size_t j = 0; j < len / 2; ++j) {
        std::complex<double> w = zeta_pows_[(j * step) % (2 * n)];
        if (inverse) w = std::conj(w);
        const std::complex<double> u = a[i + j], v = a[i + j + len / 2] * w;
        a[i + j] = u + v;
        a[i + j + len / 2] = u - v;
      }
  }
}

std::vector<double> PhantomCKKSEncoder::slots_to_coeffs(const std::vector<std::complex<double>>& values) const {
  if (values.size() > n_ / 2) throw std::invalid_argument("values has invalid size");
  std::vector<std::complex<double>> a(n_, {0.0, 0.0});
  for (size_t j = 0; j < values.size(); ++j) {
    a[slot_index_[j]] = values[j];
    a[n_ - 1 - slot_index_[j]] = std::conj(values[j]);  // root zeta^(2n - 5^j)
  }
  fft(a, true);
  std::vector<double> c(n_);
  const double inv = 1.0 / static_cast<double>(n_);
  for (size_t k = 0; k < n_; ++k) c[k] = (std::conj(zeta_pows_[k]) * a[k]).real() * inv;
  return c;
}

std::vector<std::complex<double>> PhantomCKKSEncoder::coeffs_to_slots(const std::vector<double>& coeffs) const {
  std::vector<std::complex<double>> b(n_);
  for (size_t k = 0; k < n_; ++k) b[k] = zeta_pows_[k] * coeffs[k];
  fft(b, false);
  std::vector<std::complex<double>> z(n_ / 2);
  for (size_t j = 0; j < n_ / 2; ++j) z[j] = b[slot_index_[j]];
  return z;
}

// exact residues of round(x) for any finite double x
static inline uint64_t double_to_residue(double x, uint64_t q) {
  const double r = std::nearbyint(x);
  const double a = std::fabs(r);
  uint64_t v;
  if (a < 9.2e18) {
    v = static_cast<uint64_t>(a) % q;
  } else {
    int e = 0;
    const double f = std::frexp(a, &e);  // a = f 2^e, f in [0.5, 1)
    const uint64_t mant = static_cast<uint64_t>(std::ldexp(f, 53));
    v = mul_mod(mant % q, pow_mod(2 % q, static_cast<uint64_t>(e - 53), q), q);
  }
  return (r < 0 && v) ? q - v : v;
}

void PhantomCKKSEncoder::to_rns(const std::vector<double>& coeffs, double scale, const std::vector<uint64_t>& moduli,
                                std::vector<uint64_t>& out, unsigned threads) {
  const size_t n = coeffs.size(), L = moduli.size();
  out.resize(L * n);
  std::vector<double> x(n);
  for (size_t k = 0; k < n; ++k) x[k] = coeffs[k] * scale;
  for (size_t k = 0; k < n; ++k)
    if (!std::isfinite(x[k]) || std::fabs(x[k]) >= std::ldexp(1.0, 1000)) throw std::invalid_argument("encoded values are too large");
  // exact residues; limbs spread over host threads (bootstrap setup encodes ~1,000 plaintexts)
  const unsigned nt = threads ? threads
                              : static_cast<unsigned>(std::min<size_t>(
                                    L, std::max(1u, std::min(16u, std::thread::hardware_concurrency()))));
  auto work = [&](unsigned w) {
    for (size_t l = w; l < L; l += nt)
      for (size_t k = 0; k < n; ++k) out[l * n + k] = double_to_residue(x[k], moduli[l]);
  };
  if (nt <= 1 || n * L < (1u << 16)) {
    work(0);
    for (unsigned w = 1; w < nt; ++w) work(w);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned w = 0; w < nt; ++w) th.emplace_back(work, w);
  for (auto& t : th) t.join();
}

static void upload_ntt(const PhantomContext& ctx, const std::vector<uint64_t>& host, PhantomPlaintext& out,
                       const phx::LimbMap& map) {
  hipStream_t s = ctx.stream();
  PHX_CHECK(hipMemcpyAsync(out.data(), host.data(), host.size() * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  const hipError_t e = phx::ntt_forward(ctx.gpu_rns_tables(), out.data(), out.data(), map, s);
  if (e != hipSuccess) throw hip_error(e, "encode NTT");
  PHX_CHECK(hipStreamSynchronize(s));  // `host` may be freed by the caller
}

void PhantomCKKSEncoder::encode(const PhantomContext& ctx, const std::vector<std::complex<double>>& values,
                                double scale, PhantomPlaintext& out, size_t chain_index) const {
  if (scale <= 0) throw std::invalid_argument("scale must be positive");
  const auto& mods = ctx.get_context_data(chain_index).moduli();
  std::vector<uint64_t> host;
  to_rns(slots_to_coeffs(values), scale, mods, host);
  out.resize(ctx, chain_index, ctx.stream());
  out.set_scale(scale);
  upload_ntt(ctx, host, out, phx::LimbMap::contiguous(static_cast<int>(mods.size()), 0));
}

void PhantomCKKSEncoder::encode(const PhantomContext& ctx, const std::vector<double>& values, double scale,
                                PhantomPlaintext& out, size_t chain_index) const {
  std::vector<std::complex<double>> v(values.begin(), values.end());
  encode(ctx, v, scale, out, chain_index);
}

static std::vector<uint64_t> ext_moduli(const PhantomContext& ctx, size_t chain_index) {
  std::vector<uint64_t> mods = ctx.get_context_data(chain_index).moduli();
  const auto& qp = ctx.key_moduli();
  mods.insert(mods.end(), qp.begin() + ctx.size_Q(), qp.end());
  return mods;
}

void PhantomCKKSEncoder::encode_ext_host(const PhantomContext& ctx, const std::vector<std::complex<double>>& values,
                                         double scale, size_t chain_index, std::vector<uint64_t>& host,
                                         unsigned rns_threads) const {
  to_rns(slots_to_coeffs(values), scale, ext_moduli(ctx, chain_index), host, rns_threads);
}

void PhantomCKKSEncoder::upload_ext_async(const PhantomContext& ctx, const std::vector<uint64_t>& host, double scale,
                                          PhantomPlaintext& out, size_t chain_index) const {
  const size_t size_Ql = ctx.get_context_data(chain_index).coeff_modulus_size();
  const size_t limbs = size_Ql + ctx.size_P();
  if (host.size() != limbs * n_) throw std::invalid_argument("host residues do not match the extended basis");
  hipStream_t s = ctx.stream();
  out.resize_ext(ctx, chain_index, limbs, s);
  out.set_scale(scale);
  phx::LimbMap m;
  m.num_limbs = static_cast<int>(limbs);
  m.split = static_cast<int>(size_Ql);
  m.first_a = 0;
  m.first_b = static_cast<int>(ctx.size_Q());
  PHX_CHECK(hipMemcpyAsync(out.data(), host.data(), host.size() * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  const hipError_t e = phx::ntt_forward(ctx.gpu_rns_tables(), out.data(), out.data(), m, s);
  if (e != hipSuccess) throw hip_error(e, "encode NTT");
}

void PhantomCKKSEncoder::encode_ext(const PhantomContext& ctx, const std::vector<std::complex<double>>& values,
                                    double scale, PhantomPlaintext& out, size_t chain_index) const {
  std::vector<uint64_t> host;
  encode_ext_host(ctx, values, scale, chain_index, host);
  upload_ext_async(ctx, host, scale, out, chain_index);
  PHX_CHECK(hipStreamSynchronize(ctx.stream()));  // `host` is freed on return
}

void PhantomCKKSEncoder::decode(const PhantomContext& ctx, const PhantomPlaintext& plain,
                                std::vector<std::complex<double>>& out) const {
  const size_t n = n_, L = plain.coeff_modulus_size();
  const std::vector<uint64_t>& mods = ctx.get_context_data(plain.chain_index()).moduli();
  if (mods.size() != L) throw std::invalid_argument("plaintext is not in the Ql basis of its chain index");
  hipStream_t s = ctx.stream();
  // coefficient form on a device copy
  DeviceBuffer<uint64_t> tmp(L * n, s);
  const hipError_t e = phx::ntt_inverse(ctx.gpu_rns_tables(), plain.data(), tmp.get(),
                                        phx::LimbMap::contiguous(static_cast<int>(L), 0), nullptr, nullptr, s);
  if (e != hipSuccess) throw hip_error(e, "decode INTT");
  std::vector<uint64_t> r = tmp.download(s);

  // Garner mixed-radix digits per coefficient, centered, evaluated in long double
  std::vector<uint64_t> inv_prefix(L);  // (q_0 ... q_{i-1})^-1 mod q_i
  for (size_t i = 0; i < L; ++i) {
    uint64_t pr = 1 % mods[i];
    for (size_t j = 0; j < i; ++j) pr = mul_mod(pr, mods[j] % mods[i], mods[i]);
    inv_prefix[i] = i ? inv_mod(pr, mods[i]) : 1;
  }
  std::vector<long double> radix(L);  // prod_{j<i} q_j
  radix[0] = 1.0L;
  for (size_t i = 1; i < L; ++i) radix[i] = radix[i - 1] * static_cast<long double>(mods[i - 1]);
  auto garner = [&](const uint64_t* res, uint64_t* dig) {
    for (size_t i = 0; i < L; ++i) {
      const uint64_t q = mods[i];
      // value of the digits below i, mod q
      uint64_t acc = 0, pr = 1 % q;
      for (size_t j = 0; j < i; ++j) {
        acc = (acc + mul_mod(dig[j] % q, pr, q)) % q;
        pr = mul_mod(pr, mods[j] % q, q);
      }
      const uint64_t d = (res[i] + q - acc) % q;
      dig[i] = mul_mod(d, inv_prefix[i], q);
    }
  };
  std::vector<uint64_t> half_res(L), half_dig(L);
  // (Q - 1) / 2 mod q_i = (Q - 1) 2^-1 mod q_i = (q_i - 1) 2^-1 mod q_i
  for (size_t i = 0; i < L; ++i) half_res[i] = mul_mod(mods[i] - 1, inv_mod(2, mods[i]), mods[i]);
  garner(half_res.data(), half_dig.data());

  std::vector<double> coeffs(n);
  const double inv_scale = 1.0 / plain.scale();
  const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  for (unsigned w = 0; w < nt; ++w)
    th.emplace_back([&, w] {
      std::vector<uint64_t> res(L), dig(L), cmp(L);
      for (size_t k = w; k < n; k += nt) {
        for (size_t i = 0; i < L; ++i) res[i] = r[i * n + k];
        garner(res.data(), dig.data());
        // x > (Q-1)/2 ?  compare mixed-radix digits from the top
        int c = 0;
        for (size_t i = L; i-- > 0;)
          if (dig[i] != half_dig[i]) {
            c = dig[i] > half_dig[i] ? 1 : -1;
            break;
          }
        long double v = 0.0L;
        if (c > 0) {
          // Q - x: digits (q_i - 1 - a_i) + 1 with carry
          uint64_t carry = 1;
          for (size_t i = 0; i < L; ++i) {
            uint64_t d = mods[i] - 1 - dig[i] + carry;
            carry = d >= mods[i] ? 1 : 0;
            if (carry) d -= mods[i];
            cmp[i] = d;
          }
          for (size_t i = L; i-- > 0;) v += static_cast<long double>(cmp[i]) * radix[i];
          v = -v;
        } else {
          for (size_t i = L; i-- > 0;) v += static_cast<long double>(dig[i]) * radix[i];
        }
        coeffs[k] = static_cast<double>(v * inv_scale);
      }
    });
  for (auto& t : th) t.join();
  out = coeffs_to_slots(coeffs);
}

void PhantomCKKSEncoder::decode(const PhantomContext& ctx, const PhantomPlaintext& plain,
                                std::vector<double>& out) const {
  std::vector<std::complex<double>> z;
  decode(ctx, plain, z);
  out.resize(z.size());
  for (size_t i = 0; i < z.size(); ++i) out[i] = z[i].real();
}

void PhantomCKKSEncoder::encode_sparse(const PhantomContext& ctx, const std::vector<std::complex<double>>& values,
                                       double scale, PhantomPlaintext& out, size_t chain_index) const {
  const size_t slots = n_ / 2, ns = sparse_slots_ ? sparse_slots_ : slots;
  if (ns > slots || (ns & (ns - 1)) || values.size() > ns)
    throw std::invalid_argument("sparse slot count must be a power of two <= N/2 holding every value");
  std::vector<std::complex<double>> v(slots, {0.0, 0.0});
  for (size_t j = 0; j < slots; ++j) v[j] = (j % ns) < values.size() ? values[j % ns] : std::complex<double>(0.0, 0.0);
  encode(ctx, v, scale, out, chain_index);
}

void PhantomCKKSEncoder::encode_sparse(const PhantomContext& ctx, const std::vector<double>& values, double scale,
                                       PhantomPlaintext& out, size_t chain_index) const {
  encode_sparse(ctx, std::vector<std::complex<double>>(values.begin(), values.end()), scale, out, chain_index);
}

}  // namespace phantom
