#include "ntt_tables.h"

#include <stdexcept>
#include <thread>

#include "hip_check.h"
#include "numth.h"

namespace phantom {

using namespace phantom::arith;

HostNttTable make_host_ntt_table(size_t n, uint64_t q) {
  const int logn = log2_exact(n);
  if (logn < 0) throw std::invalid_argument("ring degree must be a power of two");
  HostNttTable h;
  h.q = q;
  h.psi = minimal_primitive_root(2 * n, q);
  const uint64_t ipsi = inv_mod(h.psi, q);
  h.tw.resize(n); h.tw_shoup.resize(n); h.itw.resize(n); h.itw_shoup.resize(n);
  uint64_t p = 1, ip = 1;
  for (size_t i = 0; i < n; ++i) {
    const uint32_t r = reverse_bits(static_cast<uint32_t>(i), logn);
    h.tw[r] = p;
    h.itw[r] = ip;
    p = mul_mod(p, h.psi, q);
    ip = mul_mod(ip, ipsi, q);
  }
  for (size_t i = 0; i < n; ++i) {
    h.tw_shoup[i] = shoup(h.tw[i], q);
    h.itw_shoup[i] = shoup(h.itw[i], q);
  }
  h.n_inv = inv_mod(n % q, q);
  h.n_inv_shoup = shoup(h.n_inv, q);
  return h;
}

DeviceNttTables::DeviceNttTables(size_t n, const std::vector<uint64_t>& moduli, hipStream_t stream)
    : moduli_(moduli) {
  const size_t L = moduli.size();
  t_.n = n;
  t_.log_n = log2_exact(n);
  t_.lazy16 = true;
  for (uint64_t q : moduli) t_.lazy16 &= q < (uint64_t(1) << 60);
  t_.int_only = true;
  for (uint64_t q : moduli) t_.int_only &= q >= (uint64_t(1) << 50);
  t_.num_moduli = L;
  if (t_.log_n < 3 || t_.log_n > 17) throw std::invalid_argument("unsupported polynomial degree");

  std::vector<HostNttTable> host(L);
  {
    // table generation is O(n L) host work per context; spread it over a few threads
    const unsigned nt = std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()), 16u);
    std::vector<std::thread> th;
    for (unsigned w = 0; w < nt; ++w)
      th.emplace_back([&, w] {
        for (size_t i = w; i < L; i += nt) host[i] = make_host_ntt_table(n, moduli[i]);
      });
    for (auto& x : th) x.join();
  }
  std::vector<uint64_t> flat(n * L), mod(L), bar(2 * L), ninv(L), ninvs(L);
  for (size_t i = 0; i < L; ++i) {
    mod[i] = moduli[i];
    barrett_ratio(moduli[i], &bar[2 * i]);
    ninv[i] = host[i].n_inv;
    ninvs[i] = host[i].n_inv_shoup;
  }
  auto alloc_copy = [&](uint64_t*& dst, const std::vector<uint64_t>& src) {
    PHX_CHECK(hipMalloc(&dst, src.size() * sizeof(uint64_t)));
    PHX_CHECK(hipMemcpyAsync(dst, src.data(), src.size() * sizeof(uint64_t), hipMemcpyHostToDevice, stream));
  };
  alloc_copy(t_.modulus, mod);
  alloc_copy(t_.barrett, bar);
  alloc_copy(t_.n_inv, ninv);
  alloc_copy(t_.n_inv_shoup, ninvs);
  auto gather = [&](uint64_t*& dst, std::vector<uint64_t> HostNttTable::*member) {
    for (size_t i = 0; i < L; ++i) std::copy((host[i].*member).begin(), (host[i].*member).end(), flat.begin() + i * n);
    alloc_copy(dst, flat);
    PHX_CHECK(hipStreamSynchronize(stream));  // flat is reused
  };
  {
    // FP64 tables (csrc/ntt.hip): column-pass twiddles and the factored row-pass twiddles.
    // For row R and row-pass stage g (global stage k = s1 + g),
    //   tw[2^k + R 2^g + iloc] = psi^(2^(logn-1-k) (1 + 2 brv_s1(R))) * psi^(2^(logn-g) brv_g(iloc))
    // and itw[...] is the product of the inverses of the same two factors.
    const int logn = t_.log_n, s1 = phx::ntt_split_log_s1(logn), s2 = logn - s1;
    const size_t S1 = size_t(1) << s1, S2 = size_t(1) << s2;
    std::vector<double> qf(L), qi(L), cf(L * S1), ci(L * S1);
    std::vector<double> raf(L * S1 * 16, 0.0), rbf(L * S2, 0.0), rai(L * S1 * 16, 0.0), rbi(L * S2, 0.0);
    auto centered = [](uint64_t w, uint64_t q) {
      return w > (q - 1) / 2 ? -static_cast<double>(q - w) : static_cast<double>(w);
    };
    for (size_t i = 0; i < L; ++i) {
      const uint64_t q = moduli[i], psi = host[i].psi, ipsi = inv_mod(psi, q);
      qf[i] = static_cast<double>(q);
      qi[i] = 1.0 / static_cast<double>(q);
      for (size_t k = 0; k < S1; ++k) {
        cf[i * S1 + k] = centered(host[i].tw[k], q);
        uint64_t w = host[i].itw[k];
        if (k == 1) w = mul_mod(w, host[i].n_inv, q);
        if (k == 0) w = host[i].n_inv;
        ci[i * S1 + k] = centered(w, q);
      }
      for (size_t R = 0; R < S1; ++R)
        for (int g = 0; g < s2; ++g) {
          const uint64_t e = (uint64_t(1) << (logn - 1 - s1 - g)) * (1 + 2 * (uint64_t)reverse_bits((uint32_t)R, s1));
          raf[(i * S1 + R) * 16 + g] = centered(pow_mod(psi, e, q), q);
          rai[(i * S1 + R) * 16 + g] = centered(pow_mod(ipsi, e, q), q);
        }
      for (int g = 0; g < s2; ++g)
        for (size_t il = 0; il < (size_t(1) << g); ++il) {
          const uint64_t e = (uint64_t(1) << (logn - g)) * (uint64_t)reverse_bits((uint32_t)il, g);
          rbf[i * S2 + (size_t(1) << g) + il] = centered(pow_mod(psi, e, q), q);
          rbi[i * S2 + (size_t(1) << g) + il] = centered(pow_mod(ipsi, e, q), q);
        }
    }
    auto up = [&](double*& dst, const std::vector<double>& src) {
      PHX_CHECK(hipMalloc(&dst, src.size() * sizeof(double)));
      PHX_CHECK(hipMemcpyAsync(dst, src.data(), src.size() * sizeof(double), hipMemcpyHostToDevice, stream));
    };
    up(t_.modulus_f, qf);
    up(t_.modulus_inv, qi);
    up(t_.col_fwd, cf);
    up(t_.col_inv, ci);
    up(t_.row_a_fwd, raf);
    up(t_.row_b_fwd, rbf);
    up(t_.row_a_inv, rai);
    up(t_.row_b_inv, rbi);
    PHX_CHECK(hipStreamSynchronize(stream));
  }
  gather(t_.tw, &HostNttTable::tw);
  gather(t_.tw_shoup, &HostNttTable::tw_shoup);
  gather(t_.itw, &HostNttTable::itw);
  gather(t_.itw_shoup, &HostNttTable::itw_shoup);
}

DeviceNttTables::~DeviceNttTables() {
  for (uint64_t* p : {t_.modulus, t_.barrett, t_.tw, t_.tw_shoup, t_.itw, t_.itw_shoup, t_.n_inv, t_.n_inv_shoup})
    if (p) (void)hipFree(p);
  for (double* p : {t_.modulus_f, t_.modulus_inv, t_.col_fwd, t_.col_inv, t_.row_a_fwd, t_.row_b_fwd, t_.row_a_inv,
                    t_.row_b_inv})
    if (p) (void)hipFree(p);
}

}  // namespace phantom
