// host_math_test — CPU-only checks of the bootstrap's host mathematics (no GPU needed):
//  1. encoder: slots -> coefficients -> slots is the identity (canonical embedding and inverse);
//  2. SlotToCoeff factorisation: the stages S_1..S_logn applied to the bit-reversed complex
//     coefficient vector give the canonical embedding of the coefficients;
//  3. CoeffToSlot: the inverse stages applied top-down give back the bit-reversed vector;
//  4. grouping: composed stage groups equal the stage-by-stage product;
//  5. EvalMod: the Chebyshev interpolant of the scaled cosine followed by the double-angle
//     iterations approximates sin(2 pi K y) / (2 pi).
// Prints one JSON object; exit status 0 iff every check passes.
#include <cmath>
#include <complex>
#include <cstdio>
#include <random>
#include <vector>

#include "../host/bootstrap.h"
#include "../host/encoder.h"
#include "../host/numth.h"

using namespace phantom;
using cd = std::complex<double>;

static double max_err(const std::vector<cd>& a, const std::vector<cd>& b) {
  double m = 0;
  for (size_t i = 0; i < a.size(); ++i) m = std::max(m, std::abs(a[i] - b[i]));
  return m;
}

int main() {
  bool ok = true;
  std::mt19937_64 rng(0x5EED);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  const size_t N = 1 << 10, n = N / 2;
  const int logn = arith::log2_exact(n);
  PhantomCKKSEncoder enc(N);

  // 1. encoder round trip
  std::vector<cd> z(n);
  for (auto& x : z) x = {U(rng), U(rng)};
  const double e1 = max_err(enc.coeffs_to_slots(enc.slots_to_coeffs(z)), z);
  ok &= e1 < 1e-12;

  // 2. SlotToCoeff stages
  std::vector<double> t(N);
  for (auto& x : t) x = U(rng);
  std::vector<cd> wbr(n);
  for (size_t p = 0; p < n; ++p) {
    const uint32_t k = arith::reverse_bits(static_cast<uint32_t>(p), logn);
    wbr[p] = {t[k], t[k + n]};
  }
  std::vector<cd> v = wbr;
  for (int s = 1; s <= logn; ++s) v = boot::apply(boot::stage(n, s, false), v);
  const std::vector<cd> ref = enc.coeffs_to_slots(t);
  const double e2 = max_err(v, ref);
  ok &= e2 < 1e-9;

  // 3. CoeffToSlot stages
  std::vector<cd> w = ref;
  for (int s = logn; s >= 1; --s) w = boot::apply(boot::stage(n, s, true), w);
  const double e3 = max_err(w, wbr);
  ok &= e3 < 1e-9;

  // 4. grouped composition (two groups, top-down) equals sequential application
  boot::DiagMap g0, g1;
  g0.emplace(0, std::vector<cd>(n, 1.0));
  g1.emplace(0, std::vector<cd>(n, 1.0));
  for (int s = logn; s > logn / 2; --s) g0 = boot::compose(boot::stage(n, s, true), g0, n);
  for (int s = logn / 2; s >= 1; --s) g1 = boot::compose(boot::stage(n, s, true), g1, n);
  const double e4 = max_err(boot::apply(g1, boot::apply(g0, ref)), wbr);
  ok &= e4 < 1e-9;

  // 5. EvalMod approximation
  const double K = FHECKKSRNS::K_UNIFORM, r = FHECKKSRNS::R_UNIFORM;
  const double args[2] = {K, r};
  const std::vector<double> c = boot::chebyshev_coefficients(boot::scaled_cosine, args, FHECKKSRNS::kChebDegree);
  double e5 = 0, e5_mod = 0;
  for (int i = 0; i <= 20000; ++i) {
    const double y = -1.0 + 2.0 * i / 20000.0;
    // Clenshaw
    double b1 = 0, b2 = 0;
    for (int k = static_cast<int>(c.size()) - 1; k >= 1; --k) {
      const double b0 = 2 * y * b1 - b2 + c[k];
      b2 = b1;
      b1 = b0;
    }
    double p = y * b1 - b2 + c[0];
    e5 = std::max(e5, std::fabs(p - boot::scaled_cosine(y, args)));
    for (int j = 1; j <= static_cast<int>(r); ++j) p = 2 * p * p - std::pow(2 * M_PI, -std::pow(2.0, j - r));
    e5_mod = std::max(e5_mod, std::fabs(p - std::sin(2 * M_PI * K * y) / (2 * M_PI)));
  }
  ok &= e5 < 1e-10 && e5_mod < 1e-8;
  std::printf("{\"encoder_roundtrip\": %.3e, \"stc_stages\": %.3e, \"cts_stages\": %.3e, \"grouped\": %.3e, "
              "\"cheb_fit\": %.3e, \"evalmod_after_double_angle\": %.3e, \"ok\": %s}\n",
              e1, e2, e3, e4, e5, e5_mod, ok ? "true" : "false");
  return ok ? 0 : 1;
}
