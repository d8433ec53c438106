// chebyshev_ps.cpp — the reference's Chebyshev-series evaluation as its callers see it: the
// Paterson-Stockmeyer split of src/evaluate.cu:2998-3535 (EvalChebyshevSeriesPS,
// InnerEvalChebyshevPS) with the host helpers of src/util.cu:15-312 (PopulateParameterPS,
// GetDepthByDegree, Degree, LongDivisionChebyshev, ComputeDegreesPS), evaluated through the
// FLEXIBLEAUTO surface of flexauto.cpp.  The operation sequence is the reference's, so the levels,
// noise-scale degrees and scales a caller gets back are the reference's too (the bootstrap's own
// EvalMod uses the fused evaluator of bootstrap.cpp instead).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <memory>
#include <stdexcept>

#include "ckks_eval.h"

namespace phantom {

namespace ps {

uint32_t Degree(const std::vector<double>& c) {
  if (c.empty()) throw std::invalid_argument("The coefficients vector can not be empty");
  for (size_t i = c.size(); i-- > 0;)
    if (c[i] != 0.0) return static_cast<uint32_t>(i);
  return 0;
}

uint32_t GetDepthByDegree(size_t degree) {
  // (upper degree, depth) rows of GenerateDepthByDegreeTable, src/util.cu:44-58
  static const struct { size_t hi; uint32_t depth; } rows[] = {
      {4, 3}, {5, 4}, {13, 5}, {27, 6}, {59, 7}, {119, 8}, {247, 9}, {495, 10}, {1007, 11}, {2031, 12}};
  if (degree < 5 || degree > 2031)
    throw std::invalid_argument("Polynomial degree is supported from 5 to 2031 inclusive. Its current value is " +
                                std::to_string(degree));
  for (const auto& r : rows)
    if (degree <= r.hi) return r.depth;
  return 12;
}

uint32_t GetMultiplicativeDepthByCoeffVector(const std::vector<double>& vec, bool isNormalized) {
  if (vec.empty()) throw std::invalid_argument("Cannot perform operation on empty vector. vec.size() == 0");
  const uint32_t d = GetDepthByDegree(vec.size() - 1);
  return isNormalized ? d - 1 : d;
}

std::vector<uint32_t> ComputeDegreesPS(uint32_t n) {
  if (n == 0) throw std::invalid_argument("ComputeDegreesPS: The degree is zero. There is no need to evaluate the polynomial.");
  if (n <= 2204) {
    // m for degrees up to 2204 (PopulateParameterPS): (upper degree, m) rows
    static const struct { uint32_t hi, m; } rows[] = {{2, 1},    {11, 2},   {13, 3},   {17, 2},   {55, 3},  {59, 4},
                                                      {76, 3},   {239, 4},  {247, 5},  {284, 4},  {991, 5}, {1007, 6},
                                                      {1083, 5}, {2015, 6}, {2031, 7}, {2204, 6}};
    uint32_t m = 6;
    for (const auto& r : rows)
      if (n <= r.hi) {
        m = r.m;
        break;
      }
    return {n / ((1u << m) - 1) + 1, m};
  }
  // larger degrees: the fewest multiplications k + 2m + 2^(m-1) - 4 among n < k (2^m - 1) with
  // floor(log2 k) within one of floor(log2 sqrt(n / 2)) (first minimum in k-major order)
  uint32_t best_k = 0, best_m = 0, best = ~0u;
  const double target = std::floor(std::log2(std::sqrt(static_cast<double>(n / 2))));
  for (uint32_t k = 1; k <= n; ++k) {
    const double mmax = std::ceil(std::log2(static_cast<double>(n / k)) + 1) + 1;
    for (uint32_t m = 1; m <= mmax; ++m) {
      if (static_cast<int64_t>(n) - static_cast<int64_t>(k) * ((int64_t(1) << m) - 1) >= 0) continue;
      if (std::fabs(std::floor(std::log2(static_cast<double>(k))) - target) > 1) continue;
      const uint32_t mults = k + 2 * m + (1u << (m - 1)) - 4;
      if (mults < best) {
        best = mults;
        best_k = k;
        best_m = m;
      }
    }
  }
  return {best_k, best_m};
}

namespace {

constexpr double kOnePrec = 9.5367431640625e-07;  // 2^-20: IsNotEqualOne's window (src/util.cu:76-86)
bool not_one(double v) { return v <= 1 - kOnePrec || v >= 1 + kOnePrec; }

void trim(std::vector<double>& r) {
  if (r.size() > 1) r.resize(Degree(r) + 1);
}

}  // namespace

// Chebyshev-basis long division f = q g + r (src/util.cu:153-253): products of Chebyshev
// polynomials follow T_a T_b = (T_(a+b) + T_|a-b|) / 2; coefficient 0 is c_0 (not halved) in and out
Division LongDivisionChebyshev(const std::vector<double>& f, const std::vector<double>& g) {
  uint32_t n = Degree(f);
  const uint32_t k = Degree(g);
  if (n != f.size() - 1) throw std::invalid_argument("LongDivisionChebyshev: The dominant coefficient of the divident is zero.");
  if (k != g.size() - 1) throw std::invalid_argument("LongDivisionChebyshev: The dominant coefficient of the divisor is zero.");
  if (n < k) return {std::vector<double>(1, 0.0), f};
  std::vector<double> q(n - k + 1, 0.0), r(f), d;
  const double lead = g.back();
  // subtract d (already holding the divisor's pattern for this step) scaled by r's leading
  // coefficient over g's, in the reference's operation order
  auto subtract = [&]() {
    if (not_one(r.back()))
      for (double& x : d) x *= r.back();
    if (not_one(lead))
      for (double& x : d) x /= lead;
    for (size_t i = 0; i < r.size(); ++i) r[i] -= d[i];
    trim(r);
    n = Degree(r);
  };
  while (n > k) {
    const uint32_t s = n - k;  // T_s g lands on degree n
    d.assign(n + 1, 0.0);
    q[s] = 2 * r.back();
    if (not_one(g[k])) q[s] /= lead;
    if (k == s) {
      d[0] = 2 * g[s];
      for (uint32_t i = 1; i < 2 * k + 1; ++i) d[i] = g[static_cast<uint32_t>(std::abs(static_cast<int32_t>(s - i)))];
    } else if (k > s) {
      d[0] = 2 * g[s];
      for (uint32_t i = 1; i < k - s + 1; ++i) d[i] = g[static_cast<uint32_t>(std::abs(static_cast<int32_t>(s - i)))] + g[s + i];
      for (uint32_t i = k - s + 1; i < n + 1; ++i) d[i] = g[static_cast<uint32_t>(std::abs(static_cast<int32_t>(i - s)))];
    } else {
      d[s] = g[0];
      for (uint32_t i = n - 2 * k; i < n + 1; ++i)
        if (i != s) d[i] = g[static_cast<uint32_t>(std::abs(static_cast<int32_t>(i - s)))];
    }
    subtract();
  }
  if (n == k) {
    d = g;
    q[0] = r.back();
    if (not_one(lead)) q[0] /= lead;
    subtract();
  }
  q[0] *= 2;
  return {q, r};
}

// power-basis long division f = q g + r (src/util.cu:93-138)
Division LongDivisionPoly(const std::vector<double>& f, const std::vector<double>& g) {
  uint32_t n = Degree(f);
  const uint32_t k = Degree(g);
  if (n != f.size() - 1) throw std::invalid_argument("LongDivisionPoly: The dominant coefficient of the divident is zero.");
  if (k != g.size() - 1) throw std::invalid_argument("LongDivisionPoly: The dominant coefficient of the divisor is zero.");
  if (n < k) return {std::vector<double>(1, 0.0), f};
  std::vector<double> q(n - k + 1, 0.0), r(f);
  while (n >= k) {
    const uint32_t s = n - k;
    q[s] = r.back();
    if (not_one(g[k])) q[s] /= g.back();
    for (uint32_t i = 0; i <= k; ++i) r[s + i] -= g[i] * q[s];  // r -= q_s x^s g
    if (r.size() == 1) break;  // (a constant remainder: the reference would loop on it forever)
    n = Degree(r);
    r.resize(n + 1);
  }
  return {q, r};
}

}  // namespace ps

// ---- EvalLinearWSumMutable (src/evaluate.cu:3537-3583) --------------------------------------
PhantomCiphertext EvalLinearWSumMutable(const PhantomContext& ctx, std::vector<PhantomCiphertext*>& cts,
                                        const std::vector<double>& w, const std::vector<double>& sf,
                                        const std::vector<double>& sfBig) {
  if (cts.empty() || cts.size() != w.size()) throw std::invalid_argument("EvalLinearWSumMutable: size mismatch");
  // the operand at the deepest level (a degree-2 one among equals) sets the level of all
  size_t top = 0;
  for (size_t i = 1; i < cts.size(); ++i) {
    const size_t c = cts[i]->chain_index(), ct = cts[top]->chain_index();
    if (c > ct || (c == ct && cts[i]->GetNoiseScaleDeg() == 2)) top = i;
  }
  for (size_t i = 0; i < cts.size(); ++i)
    if (i != top) AdjustLevelsAndDepthInPlace(ctx, *cts[i], *cts[top], sf, sfBig);
  if (cts[top]->GetNoiseScaleDeg() == 2)
    for (PhantomCiphertext* c : cts) EvalModReduceInPlace(ctx, *c, 1);
  PhantomCiphertext sum = EvalMultConst(ctx, *cts[0], w[0], sf);
  for (size_t i = 1; i < cts.size(); ++i) {
    PhantomCiphertext t = EvalMultConst(ctx, *cts[i], w[i], sf);
    EvalAddAutoInplace(ctx, sum, t, sf, sfBig);
  }
  return sum;
}

PhantomCiphertext EvalLinearWSumMutable(const PhantomContext& ctx, std::vector<std::shared_ptr<PhantomCiphertext>>& cts,
                                        const std::vector<double>& w, const std::vector<double>& sf,
                                        const std::vector<double>& sfBig) {
  std::vector<PhantomCiphertext*> p(cts.size());
  for (size_t i = 0; i < cts.size(); ++i) p[i] = cts[i].get();
  return EvalLinearWSumMutable(ctx, p, w, sf, sfBig);
}

namespace {

using CtPtr = std::shared_ptr<PhantomCiphertext>;

// the evaluation state shared by the outer call and its recursion: T_1 .. T_k and T_k, T_2k, ..,
// T_(2^(m-1) k) (T2[0] is T[k-1] itself, as in the reference)
struct PsState {
  const PhantomContext& ctx;
  const PhantomRelinKey& rlk;
  const std::vector<double>& sf;
  const std::vector<double>& sfBig;
  std::vector<CtPtr> T, T2;

  PhantomCiphertext twice_minus_one(const PhantomCiphertext& t) {  // 2 t^2 - 1
    PhantomCiphertext sq = EvalSquare(ctx, t, rlk, sf, sfBig);
    PhantomCiphertext r = EvalAddAuto(ctx, sq, sq, sf, sfBig);
    EvalAddConstInPlaceWrap(ctx, r, -1.0, sf, sfBig);
    return r;
  }

  // sum_{i < deg} w[i + 1] T_(i+1) through EvalLinearWSumMutable (which adjusts T in place)
  PhantomCiphertext lin_sum(const std::vector<double>& w, uint32_t deg) {
    std::vector<PhantomCiphertext*> cts(deg);
    std::vector<double> wt(deg);
    for (uint32_t i = 0; i < deg; ++i) {
      cts[i] = T[i].get();
      wt[i] = w[i + 1];
    }
    return EvalLinearWSumMutable(ctx, cts, wt, sf, sfBig);
  }

  // the divisions shared by both levels of the algorithm: f = q T_(k 2^(m-1)) + r, then
  // r - T_(k (2^(m-1) - 1)) = c q + s' and s = s' + T_(k (2^(m-1) - 1))
  struct Split {
    ps::Division qr, cs;
    std::vector<double> s2;
  };
  static Split split(const std::vector<double>& f, uint32_t k, uint32_t m) {
    const uint32_t k2m2k = k * (1u << (m - 1)) - k;
    std::vector<double> Tkm(k2m2k + k + 1, 0.0);
    Tkm.back() = 1;
    Split s;
    s.qr = ps::LongDivisionChebyshev(f, Tkm);
    std::vector<double> r2 = s.qr.r;
    if (static_cast<int32_t>(k2m2k - ps::Degree(s.qr.r)) <= 0) {
      r2[k2m2k] -= 1;
      r2.resize(ps::Degree(r2) + 1);
    } else {
      r2.resize(k2m2k + 1, 0.0);
      r2.back() = -1;
    }
    s.cs = ps::LongDivisionChebyshev(r2, s.qr.q);
    s.s2 = s.cs.r;
    s.s2.resize(k2m2k + 1, 0.0);
    s.s2.back() = 1;
    return s;
  }

  // c(u): the quotient of the second division (flag: it has degree >= 1)
  bool eval_c(const std::vector<double>& c, PhantomCiphertext& cu) {
    const uint32_t dc = ps::Degree(c);
    if (dc < 1) return false;
    if (dc == 1) cu = c[1] != 1 ? EvalMultConst(ctx, *T[0], c[1], sf) : *T[0];
    else cu = lin_sum(c, dc);
    EvalAddConstInPlaceWrap(ctx, cu, c[0] / 2, sf, sfBig);
    return true;
  }

  // q(u) for a quotient of degree <= k.  top: the outer call adds its leading 2 T_k once, the
  // recursion adds it log2(lead) times (a power of two, m <= 4)
  PhantomCiphertext eval_q_leaf(const std::vector<double>& q, uint32_t k, bool outer) {
    std::vector<double> qc = q;
    qc.resize(k);
    const uint32_t dq = ps::Degree(qc);
    PhantomCiphertext qu;
    if (outer) {
      if (dq > 0) {
        qu = lin_sum(q, dq);
        PhantomCiphertext twice = EvalAddAuto(ctx, *T[k - 1], *T[k - 1], sf, sfBig);
        EvalAddAutoInplace(ctx, qu, twice, sf, sfBig);
      } else {
        qu = *T[k - 1];
        for (uint32_t i = 1; i < q.back(); ++i) EvalAddAutoInplace(ctx, qu, *T[k - 1], sf, sfBig);
      }
    } else {
      PhantomCiphertext lead = *T[k - 1];
      for (uint32_t i = 0; i < std::log2(q.back()); ++i) lead = EvalAddAuto(ctx, lead, lead, sf, sfBig);
      if (dq > 0) {
        qu = lin_sum(q, dq);
        EvalAddAutoInplace(ctx, qu, lead, sf, sfBig);
      } else {
        qu = std::move(lead);
      }
    }
    EvalAddConstInPlaceWrap(ctx, qu, q.front() / 2, sf, sfBig);
    return qu;
  }

  // s(u) for s of degree <= k (monic: its leading T_k added once)
  PhantomCiphertext eval_s_leaf(const std::vector<double>& s2, uint32_t k) {
    std::vector<double> sc = s2;
    sc.resize(k);
    const uint32_t ds = ps::Degree(sc);
    PhantomCiphertext su;
    if (ds > 0) {
      su = lin_sum(s2, ds);
      EvalAddAutoInplace(ctx, su, *T[k - 1], sf, sfBig);
    } else {
      su = *T[k - 1];
    }
    EvalAddConstInPlaceWrap(ctx, su, s2.front() / 2, sf, sfBig);
    return su;
  }

  // (T_(k 2^(m-1)) + c) q + s (- T_(k (2^m - 1)) at the outer level): InnerEvalChebyshevPS
  // (outer = false, src/evaluate.cu:2998-3174) and the tail of EvalChebyshevSeriesPS (outer = true)
  PhantomCiphertext eval(const std::vector<double>& f, uint32_t k, uint32_t m, bool outer,
                         const PhantomCiphertext* T2km1) {
    const Split sp = split(f, k, m);
    PhantomCiphertext cu;
    const bool flag_c = eval_c(sp.cs.q, cu);
    PhantomCiphertext qu = ps::Degree(sp.qr.q) > k ? eval(sp.qr.q, k, m - 1, false, nullptr)
                                                    : eval_q_leaf(sp.qr.q, k, outer);
    PhantomCiphertext su = ps::Degree(sp.s2) > k ? eval(sp.s2, k, m - 1, false, nullptr) : eval_s_leaf(sp.s2, k);
    PhantomCiphertext r = flag_c ? EvalAddAuto(ctx, *T2[m - 1], cu, sf, sfBig)
                                 : EvalAddConst(ctx, *T2[m - 1], sp.cs.q.front() / 2, sf, sfBig);
    r = EvalMultAuto(ctx, r, qu, rlk, sf, sfBig);
    EvalAddAutoInplace(ctx, r, su, sf, sfBig);
    if (T2km1) EvalSubAutoInplace(ctx, r, *T2km1, sf, sfBig);
    return r;
  }
};

}  // namespace

bool ChebyshevUnitInterval(double a, double b) {
  // the reference's test (src/evaluate.cu:3208, 3282): signed differences, so e.g. [-1.2, 0.9]
  // also counts as [-1, 1] and skips the affine map
  return (a - std::round(a) < 1e-10) && (b - std::round(b) < 1e-10) && std::round(a) == -1 && std::round(b) == 1;
}

PhantomCiphertext EvalChebyshevSeriesPS(const PhantomContext& ctx, const PhantomRelinKey& rlk, const PhantomCiphertext& x,
                                        const std::vector<double>& coefficients, double a, double b,
                                        const std::vector<double>& sf, const std::vector<double>& sfBig) {
  const uint32_t n = ps::Degree(coefficients);
  std::vector<double> f2 = coefficients;
  if (coefficients.back() == 0) f2.resize(n + 1);
  const std::vector<uint32_t> km = ps::ComputeDegreesPS(n);
  const uint32_t k = km[0], m = km[1];
  PsState st{ctx, rlk, sf, sfBig, std::vector<CtPtr>(k), std::vector<CtPtr>(m)};
  auto& T = st.T;
  if (ChebyshevUnitInterval(a, b)) {
    T[0] = std::make_shared<PhantomCiphertext>(x);
  } else {  // y = -1 + 2 (x - a) / (b - a): one level
    T[0] = std::make_shared<PhantomCiphertext>(EvalMultConst(ctx, x, 2 / (b - a), sf));
    EvalAddConstInPlaceWrap(ctx, *T[0], -1.0 - 2 * a / (b - a), sf, sfBig);
  }
  const PhantomCiphertext y = *T[0];
  // T_2 .. T_k: T_i = 2 T_(i/2)^2 - 1 for even i, 2 T_(i/2) T_(i/2+1) - y for odd i
  for (uint32_t i = 2; i <= k; ++i) {
    if (i % 2 == 0) {
      T[i - 1] = std::make_shared<PhantomCiphertext>(st.twice_minus_one(*T[i / 2 - 1]));
    } else {
      PhantomCiphertext pr = EvalMultAuto(ctx, *T[i / 2 - 1], *T[i / 2], rlk, sf, sfBig);
      T[i - 1] = std::make_shared<PhantomCiphertext>(EvalAddAuto(ctx, pr, pr, sf, sfBig));
      EvalSubAutoInplace(ctx, *T[i - 1], y, sf, sfBig);
    }
  }
  for (uint32_t i = 1; i < k; ++i) AdjustLevelsAndDepthInPlace(ctx, *T[i - 1], *T[k - 1], sf, sfBig);
  // T_k, T_2k, .., T_(2^(m-1) k), and T_(k (2^m - 1)) = 2 T_(k (2^(i) - 1)) T_(2^i k) - T_k
  auto& T2 = st.T2;
  T2[0] = T[k - 1];
  for (uint32_t i = 1; i < m; ++i) T2[i] = std::make_shared<PhantomCiphertext>(st.twice_minus_one(*T2[i - 1]));
  CtPtr T2km1 = T2[0];
  for (uint32_t i = 1; i < m; ++i) {
    PhantomCiphertext pr = EvalMultAuto(ctx, *T2km1, *T2[i], rlk, sf, sfBig);
    T2km1 = std::make_shared<PhantomCiphertext>(EvalAddAuto(ctx, pr, pr, sf, sfBig));
    EvalSubAutoInplace(ctx, *T2km1, *T2[0], sf, sfBig);
  }
  // f + T_(k (2^m - 1)) is split and evaluated; the added term is subtracted at the end
  const uint32_t k2m2k = k * (1u << (m - 1)) - k;
  f2.resize(2 * k2m2k + k + 1, 0.0);
  f2.back() = 1;
  return st.eval(f2, k, m, true, T2km1.get());
}

}  // namespace phantom
