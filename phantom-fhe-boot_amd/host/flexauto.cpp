// flexauto.cpp — the reference's FLEXIBLEAUTO evaluator surface (include/evaluate.cuh:270-452,
// src/evaluate.cu:2284-3630) with its exact level / degree / scale bookkeeping, so that code
// written against PhantomFHE's bootstrapping API (bootstrapping_example.cu, the reference's own
// Chebyshev series) runs unchanged.  The bootstrap itself uses the fused forms of ckks_eval.h.
#include <algorithm>
#include <cmath>
#include <stdexcept>

#include "../csrc/ckks.h"
#include "../csrc/ntt.h"
#include "../csrc/rns.h"
#include "ckks_eval.h"
#include "evaluate.h"
#include "numth.h"

namespace phantom {

using namespace arith;

PhantomCiphertext ModReduce(const PhantomContext& ctx, const PhantomCiphertext& ct, size_t levels) {
  PhantomCiphertext d = ct;
  EvalModReduceInPlace(ctx, d, levels);
  return d;
}

void ModSwitchLevelInPlace(const PhantomContext& ctx, PhantomCiphertext& ct, size_t levels) {
  const size_t deg = ct.GetNoiseScaleDeg();
  if (levels) mod_switch_to_inplace(ctx, ct, ct.chain_index() + levels);
  ct.SetNoiseScaleDeg(deg);
}

// AdjustLevelsAndDepthInPlace (src/evaluate.cu:2611-2779), written once for "lo is the operand at
// the lower level": lo is brought to hi's level and scale; the branches are the reference's
static void adjust_lower(const PhantomContext& ctx, PhantomCiphertext& lo, const PhantomCiphertext& hi,
                         const std::vector<double>& sf, const std::vector<double>& sfBig) {
  const size_t lo_lvl = level_of(lo), hi_lvl = level_of(hi);
  const size_t lo_deg = lo.GetNoiseScaleDeg(), hi_deg = hi.GetNoiseScaleDeg();
  const double s_lo = lo.scale(), s_hi = hi.scale(), s_target = hi.scale();
  const double q_lo = static_cast<double>(ctx.get_context_data(lo.chain_index()).moduli().back());
  const double scf = sf.at(lo_lvl);
  if (lo_deg == 2) {
    if (hi_deg == 2) {
      EvalMultConstInplaceCore(ctx, lo, s_hi / s_lo * q_lo / scf, sf);
      EvalModReduceInPlace(ctx, lo, 1);
      if (lo_lvl + 1 < hi_lvl) ModSwitchLevelInPlace(ctx, lo, hi_lvl - lo_lvl - 1);
      lo.set_scale(s_target);
    } else if (lo_lvl + 1 == hi_lvl) {
      EvalModReduceInPlace(ctx, lo, 1);
    } else {
      EvalMultConstInplaceCore(ctx, lo, sfBig.at(hi_lvl - 1) / s_lo * q_lo / scf, sf);
      EvalModReduceInPlace(ctx, lo, 1);
      if (lo_lvl + 2 < hi_lvl) ModSwitchLevelInPlace(ctx, lo, hi_lvl - lo_lvl - 2);
      EvalModReduceInPlace(ctx, lo, 1);
      lo.set_scale(s_target);
    }
  } else if (hi_deg == 2) {
    EvalMultConstInplaceCore(ctx, lo, s_hi / s_lo / scf, sf);
    ModSwitchLevelInPlace(ctx, lo, hi_lvl - lo_lvl);
    lo.set_scale(s_target);
  } else {
    EvalMultConstInplaceCore(ctx, lo, sfBig.at(hi_lvl - 1) / s_lo / scf, sf);
    if (lo_lvl + 1 < hi_lvl) ModSwitchLevelInPlace(ctx, lo, hi_lvl - lo_lvl - 1);
    EvalModReduceInPlace(ctx, lo, 1);
    lo.set_scale(s_target);
  }
}

void AdjustLevelsAndDepthInPlace(const PhantomContext& ctx, PhantomCiphertext& c1, PhantomCiphertext& c2,
                                 const std::vector<double>& sf, const std::vector<double>& sfBig) {
  const size_t l1 = level_of(c1), l2 = level_of(c2);
  if (l1 < l2) {
    adjust_lower(ctx, c1, c2, sf, sfBig);
  } else if (l1 > l2) {
    adjust_lower(ctx, c2, c1, sf, sfBig);
  } else if (c1.GetNoiseScaleDeg() < c2.GetNoiseScaleDeg()) {
    EvalMultConstInplaceCore(ctx, c1, 1.0, sf);
  } else if (c2.GetNoiseScaleDeg() < c1.GetNoiseScaleDeg()) {
    EvalMultConstInplaceCore(ctx, c2, 1.0, sf);
  }
}

PhantomCiphertext EvalMultAuto(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomCiphertext& b,
                               const PhantomRelinKey& rlk, const std::vector<double>& sf,
                               const std::vector<double>& sfBig) {
  PhantomCiphertext x = a, y = b;
  AdjustLevelsAndDepthInPlace(ctx, x, y, sf, sfBig);
  if (x.GetNoiseScaleDeg() == 2) {
    EvalModReduceInPlace(ctx, x, 1);
    EvalModReduceInPlace(ctx, y, 1);
  }
  const size_t deg = x.GetNoiseScaleDeg() + y.GetNoiseScaleDeg();
  multiply_and_relin_inplace(ctx, x, y, rlk);
  x.SetNoiseScaleDeg(deg);
  return x;
}

PhantomCiphertext EvalSquare(const PhantomContext& ctx, const PhantomCiphertext& ct, const PhantomRelinKey& rlk,
                             const std::vector<double>& sf, const std::vector<double>& sfBig) {
  (void)sf;
  (void)sfBig;
  PhantomCiphertext d = ct;
  if (d.GetNoiseScaleDeg() != 1) EvalModReduceInPlace(ctx, d, 1);
  const size_t deg = 2 * d.GetNoiseScaleDeg();
  multiply_and_relin_inplace(ctx, d, d, rlk);  // the squaring kernel (same object)
  d.SetNoiseScaleDeg(deg);
  return d;
}

void EvalMultBroadcast(const PhantomContext& ctx, PhantomCiphertext& ct, const PhantomCiphertext& single) {
  const size_t n = ctx.poly_degree(), L = ctx.get_context_data(ct.chain_index()).coeff_modulus_size();
  hip_ok(phx::poly_mul(ct.data(), single.data(), ct.data(), ctx.mod_QP(), n, L, ctx.stream(), ct.size(), 0),
         "broadcast multiply");
  ct.set_scale(ct.scale() * single.scale());
  ct.SetNoiseScaleDeg(ct.GetNoiseScaleDeg() + single.GetNoiseScaleDeg());
}

void EvalMultAutoInplace(const PhantomContext& ctx, PhantomCiphertext& ct, const PhantomPlaintext& pt,
                         const std::vector<double>& sf, const std::vector<double>& sfBig) {
  // MorphPlaintext (src/evaluate.cu:2781-2792): the plaintext as a one-polynomial ciphertext
  PhantomCiphertext morph;
  morph.resize(ctx, pt.chain_index(), 1, ctx.stream(), false);
  PHX_CHECK(hipMemcpyAsync(morph.data(), pt.data(), pt.coeff_modulus_size() * ctx.poly_degree() * sizeof(uint64_t),
                           hipMemcpyDeviceToDevice, ctx.stream()));
  morph.set_ntt_form(true);
  morph.set_scale(pt.scale());
  morph.SetNoiseScaleDeg(pt.GetNoiseScaleDeg());
  AdjustLevelsAndDepthInPlace(ctx, ct, morph, sf, sfBig);
  if (ct.GetNoiseScaleDeg() == 2) {
    EvalModReduceInPlace(ctx, ct, 1);
    EvalModReduceInPlace(ctx, morph, 1);
  }
  EvalMultBroadcast(ctx, ct, morph);
}

void EvalAddAutoInplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b,
                        const std::vector<double>& sf, const std::vector<double>& sfBig) {
  PhantomCiphertext y = b;
  AdjustLevelsAndDepthInPlace(ctx, a, y, sf, sfBig);
  add_inplace(ctx, a, y);
}

void EvalSubAutoInplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b,
                        const std::vector<double>& sf, const std::vector<double>& sfBig) {
  PhantomCiphertext y = b;
  AdjustLevelsAndDepthInPlace(ctx, a, y, sf, sfBig);
  sub_inplace(ctx, a, y);
}

std::vector<uint64_t> GetElementForEvalAddOrSub(const PhantomContext& ctx, const PhantomCiphertext& ct, double operand,
                                                const std::vector<double>& sf, const std::vector<double>& sfBig) {
  (void)sfBig;
  const auto& mods = ctx.get_context_data(ct.chain_index()).moduli();
  const double scFactor = sf.at(ct.chain_index() - 1);
  int32_t logApprox = 0;
  const double res = std::fabs(operand * scFactor);
  if (res > 0) {
    const int32_t logSF = static_cast<int32_t>(std::ceil(std::log2(res)));
    logApprox = logSF - std::min<int32_t>(logSF, 61);
  }
  const double approxFactor = std::pow(2.0, logApprox);
  if (operand < 0) throw std::invalid_argument("EvalAddConstInPlace takes a non-negative operand (use the Wrap form)");
  const uint64_t scConstant = static_cast<uint64_t>(operand * scFactor / approxFactor + 0.5);
  std::vector<uint64_t> c(mods.size());
  for (size_t i = 0; i < mods.size(); ++i) c[i] = scConstant % mods[i];
  while (logApprox > 0) {
    const int32_t step = std::min<int32_t>(logApprox, 60);
    for (size_t i = 0; i < mods.size(); ++i) c[i] = mul_mod(c[i], (uint64_t(1) << step) % mods[i], mods[i]);
    logApprox -= step;
  }
  // the constant is at scale sf^deg: times round(sf) once per degree above 1
  const uint64_t intScFactor = static_cast<uint64_t>(scFactor + 0.5);
  for (size_t d = 1; d < ct.GetNoiseScaleDeg(); ++d)
    for (size_t i = 0; i < mods.size(); ++i) c[i] = mul_mod(c[i], intScFactor % mods[i], mods[i]);
  return c;
}

static void add_residues_c0(const PhantomContext& ctx, PhantomCiphertext& ct, const std::vector<uint64_t>& r) {
  const size_t L = ct.coeff_modulus_size();
  phx::LimbScalars v;
  for (size_t l = 0; l < L; ++l) v.v[l] = r[l];
  hip_ok(phx::add_scalar_v(ct.data(), v, ct.data(), ctx.mod_QP().q, ctx.poly_degree(), L, ctx.stream()), "add const");
}

void EvalAddConstInPlace(const PhantomContext& ctx, PhantomCiphertext& ct, double operand, const std::vector<double>& sf,
                         const std::vector<double>& sfBig) {
  add_residues_c0(ctx, ct, GetElementForEvalAddOrSub(ctx, ct, operand, sf, sfBig));
}

void EvalSubConstInPlace(const PhantomContext& ctx, PhantomCiphertext& ct, double operand, const std::vector<double>& sf,
                         const std::vector<double>& sfBig) {
  std::vector<uint64_t> r = GetElementForEvalAddOrSub(ctx, ct, operand, sf, sfBig);
  const auto& mods = ctx.get_context_data(ct.chain_index()).moduli();
  for (size_t i = 0; i < r.size(); ++i) r[i] = r[i] ? mods[i] - r[i] : 0;
  add_residues_c0(ctx, ct, r);
}

void EvalAddConstInPlaceWrap(const PhantomContext& ctx, PhantomCiphertext& ct, double operand,
                             const std::vector<double>& sf, const std::vector<double>& sfBig) {
  if (operand > 0) EvalAddConstInPlace(ctx, ct, operand, sf, sfBig);
  else if (operand < 0) EvalSubConstInPlace(ctx, ct, -operand, sf, sfBig);
}

static void transform_all(const PhantomContext& ctx, PhantomCiphertext& ct, bool forward) {
  const size_t n = ctx.poly_degree(), L = ct.coeff_modulus_size();
  for (size_t i = 0; i < ct.size(); ++i) {
    uint64_t* p = ct.data() + i * L * n;
    const phx::LimbMap m = phx::LimbMap::contiguous(static_cast<int>(L), 0);
    if (forward) hip_ok(phx::ntt_forward(ctx.gpu_rns_tables(), p, p, m, ctx.stream()), "ConvertToEval");
    else hip_ok(phx::ntt_inverse(ctx.gpu_rns_tables(), p, p, m, nullptr, nullptr, ctx.stream()), "ConvertToCoeff");
  }
  ct.set_ntt_form(forward);
}

void ConvertToEval(const PhantomContext& ctx, PhantomCiphertext& ct) {
  if (!ct.is_ntt_form()) transform_all(ctx, ct, true);
}

void ConvertToCoeff(const PhantomContext& ctx, PhantomCiphertext& ct) {
  if (ct.is_ntt_form()) transform_all(ctx, ct, false);
}

std::vector<double> EvalChebyshevCoefficients(const std::function<double(double)>& func, double a, double b,
                                              uint32_t degree) {
  if (!degree) throw std::invalid_argument("The degree of approximation can not be zero");
  // Chebyshev nodes of [a, b]; coefficient 0 is not halved (the series adds c_0 / 2)
  const size_t m = degree + 1;
  const double half_w = 0.5 * (b - a), mid = 0.5 * (b + a), step = M_PI / static_cast<double>(m);
  std::vector<double> fx(m), c(m, 0.0);
  for (size_t j = 0; j < m; ++j) fx[j] = func(std::cos(step * (static_cast<double>(j) + 0.5)) * half_w + mid);
  for (size_t k = 0; k < m; ++k) {
    double acc = 0.0;
    for (size_t j = 0; j < m; ++j) acc += fx[j] * std::cos(step * static_cast<double>(k) * (static_cast<double>(j) + 0.5));
    c[k] = acc * 2.0 / static_cast<double>(m);
  }
  return c;
}

// EvalChebyshevSeriesLinear (src/evaluate.cu:3188-3262): T_1..T_k by the doubling / product
// recurrences, then sum c_i T_i + c_0 / 2, all through the FLEXIBLEAUTO helpers above
PhantomCiphertext EvalChebyshevSeriesLinear(const PhantomContext& ctx, const PhantomRelinKey& rlk,
                                            const PhantomCiphertext& x, const std::vector<double>& coeffs, double a,
                                            double b, const std::vector<double>& sf, const std::vector<double>& sfBig) {
  // k = coefficients.size() - 1 as the reference takes it: trailing zero coefficients still
  // build their T_i (and cost their levels)
  const size_t k = coeffs.size() - 1;
  if (k < 1) throw std::invalid_argument("a Chebyshev series needs degree 1 or more");
  std::vector<PhantomCiphertext> T(k);
  if (ChebyshevUnitInterval(a, b)) {
    T[0] = x;
  } else {  // y = (2 x - a - b) / (b - a)
    T[0] = EvalMultConst(ctx, x, 2.0 / (b - a), sf);
    EvalAddConstInPlaceWrap(ctx, T[0], -1.0 - 2.0 * a / (b - a), sf, sfBig);
  }
  const PhantomCiphertext& y = T[0];
  for (size_t i = 2; i <= k; ++i) {
    const bool pow2 = (i & (i - 1)) == 0;
    if (pow2 || i % 2 == 0) {  // T_i = 2 T_(i/2)^2 - 1
      PhantomCiphertext sq = EvalSquare(ctx, T[i / 2 - 1], rlk, sf, sfBig);
      PhantomCiphertext t = sq;
      EvalAddAutoInplace(ctx, t, sq, sf, sfBig);
      EvalAddConstInPlaceWrap(ctx, t, -1.0, sf, sfBig);
      T[i - 1] = std::move(t);
    } else {  // T_i = 2 T_(i/2) T_(i/2 + 1) - y
      PhantomCiphertext pr = EvalMultAuto(ctx, T[i / 2 - 1], T[i / 2], rlk, sf, sfBig);
      PhantomCiphertext t = pr;
      EvalAddAutoInplace(ctx, t, pr, sf, sfBig);
      EvalSubAutoInplace(ctx, t, y, sf, sfBig);
      T[i - 1] = std::move(t);
    }
  }
  PhantomCiphertext result = EvalMultConst(ctx, T[k - 1], coeffs[k], sf);
  for (size_t i = 0; i + 1 < k; ++i) {
    if (coeffs[i + 1] == 0) continue;
    EvalMultConstInplace(ctx, T[i], coeffs[i + 1], sf);
    EvalAddAutoInplace(ctx, result, T[i], sf, sfBig);
  }
  EvalAddConstInPlaceWrap(ctx, result, coeffs[0] / 2, sf, sfBig);
  return result;
}

PhantomCiphertext EvalChebyshevSeries(const PhantomContext& ctx, const PhantomRelinKey& rlk, const PhantomCiphertext& x,
                                      const std::vector<double>& coeffs, double a, double b,
                                      const std::vector<double>& sf, const std::vector<double>& sfBig) {
  // src/evaluate.cu:3176-3186: the degree picks the method, the vector goes in as given
  if (ps::Degree(coeffs) < 5) return EvalChebyshevSeriesLinear(ctx, rlk, x, coeffs, a, b, sf, sfBig);
  return EvalChebyshevSeriesPS(ctx, rlk, x, coeffs, a, b, sf, sfBig);
}

}  // namespace phantom
