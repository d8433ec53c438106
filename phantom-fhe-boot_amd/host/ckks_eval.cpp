#include "ckks_eval.h"

#include <cmath>
#include <map>
#include <mutex>
#include <stdexcept>

#include "../csrc/ckks.h"
#include "../csrc/ntt.h"
#include "../csrc/rns.h"
#include "evaluate.h"
#include "numth.h"
#include "traffic.h"

namespace phantom {

using namespace arith;

// exact residue of round(x) mod q for any finite double
static uint64_t residue_of_double(double x, uint64_t q) {
  const double r = std::nearbyint(x);
  const double a = std::fabs(r);
  uint64_t v;
  if (a < 9.2e18) {
    v = static_cast<uint64_t>(a) % q;
  } else {
    int e = 0;
    const double f = std::frexp(a, &e);
    const uint64_t mant = static_cast<uint64_t>(std::ldexp(f, 53));
    v = mul_mod(mant % q, pow_mod(2 % q, static_cast<uint64_t>(e - 53), q), q);
  }
  return (r < 0 && v) ? q - v : v;
}

// per-limb scalar and Shoup arrays on the device (setup-style upload; waits for the copy)
struct Scalars {
  DeviceBuffer<uint64_t> v, vs;
};
static Scalars upload_scalars(const std::vector<uint64_t>& vals, const std::vector<uint64_t>& mods, hipStream_t s) {
  std::vector<uint64_t> sh(vals.size());
  for (size_t i = 0; i < vals.size(); ++i) sh[i] = shoup(vals[i], mods[i]);
  Scalars r;
  r.v.upload(vals, s);
  r.vs.upload(sh, s);
  return r;
}

std::vector<double> precompute_scaling_factors(const PhantomContext& ctx, double scale) {
  const size_t sizeQ = ctx.size_Q();
  const auto& m = ctx.key_moduli();
  std::vector<double> sf(sizeQ);
  if (sizeQ == 1) {
    sf[0] = scale;
    return sf;
  }
  sf[0] = static_cast<double>(m[sizeQ - 1]);
  for (size_t k = 1; k < sizeQ; ++k) {
    sf[k] = sf[k - 1] * sf[k - 1] / static_cast<double>(m[sizeQ - k]);
    const double ratio = sf[k] / sf[0];
    if (ratio <= 0.5 || ratio >= 2.0)
      throw std::invalid_argument("FLEXIBLEAUTO cannot support this number of levels in this parameter setting");
  }
  return sf;
}

void mult_by_real_integer_inplace(const PhantomContext& ctx, PhantomCiphertext& ct, double k) {
  const auto& mods = ctx.get_context_data(ct.chain_index()).moduli();
  const size_t n = ctx.poly_degree(), L = ct.coeff_modulus_size();
  traffic::ciphertexts(traffic::limb_bytes(2 * ct.size() * L, n));
  std::vector<uint64_t> r(L);
  for (size_t l = 0; l < L; ++l) r[l] = residue_of_double(k, mods[l]);
  if (L <= static_cast<size_t>(phx::kMaxScalarLimbs)) {
    // constants travel in the kernel arguments: no upload, no stream synchronisation
    phx::LimbScalars c;
    for (size_t l = 0; l < L; ++l) {
      c.v[l] = r[l];
      c.vs[l] = shoup(r[l], mods[l]);
    }
    hip_ok(phx::mul_scalar_v(ct.data(), c, ct.data(), ctx.mod_QP().q, n, L, ctx.stream(), ct.size()),
           "mult by integer");
    return;
  }
  Scalars sc = upload_scalars(r, mods, ctx.stream());
  hip_ok(phx::poly_mul_scalar(ct.data(), sc.v.get(), sc.vs.get(), ct.data(), ctx.mod_QP(), n, L, ctx.stream(),
                              ct.size()),
         "mult by integer");
}

void MultByIntegerInPlace(const PhantomContext& ctx, PhantomCiphertext& ct, uint64_t k) {
  mult_by_real_integer_inplace(ctx, ct, static_cast<double>(k));
  if (static_cast<uint64_t>(static_cast<double>(k)) != k) throw std::invalid_argument("integer not exact in double");
}

// GetElementForEvalMult (src/evaluate.cu:2332-2412): round(operand * sf[level]) as residues, the
// reference's exact integer path (a 125-bit window rounded half up, then scaled back by powers of 2)
std::vector<uint64_t> GetElementForEvalMult(const PhantomContext& ctx, const PhantomCiphertext& ct, double operand,
                                            const std::vector<double>& sf) {
  const auto& mods = ctx.get_context_data(ct.chain_index()).moduli();
  const double scFactor = sf.at(ct.chain_index() - 1);
  int32_t logApprox = 0;
  const double res = std::fabs(operand * scFactor);
  if (res > 0) {
    const int32_t logSF = static_cast<int32_t>(std::ceil(std::log2(res)));
    logApprox = logSF - std::min<int32_t>(logSF, 125);
  }
  const double approxFactor = std::pow(2.0, logApprox);
  using i128 = __int128;
  const i128 large = static_cast<i128>(operand / approxFactor * scFactor + 0.5);
  std::vector<uint64_t> f(mods.size());
  for (size_t i = 0; i < mods.size(); ++i) {
    const i128 r = large % static_cast<i128>(mods[i]);
    f[i] = static_cast<uint64_t>(r < 0 ? r + static_cast<i128>(mods[i]) : r);
  }
  while (logApprox > 0) {  // times 2^logApprox, 60 bits at a time
    const int32_t step = std::min<int32_t>(logApprox, 60);
    for (size_t i = 0; i < mods.size(); ++i) f[i] = mul_mod(f[i], (uint64_t(1) << step) % mods[i], mods[i]);
    logApprox -= step;
  }
  return f;
}

// ct *= per-limb residues `r` (Shoup constants in the kernel arguments when they fit)
static void mult_by_residues(const PhantomContext& ctx, PhantomCiphertext& ct, const std::vector<uint64_t>& r) {
  const auto& mods = ctx.get_context_data(ct.chain_index()).moduli();
  const size_t n = ctx.poly_degree(), L = ct.coeff_modulus_size();
  traffic::ciphertexts(traffic::limb_bytes(2 * ct.size() * L, n));
  if (L <= static_cast<size_t>(phx::kMaxScalarLimbs)) {
    phx::LimbScalars c;
    for (size_t l = 0; l < L; ++l) {
      c.v[l] = r[l];
      c.vs[l] = shoup(r[l], mods[l]);
    }
    hip_ok(phx::mul_scalar_v(ct.data(), c, ct.data(), ctx.mod_QP().q, n, L, ctx.stream(), ct.size()), "mult const");
    return;
  }
  Scalars sc = upload_scalars(r, mods, ctx.stream());
  hip_ok(phx::poly_mul_scalar(ct.data(), sc.v.get(), sc.vs.get(), ct.data(), ctx.mod_QP(), n, L, ctx.stream(),
                              ct.size()),
         "mult const");
}

void EvalMultConstInplaceCore(const PhantomContext& ctx, PhantomCiphertext& ct, double c, const std::vector<double>& sf) {
  mult_by_residues(ctx, ct, GetElementForEvalMult(ctx, ct, c, sf));
  ct.SetNoiseScaleDeg(ct.GetNoiseScaleDeg() + 1);
  ct.set_scale(ct.scale() * sf.at(level_of(ct)));
}

void EvalMultConstInplace(const PhantomContext& ctx, PhantomCiphertext& ct, double c, const std::vector<double>& sf) {
  if (ct.GetNoiseScaleDeg() == 2) EvalModReduceInPlace(ctx, ct, 1);  // include/evaluate.cuh:317-326
  EvalMultConstInplaceCore(ctx, ct, c, sf);
}

void EvalAddConstInplace(const PhantomContext& ctx, PhantomCiphertext& ct, double c) {
  const auto& mods = ctx.get_context_data(ct.chain_index()).moduli();
  const size_t n = ctx.poly_degree(), L = ct.coeff_modulus_size();
  std::vector<uint64_t> r(L);
  for (size_t l = 0; l < L; ++l) r[l] = residue_of_double(c * ct.scale(), mods[l]);
  // NTT of a constant polynomial is that constant at every evaluation point
  if (L <= static_cast<size_t>(phx::kMaxScalarLimbs)) {
    phx::LimbScalars v;
    for (size_t l = 0; l < L; ++l) v.v[l] = r[l];
    hip_ok(phx::add_scalar_v(ct.data(), v, ct.data(), ctx.mod_QP().q, n, L, ctx.stream()), "add const");
    return;
  }
  Scalars sc = upload_scalars(r, mods, ctx.stream());
  hip_ok(phx::poly_add_scalar(ct.data(), sc.v.get(), ct.data(), ctx.mod_QP(), n, L, ctx.stream()), "add const");
}

void MultByMonomialInPlace(const PhantomContext& ctx, PhantomCiphertext& ct, uint32_t power) {
  const size_t n = ctx.poly_degree(), L = ct.coeff_modulus_size();
  hipStream_t s = ctx.stream();
  const uint64_t* mono = ctx.monomial_ntt(power, L);
  traffic::ciphertexts(traffic::limb_bytes(2 * ct.size() * L, n));
  hip_ok(phx::poly_mul(ct.data(), mono, ct.data(), ctx.mod_QP(), n, L, s, ct.size(), 0), "monomial");
}

void EvalModReduceInPlace(const PhantomContext& ctx, PhantomCiphertext& ct, size_t levels) {
  for (size_t i = 0; i < levels; ++i) {
    const size_t deg = ct.GetNoiseScaleDeg();
    ct = rescale_to_next(ctx, ct);
    ct.SetNoiseScaleDeg(deg > 1 ? deg - 1 : 1);
  }
}

void ScalarResidues(const PhantomContext& ctx, size_t chain, double k, uint64_t* v, uint64_t* vs) {
  const auto& mods = ctx.get_context_data(chain).moduli();
  for (size_t l = 0; l < mods.size(); ++l) {
    v[l] = residue_of_double(k, mods[l]);
    if (vs) vs[l] = shoup(v[l], mods[l]);
  }
}

// exact residues of round(k) at `chain` as kernel-argument constants (L <= kMaxScalarLimbs)
static phx::LimbScalars limb_scalars(const PhantomContext& ctx, size_t chain, double k) {
  const auto& mods = ctx.get_context_data(chain).moduli();
  if (mods.size() > static_cast<size_t>(phx::kMaxScalarLimbs)) throw std::invalid_argument("too many limbs");
  phx::LimbScalars c;
  for (size_t l = 0; l < mods.size(); ++l) {
    c.v[l] = residue_of_double(k, mods[l]);
    c.vs[l] = shoup(c.v[l], mods[l]);
  }
  return c;
}

PhantomCiphertext ScaledModSwitch(const PhantomContext& ctx, const PhantomCiphertext& ct, size_t chain, double k) {
  if (chain < ct.chain_index()) throw std::invalid_argument("cannot switch to higher level modulus");
  const size_t n = ctx.poly_degree();
  PhantomCiphertext out;
  out.resize(ctx, chain, ct.size(), ctx.stream(), false);
  const size_t L = out.coeff_modulus_size();
  if (L > static_cast<size_t>(phx::kMaxScalarLimbs)) {
    out = mod_switch_to(ctx, ct, chain);
    mult_by_real_integer_inplace(ctx, out, k);
    return out;
  }
  hip_ok(phx::mul_scalar_v(ct.data(), limb_scalars(ctx, chain, k), out.data(), ctx.mod_QP().q, n, L, ctx.stream(),
                           ct.size(), ct.coeff_modulus_size() * n),
         "scaled mod switch");
  out.set_scale(ct.scale());
  out.set_ntt_form(ct.is_ntt_form());
  out.set_correction_factor(ct.correction_factor());
  out.SetNoiseScaleDeg(ct.GetNoiseScaleDeg());
  return out;
}

void AccumulateScaled(const PhantomContext& ctx, PhantomCiphertext& acc, const PhantomCiphertext& ct, double k) {
  if (acc.chain_index() < ct.chain_index() || acc.size() != ct.size())
    throw std::invalid_argument("accumulate: operand below the accumulator's level");
  const size_t n = ctx.poly_degree(), L = acc.coeff_modulus_size();
  hip_ok(phx::mul_scalar_v(ct.data(), limb_scalars(ctx, acc.chain_index(), k), acc.data(), ctx.mod_QP().q, n, L,
                           ctx.stream(), ct.size(), ct.coeff_modulus_size() * n, acc.data()),
         "accumulate scaled");
}

// degree-1 `ct` (level < target) -> level `target` at scale sf[target]: drop to level target - 1
// and multiply by the integer that makes the next rescale land on sf[target], in one kernel,
// then rescale
static PhantomCiphertext adjusted(const PhantomContext& ctx, const PhantomCiphertext& ct, size_t target,
                                  const std::vector<double>& sf) {
  const size_t chain_mid = target;  // chain index = level + 1
  const double qdrop = static_cast<double>(ctx.get_context_data(chain_mid).moduli().back());
  const double k = sf.at(target) * qdrop / ct.scale();
  PhantomCiphertext t = ScaledModSwitch(ctx, ct, chain_mid, k);
  t.set_scale(ct.scale() * std::nearbyint(k));
  t.SetNoiseScaleDeg(2);
  PhantomCiphertext r = rescale_to_next(ctx, t);
  r.SetNoiseScaleDeg(1);
  r.set_scale(sf.at(target));
  return r;
}

static size_t level_after_reduce(const PhantomCiphertext& ct) {
  return level_of(ct) + (ct.GetNoiseScaleDeg() > 1 ? 1 : 0);
}

// `ct` at degree 1 and level `target` (>= its level after reduction): ct itself when it already
// is, otherwise a new ciphertext held in `tmp`
const PhantomCiphertext& AtLevel(const PhantomContext& ctx, const PhantomCiphertext& ct, size_t target,
                                 const std::vector<double>& sf, PhantomCiphertext& tmp) {
  if (ct.GetNoiseScaleDeg() <= 1 && level_of(ct) == target) return ct;
  if (level_after_reduce(ct) > target) throw std::invalid_argument("cannot raise a ciphertext's level");
  const PhantomCiphertext* src = &ct;
  PhantomCiphertext reduced;
  if (ct.GetNoiseScaleDeg() > 1) {
    reduced = rescale_to_next(ctx, ct);
    reduced.SetNoiseScaleDeg(ct.GetNoiseScaleDeg() - 1);
    src = &reduced;
  }
  if (level_of(*src) == target) {
    tmp = std::move(reduced);
  } else {
    tmp = adjusted(ctx, *src, target, sf);
  }
  return tmp;
}

std::vector<PhantomCiphertext> AtLevelBatch(const PhantomContext& ctx, const std::vector<const PhantomCiphertext*>& cts,
                                            const std::vector<size_t>& targets, const std::vector<double>& sf) {
  if (cts.size() != targets.size()) throw std::invalid_argument("AtLevelBatch: size mismatch");
  std::vector<PhantomCiphertext> out(cts.size());
  const size_t n = ctx.poly_degree();
  hipStream_t s = ctx.stream();
  // the ones adjusted() would handle (degree 1, two polynomials, below their target), grouped by
  // target level; the rest one by one (AtLevel)
  std::map<size_t, std::vector<size_t>> groups;
  for (size_t k = 0; k < cts.size(); ++k) {
    const PhantomCiphertext& c = *cts[k];
    if (c.GetNoiseScaleDeg() <= 1 && level_of(c) == targets[k]) continue;  // as it is (empty result)
    if (c.GetNoiseScaleDeg() <= 1 && c.size() == 2 && level_of(c) < targets[k]) {
      groups[targets[k]].push_back(k);
    } else {
      PhantomCiphertext tmp;
      const PhantomCiphertext& r = AtLevel(ctx, c, targets[k], sf, tmp);
      out[k] = &r == &c ? PhantomCiphertext(c) : std::move(tmp);
    }
  }
  for (auto& [target, ks] : groups) {
    // adjusted(): round(k) times the leading limbs at chain `target` (one level above the target
    // level), then one rescale; every ciphertext's scaled copy side by side, the rescale batched
    const size_t mid = target, L = ctx.get_context_data(mid).coeff_modulus_size(), words = 2 * L * n;
    const RnsTool& rt = ctx.get_context_data(mid).gpu_rns_tool();
    const double qdrop = static_cast<double>(rt.base_Ql().back());
    for (size_t c0 = 0; c0 < ks.size(); c0 += phx::kMaxKsProds) {
      const size_t cnt = std::min<size_t>(phx::kMaxKsProds, ks.size() - c0);
      DeviceBuffer<uint64_t> w(cnt * words, s);
      std::vector<uint64_t*> outs(cnt);
      for (size_t j = 0; j < cnt; ++j) {
        const PhantomCiphertext& c = *cts[ks[c0 + j]];
        const double k = sf.at(target) * qdrop / c.scale();
        hip_ok(phx::mul_scalar_v(c.data(), limb_scalars(ctx, mid, k), w.get() + j * words, ctx.mod_QP().q, n, L, s, 2,
                                 c.coeff_modulus_size() * n),
               "scaled mod switch");
        PhantomCiphertext& o = out[ks[c0 + j]];
        o.resize(ctx, mid + 1, 2, s, false);
        o.set_ntt_form(true);
        o.set_scale(sf.at(target));
        o.SetNoiseScaleDeg(1);
        outs[j] = o.data();
      }
      rt.rescale_ntt_to(w.get(), outs.data(), cnt, ctx.gpu_rns_tables(), s);
    }
  }
  return out;
}

void AdjustToLevel(const PhantomContext& ctx, PhantomCiphertext& ct, size_t target, const std::vector<double>& sf) {
  if (ct.GetNoiseScaleDeg() > 1) EvalModReduceInPlace(ctx, ct, 1);
  const size_t lvl = level_of(ct);
  if (lvl > target) throw std::invalid_argument("cannot raise a ciphertext's level");
  if (lvl == target) return;
  ct = adjusted(ctx, ct, target, sf);
}

void EvalAddAutoInplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b,
                        const std::vector<double>& sf) {
  const size_t target = std::max(level_after_reduce(a), level_after_reduce(b));
  AdjustToLevel(ctx, a, target, sf);
  PhantomCiphertext tmp;
  add_inplace(ctx, a, AtLevel(ctx, b, target, sf, tmp));
}

void EvalSubAutoInplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b,
                        const std::vector<double>& sf) {
  const size_t target = std::max(level_after_reduce(a), level_after_reduce(b));
  AdjustToLevel(ctx, a, target, sf);
  PhantomCiphertext tmp;
  sub_inplace(ctx, a, AtLevel(ctx, b, target, sf, tmp));
}

void relinearize_rescale_raw(const PhantomContext& ctx, size_t chain_index, const uint64_t* d3, uint64_t* out,
                             const uint64_t* const* evk, hipStream_t s) {
  if (chain_index < 1 || chain_index + 1 >= ctx.total_parm_size())
    throw std::invalid_argument("end of modulus switching chain reached");
  const RnsTool& rt = ctx.get_context_data(chain_index).gpu_rns_tool();
  const size_t n = ctx.poly_degree(), Ql = rt.size_Ql(), QlP = Ql + ctx.size_P(), beta = rt.beta();
  uint64_t* t_mod_up = rt.workspace().get(s, Workspace::kKsModup, beta * QlP * n);
  rt.modup(t_mod_up, d3 + 2 * Ql * n, ctx.gpu_rns_tables(), s);
  uint64_t* cx = rt.workspace().get(s, Workspace::kKsCx, 2 * QlP * n);
  // the inner product is formed inside the moddown-rescale: its dropped limbs (q_last with the
  // addend, P) in the INTT's prologue, its first Ql - 1 limbs in the finish's epilogue (ntt.h
  // ntt_inverse_ks, NttEpilogue::ks_beta), so no limb of it makes an HBM round trip
  // (PHX_KS_EPI=0: the whole inner product in one kernel)
  const bool fuse = ks_epilogue_enabled() && beta <= (size_t)phx::kMaxKsBeta && n >= 1024 && Ql >= 2;
  if (!fuse) {
    phx::KsAddend add;
    add.c = d3;
    add.pmod = rt.bigP_mod_q();
    add.pmod_shoup = rt.bigP_mod_q_shoup();
    hip_ok(phx::keyswitch_inner_prod(t_mod_up, evk, cx, ctx.mod_QP().q, ctx.mod_QP().barrett, n, Ql, ctx.size_Q(),
                                     ctx.size_P(), beta, s, add),
           "relinearize inner product");
  }
  phx::NttEpilogue ks;
  if (fuse) {
    ks.ks_beta = (int)beta;
    ks.tmu = t_mod_up;
    ks.tmu_stride = QlP * n;
    ks.evk = evk;
    ks.evk_poly_stride = ctx.size_QP() * n;
    ks.add_c = d3;
    ks.add_stride = Ql * n;
    ks.pmod = rt.bigP_mod_q();
    ks.pmod_shoup = rt.bigP_mod_q_shoup();
  }
  traffic::keys(traffic::limb_bytes(beta * 2 * QlP, n));
  traffic::ciphertexts(traffic::limb_bytes(3 * Ql + 2 * (Ql - 1), n));  // d read, the rescaled result written
  rt.moddown_rescale(out, cx, ctx.gpu_rns_tables(), s, 2, fuse ? &ks : nullptr);
}

void relinearize_rescale_batch_raw(const PhantomContext& ctx, size_t chain_index, const uint64_t* d3, size_t d3_stride,
                                   size_t count, uint64_t* const* out, const uint64_t* const* evk, hipStream_t s) {
  if (chain_index < 1 || chain_index + 1 >= ctx.total_parm_size())
    throw std::invalid_argument("end of modulus switching chain reached");
  const RnsTool& rt = ctx.get_context_data(chain_index).gpu_rns_tool();
  const size_t n = ctx.poly_degree(), Ql = rt.size_Ql(), QlP = Ql + ctx.size_P(), beta = rt.beta();
  if (count < 1 || count > static_cast<size_t>(phx::kMaxKsProds) || (count > 1 && d3_stride < 3 * Ql * n))
    throw std::invalid_argument("relinearize_rescale_batch: bad batch");
  const bool fuse = ks_epilogue_enabled() && beta <= (size_t)phx::kMaxKsBeta && n >= 1024 && Ql >= 2;
  if (!fuse || count == 1) {
    for (size_t k = 0; k < count; ++k) relinearize_rescale_raw(ctx, chain_index, d3 + k * d3_stride, out[k], evk, s);
    return;
  }
  // every stage once over all `count` key switches: one batched modup (INTT, digit conversions,
  // digit NTTs), one moddown-rescale over 2 count polynomials with the inner products formed in
  // its INTT prologue and NTT epilogue (ntt.h NttEpilogue::ks_prods)
  uint64_t* t_mod_up = rt.workspace().get(s, Workspace::kKsModup, count * beta * QlP * n);
  rt.modup(t_mod_up, d3 + 2 * Ql * n, ctx.gpu_rns_tables(), s, count, d3_stride);
  uint64_t* cx = rt.workspace().get(s, Workspace::kKsCx, 2 * count * QlP * n);
  phx::NttEpilogue ks;
  ks.ks_beta = (int)beta;
  ks.tmu = t_mod_up;
  ks.tmu_stride = QlP * n;
  ks.evk = evk;
  ks.evk_poly_stride = ctx.size_QP() * n;
  ks.add_c = d3;
  ks.add_stride = Ql * n;
  ks.pmod = rt.bigP_mod_q();
  ks.pmod_shoup = rt.bigP_mod_q_shoup();
  ks.ks_prods = static_cast<int>(count);
  ks.tmu_prod_stride = beta * QlP * n;
  for (size_t k = 0; k < count; ++k) {
    ks.out_p[k] = out[k];
    ks.add_p[k] = d3 + k * d3_stride;
  }
  traffic::keys(traffic::limb_bytes(count * beta * 2 * QlP, n));
  traffic::ciphertexts(traffic::limb_bytes(count * (3 * Ql + 2 * (Ql - 1)), n));
  rt.moddown_rescale(out[0], cx, ctx.gpu_rns_tables(), s, 2 * count, &ks);
}

std::vector<PhantomCiphertext> MulAddRescaleBatch(const PhantomContext& ctx, const std::vector<MulAddJob>& jobs,
                                                  const PhantomRelinKey& rlk) {
  std::vector<PhantomCiphertext> res;
  if (jobs.empty()) return res;
  const size_t chain = jobs[0].a->chain_index();
  for (const MulAddJob& j : jobs)
    if (j.a->chain_index() != chain) throw std::invalid_argument("MulAddRescaleBatch: products at different levels");
  const size_t n = ctx.poly_degree(), L = jobs[0].a->coeff_modulus_size();
  bool positive = true;  // the batched tensor kernel takes a factor >= 1 (the EvalMod products' 1 and 2)
  for (const MulAddJob& j : jobs) positive &= j.factor >= 1;
  if (L > static_cast<size_t>(phx::kMaxScalarLimbs) || !positive) {  // (the per-limb constants travel by value)
    for (const MulAddJob& j : jobs) res.push_back(MulAddRescale(ctx, *j.a, *j.b, rlk, j.factor, j.terms, j.constant));
    return res;
  }
  hipStream_t s = ctx.stream();
  const uint64_t* q = ctx.mod_QP().q;
  for (size_t b0 = 0; b0 < jobs.size(); b0 += phx::kMaxKsProds) {
    const size_t cnt = std::min<size_t>(phx::kMaxKsProds, jobs.size() - b0);
    // the products' tensors side by side in one buffer (the batched modup reads their c2 with one
    // stride); the buffer is freed on this stream after the key switch has read it
    DeviceBuffer<uint64_t> d(cnt * 3 * L * n, s);
    std::vector<double> scales(cnt);
    // the tensors (factor, first term and constant folded in) in shared launches of up to
    // kTensorBatchMax products; further terms (rare) after them
    const auto& mods = ctx.get_context_data(chain).moduli();
    phx::TensorLinBatchArgs tb;
    tb.q = q;
    tb.barrett = ctx.mod_QP().barrett;
    tb.L = static_cast<uint32_t>(L);
    auto flush = [&] {
      if (!tb.count) return;
      hip_ok(phx::tensor_lin_batch(tb, n, s), "tensor + linear epilogue (batch)");
      tb.count = 0;
    };
    for (size_t k = 0; k < cnt; ++k) {
      const MulAddJob& j = jobs[b0 + k];
      if (j.a->chain_index() != j.b->chain_index() || j.a->GetNoiseScaleDeg() > 1 || j.b->GetNoiseScaleDeg() > 1)
        throw std::invalid_argument("MulAddRescale: operands must be level-aligned and of degree 1");
      for (const ScaledTerm& t : j.terms)
        if (t.ct->chain_index() > chain || t.ct->GetNoiseScaleDeg() > 1 || t.ct->size() != 2)
          throw std::invalid_argument("MulAddRescale: a term is below the product's level");
      const double S = j.a->scale() * j.b->scale();
      scales[k] = S;
      if (tb.count == static_cast<uint32_t>(phx::kTensorBatchMax) ||
          (tb.count + 1) * 2 * L > static_cast<size_t>(phx::kTensorBatchLimbWords))
        flush();
      phx::TensorLinJob& tj = tb.job[tb.count];
      uint64_t* cl = tb.limb + static_cast<size_t>(tb.count) * 2 * L;
      tj.ct1 = j.a->data();
      tj.ct2 = j.b->data();
      tj.out = d.get() + k * 3 * L * n;
      tj.factor = static_cast<uint64_t>(j.factor);
      tj.t = nullptr;
      tj.t_stride = 0;
      if (!j.terms.empty()) {
        // round(c S / scale_t) t carries c m_t at the product's scale S
        tj.t = j.terms[0].ct->data();
        tj.t_stride = j.terms[0].ct->coeff_modulus_size() * n;
        for (size_t l = 0; l < L; ++l) cl[l] = residue_of_double(j.terms[0].coeff * S / j.terms[0].ct->scale(), mods[l]);
      }
      tj.has_const = j.constant != 0.0;
      if (tj.has_const)
        for (size_t l = 0; l < L; ++l) cl[L + l] = residue_of_double(j.constant * S, mods[l]);
      ++tb.count;
      traffic::ciphertexts(traffic::limb_bytes(4 * L + 2 * L * j.terms.size(), n));
    }
    flush();
    for (size_t k = 0; k < cnt; ++k) {
      const MulAddJob& j = jobs[b0 + k];
      for (size_t i = 1; i < j.terms.size(); ++i) {
        const ScaledTerm& t = j.terms[i];
        const phx::LimbScalars cb = limb_scalars(ctx, chain, t.coeff * scales[k] / t.ct->scale());
        hip_ok(phx::lin_comb_v(d.get() + k * 3 * L * n, 2, nullptr, t.ct->data(), 2, t.ct->coeff_modulus_size() * n, cb,
                               q, n, L, s),
               "mul-add term");
      }
    }
    std::vector<uint64_t*> outs(cnt);
    for (size_t k = 0; k < cnt; ++k) {
      PhantomCiphertext o;
      o.resize(ctx, chain + 1, 2, s, false);
      outs[k] = o.data();
      res.push_back(std::move(o));
    }
    relinearize_rescale_batch_raw(ctx, chain, d.get(), 3 * L * n, cnt, outs.data(), rlk.public_keys_ptr(), s);
    const double qlast = static_cast<double>(ctx.get_context_data(chain).gpu_rns_tool().base_Ql().back());
    for (size_t k = 0; k < cnt; ++k) {
      PhantomCiphertext& o = res[b0 + k];
      o.set_ntt_form(true);
      o.set_scale(scales[k] / qlast);
      o.set_correction_factor(jobs[b0 + k].a->correction_factor());
      o.SetNoiseScaleDeg(1);
    }
  }
  return res;
}

PhantomCiphertext RelinearizeRescale(const PhantomContext& ctx, const PhantomCiphertext& d, const PhantomRelinKey& rlk) {
  if (d.size() != 3) throw std::invalid_argument("destination_size must be 3");
  if (d.chain_index() + 1 >= ctx.total_parm_size()) throw std::invalid_argument("end of modulus switching chain reached");
  const RnsTool& rt = ctx.get_context_data(d.chain_index()).gpu_rns_tool();
  hipStream_t s = ctx.stream();
  PhantomCiphertext out;
  out.resize(ctx, d.chain_index() + 1, 2, s, false);
  relinearize_rescale_raw(ctx, d.chain_index(), d.data(), out.data(), rlk.public_keys_ptr(), s);
  out.set_ntt_form(true);
  out.set_scale(d.scale() / static_cast<double>(rt.base_Ql().back()));
  out.set_correction_factor(d.correction_factor());
  out.SetNoiseScaleDeg(d.GetNoiseScaleDeg() > 1 ? d.GetNoiseScaleDeg() - 1 : 1);
  return out;
}

PhantomCiphertext KeySwitchDownRescale(const PhantomContext& ctx, PhantomCiphertext& ext) {
  const RnsTool& rt = ctx.get_context_data(ext.chain_index()).gpu_rns_tool();
  const size_t QlP = rt.size_Ql() + ctx.size_P();
  if (ext.size() != 2 || ext.coeff_modulus_size() != QlP) throw std::invalid_argument("not an extended-basis ciphertext");
  if (ext.chain_index() + 1 >= ctx.total_parm_size()) throw std::invalid_argument("end of modulus switching chain reached");
  hipStream_t s = ctx.stream();
  PhantomCiphertext out;
  out.resize(ctx, ext.chain_index() + 1, 2, s, false);
  rt.moddown_rescale(out.data(), ext.data(), ctx.gpu_rns_tables(), s, 2);
  out.set_ntt_form(true);
  out.set_scale(ext.scale() / static_cast<double>(rt.base_Ql().back()));
  out.SetNoiseScaleDeg(ext.GetNoiseScaleDeg() > 1 ? ext.GetNoiseScaleDeg() - 1 : 1);
  return out;
}

PhantomCiphertext MulAddRescale(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomCiphertext& b,
                                const PhantomRelinKey& rlk, int factor, const std::vector<ScaledTerm>& terms,
                                double constant) {
  if (a.chain_index() != b.chain_index() || a.GetNoiseScaleDeg() > 1 || b.GetNoiseScaleDeg() > 1)
    throw std::invalid_argument("MulAddRescale: operands must be level-aligned and of degree 1");
  const size_t n = ctx.poly_degree(), chain = a.chain_index();
  const size_t L = a.coeff_modulus_size();
  hipStream_t s = ctx.stream();
  const uint64_t* q = ctx.mod_QP().q;
  for (const ScaledTerm& t : terms)
    if (t.ct->chain_index() > chain || t.ct->GetNoiseScaleDeg() > 1 || t.ct->size() != 2)
      throw std::invalid_argument("MulAddRescale: a term is below the product's level");
  // tensor product with the factor and the first term fused into one pass
  PhantomCiphertext d;
  d.resize(ctx, chain, 3, s, false);
  d.set_ntt_form(true);
  d.set_correction_factor(a.correction_factor());
  d.set_scale(a.scale() * b.scale());
  const double S = d.scale();
  phx::TensorLinArgs ta;
  ta.ct1 = a.data();
  ta.ct2 = b.data();
  ta.out = d.data();
  ta.q = q;
  ta.barrett = ctx.mod_QP().barrett;
  ta.scale = factor != 1;
  if (ta.scale) ta.f = limb_scalars(ctx, chain, static_cast<double>(factor));
  if (!terms.empty()) {
    // round(c S / scale_t) t carries c m_t at the product's scale S
    ta.t = terms[0].ct->data();
    ta.t_stride = terms[0].ct->coeff_modulus_size() * n;
    ta.c = limb_scalars(ctx, chain, terms[0].coeff * S / terms[0].ct->scale());
  }
  hip_ok(phx::tensor_lin(ta, n, L, s), "tensor + linear epilogue");
  traffic::ciphertexts(traffic::limb_bytes(4 * L + 2 * L * terms.size(), n));  // a, b and the terms read
  for (size_t i = 1; i < terms.size(); ++i) {
    const ScaledTerm& t = terms[i];
    const phx::LimbScalars cb = limb_scalars(ctx, chain, t.coeff * S / t.ct->scale());
    hip_ok(phx::lin_comb_v(d.data(), 2, nullptr, t.ct->data(), 2, t.ct->coeff_modulus_size() * n, cb, q, n, L, s),
           "mul-add term");
  }
  if (constant != 0.0) EvalAddConstInplace(ctx, d, constant);
  d.SetNoiseScaleDeg(2);
  return RelinearizeRescale(ctx, d, rlk);
}

PhantomCiphertext EvalMultRescale(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomCiphertext& b,
                                  const PhantomRelinKey& rlk, const std::vector<double>& sf) {
  const size_t target = std::max(level_after_reduce(a), level_after_reduce(b));
  PhantomCiphertext ta, tb;
  const PhantomCiphertext& x = AtLevel(ctx, a, target, sf, ta);
  const PhantomCiphertext& y = &a == &b ? x : AtLevel(ctx, b, target, sf, tb);
  PhantomCiphertext d = multiply(ctx, x, y);
  d.SetNoiseScaleDeg(2);
  return RelinearizeRescale(ctx, d, rlk);
}

PhantomCiphertext RaiseMod(const PhantomContext& ctx, const PhantomCiphertext& ct, size_t chain_index) {
  if (chain_index < 1 || chain_index >= ctx.total_parm_size()) throw std::invalid_argument("invalid chain index");
  const size_t n = ctx.poly_degree(), L = ct.coeff_modulus_size();
  const size_t Q = ctx.get_context_data(chain_index).coeff_modulus_size();
  hipStream_t s = ctx.stream();
  DeviceBuffer<uint64_t> c(n, s);
  PhantomCiphertext out;
  out.resize(ctx, chain_index, 2, s, false);
  for (size_t i = 0; i < 2; ++i) {
    // limb q0 to coefficient form
    hip_ok(phx::ntt_inverse(ctx.gpu_rns_tables(), ct.data() + i * L * n, c.get(), phx::LimbMap::contiguous(1, 0),
                            nullptr, nullptr, s),
           "raise INTT");
    uint64_t* o = out.data() + i * Q * n;
    hip_ok(phx::switch_modulus_raise(c.get(), o, ctx.mod_QP().q, ctx.mod_QP().barrett, n, Q, s), "raise lift");
    hip_ok(phx::ntt_forward(ctx.gpu_rns_tables(), o, o, phx::LimbMap::contiguous((int)Q, 0), s), "raise NTT");
  }
  out.set_scale(ct.scale());
  out.set_ntt_form(true);
  out.SetNoiseScaleDeg(ct.GetNoiseScaleDeg());
  traffic::ciphertexts(traffic::limb_bytes(2 + 2 * Q, n));
  return out;
}

// ---- hoisted rotations -----------------------------------------------------------------

uint32_t FindAutomorphismIndex2nComplex(int index, size_t n) {
  const int64_t slots = static_cast<int64_t>(n / 2);
  int64_t r = index % slots;
  if (r < 0) r += slots;
  if (r == 0) return 1;
  uint64_t g = 1;
  const uint64_t m = 2 * n;
  uint64_t b = 5;
  for (uint64_t e = static_cast<uint64_t>(r); e; e >>= 1, b = b * b % m)
    if (e & 1) g = g * b % m;
  return static_cast<uint32_t>(g);
}

DeviceBuffer<uint64_t> EvalFastRotationPrecompute(const PhantomContext& ctx, const PhantomCiphertext& ct) {
  const RnsTool& rt = ctx.get_context_data(ct.chain_index()).gpu_rns_tool();
  const size_t n = ctx.poly_degree(), Ql = rt.size_Ql(), QlP = Ql + ctx.size_P();
  DeviceBuffer<uint64_t> digits(rt.beta() * QlP * n, ctx.stream());
  rt.modup(digits.get(), ct.data() + Ql * n, ctx.gpu_rns_tables(), ctx.stream());
  traffic::ciphertexts(traffic::limb_bytes(2 * Ql, n));  // (c0, c1) of the rotated ciphertext read
  return digits;
}

PhantomCiphertext EvalFastAutomorphismExt(const PhantomContext& ctx, const PhantomCiphertext& ct,
                                          const PhantomGaloisKey& keys, uint32_t elt, const uint64_t* digits,
                                          bool add_first) {
  if (ct.size() != 2) throw std::invalid_argument("encrypted size must be 2");
  const RnsTool& rt = ctx.get_context_data(ct.chain_index()).gpu_rns_tool();
  const size_t n = ctx.poly_degree(), Ql = rt.size_Ql(), QlP = Ql + ctx.size_P();
  hipStream_t s = ctx.stream();
  PhantomCiphertext out;
  out.resize(2, QlP, n, s, false);
  out.set_chain_index(ct.chain_index());
  out.set_scale(ct.scale());
  out.SetNoiseScaleDeg(ct.GetNoiseScaleDeg());
  // inner product, + P c0 and the permutation in one pass (the key switch's output never goes to
  // HBM before the permutation)
  phx::KsRotateArgs g;
  g.digits = digits;
  g.evk = keys.get(elt).public_keys_ptr();
  g.qp = ctx.mod_QP().q;
  g.qp_barrett = ctx.mod_QP().barrett;
  g.c0 = ct.data();
  g.pmod = rt.bigP_mod_q();
  g.pmod_shoup = rt.bigP_mod_q_shoup();
  g.out = out.data();
  g.perm = ctx.galois_perm(elt);
  g.ql = static_cast<uint32_t>(Ql);
  g.qlp = static_cast<uint32_t>(QlP);
  g.size_q = static_cast<uint32_t>(ctx.size_Q());
  g.size_p = static_cast<uint32_t>(ctx.size_P());
  g.beta = static_cast<uint32_t>(rt.beta());
  hip_ok(phx::keyswitch_rotate(g, add_first ? 1 : 0, n, s), "fast rotation key switch + permute");
  traffic::keys(traffic::limb_bytes(rt.beta() * 2 * QlP, n));
  traffic::ciphertexts(traffic::limb_bytes(2 * QlP, n));  // the rotated extended ciphertext written
  return out;
}

// inner product, + c0 (P-scaled, extended basis), permutation and accumulation in one pass
static void rotate_ext_accumulate(const PhantomContext& ctx, const RnsTool& rt, const uint64_t* c0,
                                  const uint64_t* digits, const PhantomGaloisKey& keys, uint32_t elt,
                                  PhantomCiphertext& acc, bool accumulate) {
  const size_t n = ctx.poly_degree(), Ql = rt.size_Ql(), QlP = Ql + ctx.size_P();
  phx::KsRotateArgs g;
  g.digits = digits;
  g.evk = keys.get(elt).public_keys_ptr();
  g.qp = ctx.mod_QP().q;
  g.qp_barrett = ctx.mod_QP().barrett;
  g.c0 = c0;
  g.out = acc.data();
  g.perm = ctx.galois_perm(elt);
  g.ql = static_cast<uint32_t>(Ql);
  g.qlp = static_cast<uint32_t>(QlP);
  g.size_q = static_cast<uint32_t>(ctx.size_Q());
  g.size_p = static_cast<uint32_t>(ctx.size_P());
  g.beta = static_cast<uint32_t>(rt.beta());
  g.accumulate = accumulate;
  hip_ok(phx::keyswitch_rotate(g, 2, n, ctx.stream()), "giant step key switch + permute + accumulate");
  traffic::keys(traffic::limb_bytes(rt.beta() * 2 * QlP, n));
}

void EvalRotateExtAccumulate(const PhantomContext& ctx, PhantomCiphertext& ext, const PhantomGaloisKey& keys,
                             int index, PhantomCiphertext& acc, bool accumulate) {
  const RnsTool& rt = ctx.get_context_data(ext.chain_index()).gpu_rns_tool();
  const size_t n = ctx.poly_degree(), Ql = rt.size_Ql(), QlP = Ql + ctx.size_P();
  if (ext.size() != 2 || ext.coeff_modulus_size() != QlP) throw std::invalid_argument("not an extended-basis ciphertext");
  hipStream_t s = ctx.stream();
  const uint32_t elt = FindAutomorphismIndex2nComplex(index, n);
  // only c1 comes down to Ql (it is what the key switch consumes), straight into its digits;
  // c0 stays P-scaled in QlP
  DeviceBuffer<uint64_t> digits(rt.beta() * QlP * n, s);
  rt.moddown_modup(digits.get(), ext.data() + QlP * n, ctx.gpu_rns_tables(), s);
  if (!accumulate) {
    acc.resize(2, QlP, n, s, false);
    acc.set_chain_index(ext.chain_index());
    acc.set_scale(ext.scale());
    acc.SetNoiseScaleDeg(ext.GetNoiseScaleDeg());
    acc.set_ntt_form(true);
  }
  rotate_ext_accumulate(ctx, rt, ext.data(), digits.get(), keys, elt, acc, accumulate);
}

void EvalRotateExtAccumulateDigits(const PhantomContext& ctx, size_t chain, const uint64_t* c0,
                                   const uint64_t* digits, const PhantomGaloisKey& keys, int index,
                                   PhantomCiphertext& acc) {
  const RnsTool& rt = ctx.get_context_data(chain).gpu_rns_tool();
  if (acc.size() != 2 || acc.coeff_modulus_size() != rt.size_Ql() + ctx.size_P())
    throw std::invalid_argument("not an extended-basis accumulator");
  rotate_ext_accumulate(ctx, rt, c0, digits, keys, FindAutomorphismIndex2nComplex(index, ctx.poly_degree()), acc,
                        true);
}

PhantomCiphertext EvalFastRotationExt(const PhantomContext& ctx, const PhantomCiphertext& ct,
                                      const PhantomGaloisKey& keys, int index, const uint64_t* digits,
                                      bool add_first) {
  return EvalFastAutomorphismExt(ctx, ct, keys, FindAutomorphismIndex2nComplex(index, ctx.poly_degree()), digits,
                                 add_first);
}

PhantomCiphertext KeySwitchExt(const PhantomContext& ctx, const PhantomCiphertext& ct) {
  const RnsTool& rt = ctx.get_context_data(ct.chain_index()).gpu_rns_tool();
  const size_t n = ctx.poly_degree(), Ql = rt.size_Ql(), QlP = Ql + ctx.size_P();
  hipStream_t s = ctx.stream();
  PhantomCiphertext out;
  out.resize(2, QlP, n, s, false);
  out.set_chain_index(ct.chain_index());
  out.set_scale(ct.scale());
  out.SetNoiseScaleDeg(ct.GetNoiseScaleDeg());
  PHX_CHECK(hipMemsetAsync(out.data(), 0, 2 * QlP * n * sizeof(uint64_t), s));
  for (size_t i = 0; i < 2; ++i)
    hip_ok(phx::mul_scalar_add(ct.data() + i * Ql * n, rt.bigP_mod_q(), rt.bigP_mod_q_shoup(), nullptr,
                               out.data() + i * QlP * n, ctx.mod_QP().q, n, Ql, s),
           "P c");
  return out;
}

PhantomCiphertext KeySwitchDown(const PhantomContext& ctx, PhantomCiphertext& ext) {
  const RnsTool& rt = ctx.get_context_data(ext.chain_index()).gpu_rns_tool();
  const size_t Ql = rt.size_Ql(), QlP = Ql + ctx.size_P();
  if (ext.coeff_modulus_size() != QlP) throw std::invalid_argument("not an extended-basis ciphertext");
  hipStream_t s = ctx.stream();
  PhantomCiphertext out;
  out.resize(ctx, ext.chain_index(), 2, s, false);
  rt.moddown_add(out.data(), ext.data(), false, ctx.gpu_rns_tables(), s, 2);
  traffic::ciphertexts(traffic::limb_bytes(2 * QlP + 2 * Ql, ctx.poly_degree()));
  out.set_scale(ext.scale());
  out.SetNoiseScaleDeg(ext.GetNoiseScaleDeg());
  out.set_ntt_form(true);
  return out;
}

PhantomCiphertext KeySwitchDown(const PhantomContext& ctx, const PhantomCiphertext& ext) {
  PhantomCiphertext t = ext;  // the moddown uses its input's P limbs as scratch
  return KeySwitchDown(ctx, t);
}

PhantomCiphertext KeySwitchDownFirstElement(const PhantomContext& ctx, const PhantomCiphertext& ext) {
  const RnsTool& rt = ctx.get_context_data(ext.chain_index()).gpu_rns_tool();
  const size_t n = ctx.poly_degree(), Ql = rt.size_Ql(), QlP = Ql + ctx.size_P();
  if (ext.coeff_modulus_size() != QlP) throw std::invalid_argument("not an extended-basis ciphertext");
  hipStream_t s = ctx.stream();
  // moddown_from_NTT of the first polynomial alone (src/evaluate.cu:2875-2892), from a copy of it
  // (the moddown uses its input's P limbs as scratch; the argument stays intact)
  DeviceBuffer<uint64_t> c0(QlP * n, s);
  PHX_CHECK(hipMemcpyAsync(c0.get(), ext.data(), QlP * n * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
  PhantomCiphertext out;
  out.resize(ctx, ext.chain_index(), 1, s, false);
  rt.moddown_add(out.data(), c0.get(), false, ctx.gpu_rns_tables(), s, 1);
  out.set_scale(ext.scale());
  out.SetNoiseScaleDeg(ext.GetNoiseScaleDeg());
  out.set_ntt_form(true);
  return out;
}

// one launch over both polynomials of an extended-basis ciphertext (moduli Ql u P)
static void ext_binary(const PhantomContext& ctx, size_t chain, uint64_t* a, const uint64_t* b, size_t b_stride,
                       size_t polys, bool mul) {
  const RnsTool& rt = ctx.get_context_data(chain).gpu_rns_tool();
  const size_t n = ctx.poly_degree(), QlP = rt.size_Ql() + ctx.size_P();
  if (mul) hip_ok(phx::poly_mul(a, b, a, rt.mod_QlP(), n, QlP, ctx.stream(), polys, b_stride), "ext mul");
  else hip_ok(phx::poly_add(a, b, a, rt.mod_QlP(), n, QlP, ctx.stream(), polys, b_stride), "ext add");
}

void EvalMultExtInPlace(const PhantomContext& ctx, PhantomCiphertext& ext, const PhantomPlaintext& pt) {
  if (ext.chain_index() != pt.chain_index()) throw std::invalid_argument("Eval Mult Ext: chain index mismatch");
  const size_t Ql = ctx.get_context_data(ext.chain_index()).coeff_modulus_size();
  if (pt.coeff_modulus_size() != Ql + ctx.size_P() || ext.coeff_modulus_size() != Ql + ctx.size_P())
    throw std::invalid_argument("Eval Mult Ext: operands are not in the extended basis");
  ext_binary(ctx, ext.chain_index(), ext.data(), pt.data(), 0, 2, true);
  ext.set_scale(ext.scale() * pt.scale());
  ext.SetNoiseScaleDeg(ext.GetNoiseScaleDeg() + pt.GetNoiseScaleDeg());
}

void EvalAddExtInPlace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b) {
  if (a.chain_index() != b.chain_index() || a.GetNoiseScaleDeg() != b.GetNoiseScaleDeg())
    throw std::invalid_argument("Eval Add Ext Failed.");
  const size_t Ql = ctx.get_context_data(a.chain_index()).coeff_modulus_size();
  ext_binary(ctx, a.chain_index(), a.data(), b.data(), (Ql + ctx.size_P()) * ctx.poly_degree(), 2, false);
}

PhantomCiphertext EvalRotateFused(const PhantomContext& ctx, const PhantomCiphertext& ct, const PhantomGaloisKey& keys,
                                  int index) {
  DeviceBuffer<uint64_t> d = EvalFastRotationPrecompute(ctx, ct);
  PhantomCiphertext e = EvalFastRotationExt(ctx, ct, keys, index, d.get(), true);
  return KeySwitchDown(ctx, e);
}

PhantomCiphertext EvalConjFused(const PhantomContext& ctx, const PhantomCiphertext& ct, const PhantomGaloisKey& keys) {
  DeviceBuffer<uint64_t> d = EvalFastRotationPrecompute(ctx, ct);
  PhantomCiphertext e =
      EvalFastAutomorphismExt(ctx, ct, keys, static_cast<uint32_t>(2 * ctx.poly_degree() - 1), d.get(), true);
  return KeySwitchDown(ctx, e);
}

}  // namespace phantom
