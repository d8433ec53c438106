// ckks_eval.h — the CKKS evaluator pieces the bootstrap is built from (the helpers of
// src/evaluate.cu:2284-2554 and :3631-3940 in the reference), with FLEXIBLEAUTO scale management
// (PhantomCiphertext::PreComputeScale, include/ciphertext.h:320-367).
//
// Conventions: level(ct) = chain_index - 1 (the number of dropped primes).  A ciphertext at
// level l with noise-scale degree 1 carries scale sf[l]; a product has degree 2 and scale
// sf[l]^2, and a rescale divides by the dropped prime: sf[l]^2 / q = sf[l+1].
//
// Extended-basis ("Ext") ciphertexts are [2][size_Ql + size_P][n] NTT-form polynomials that
// hold P * (c0, c1) (+ key-switch terms); KeySwitchDown divides by P and returns to Ql.
#pragma once

#include <complex>
#include <cstdint>
#include <functional>
#include <memory>
#include <vector>

#include "ciphertext.h"
#include "context.h"
#include "keys.h"

namespace phantom {

inline size_t level_of(const PhantomCiphertext& ct) { return ct.chain_index() - 1; }

// FLEXIBLEAUTO scaling factors per level (PreComputeScale): sf[0] = q_{L-1}, sf[k] = sf[k-1]^2 / q_{L-k}
std::vector<double> precompute_scaling_factors(const PhantomContext& ctx, double scale);

// residues of round(k) modulo every prime of `chain` (v), with Shoup quotients (vs, optional)
void ScalarResidues(const PhantomContext& ctx, size_t chain, double k, uint64_t* v, uint64_t* vs);
// multiply every polynomial by round(k) (exact residues of a double; scale metadata unchanged)
void mult_by_real_integer_inplace(const PhantomContext& ctx, PhantomCiphertext& ct, double k);
// MultByIntegerInPlace (src/evaluate.cu:3942-3970)
void MultByIntegerInPlace(const PhantomContext& ctx, PhantomCiphertext& ct, uint64_t k);
// GetElementForEvalMult (src/evaluate.cu:2332-2412): residues of round(c * sf[level]) as the
// reference rounds it (125-bit window, half up)
std::vector<uint64_t> GetElementForEvalMult(const PhantomContext& ctx, const PhantomCiphertext& ct, double c,
                                            const std::vector<double>& sf);
// EvalMultConstInplaceCore (src/evaluate.cu:2299-2330): times round(c * sf[level]), degree + 1,
// scale times sf[level]
void EvalMultConstInplaceCore(const PhantomContext& ctx, PhantomCiphertext& ct, double c, const std::vector<double>& sf);
// EvalMultConstInplace (include/evaluate.cuh:317-326): a degree-2 input is rescaled first (the
// lazy rescale that lets bootstrapping_example.cu:150-153 call it 25 times in a row), then Core
void EvalMultConstInplace(const PhantomContext& ctx, PhantomCiphertext& ct, double c, const std::vector<double>& sf);
inline PhantomCiphertext EvalMultConst(const PhantomContext& ctx, const PhantomCiphertext& ct, double c,
                                       const std::vector<double>& sf) {
  PhantomCiphertext d = ct;
  EvalMultConstInplace(ctx, d, c, sf);
  return d;
}
inline PhantomCiphertext EvalMultConstCore(const PhantomContext& ctx, const PhantomCiphertext& ct, double c,
                                           const std::vector<double>& sf) {
  return EvalMultConst(ctx, ct, c, sf);
}
// add the constant c to every slot (c * scale on the constant coefficient)
void EvalAddConstInplace(const PhantomContext& ctx, PhantomCiphertext& ct, double c);
// MultByMonomialInPlace (src/evaluate.cu:2505-2554): times X^power (slots times zeta^(power 5^j))
void MultByMonomialInPlace(const PhantomContext& ctx, PhantomCiphertext& ct, uint32_t power);
// rescale once, degree - 1 (ModReduce / EvalModReduceInPlace, src/evaluate.cu:2284-2297)
void EvalModReduceInPlace(const PhantomContext& ctx, PhantomCiphertext& ct, size_t levels = 1);
// bring a degree-1 (or 2) ciphertext to `target_level` with scale sf[target_level]: mod-switch,
// then one scaling multiply + rescale (AdjustLevelsAndDepth of FLEXIBLEAUTO)
void AdjustToLevel(const PhantomContext& ctx, PhantomCiphertext& ct, size_t target_level,
                   const std::vector<double>& sf);
// round(k) * (the leading limbs of ct at `chain`) as a new ciphertext, one kernel (metadata of
// ct; the caller sets the scale)
PhantomCiphertext ScaledModSwitch(const PhantomContext& ctx, const PhantomCiphertext& ct, size_t chain, double k);
// acc += round(k) * ct, ct at acc's level or above (its extra limbs are ignored); one kernel
void AccumulateScaled(const PhantomContext& ctx, PhantomCiphertext& acc, const PhantomCiphertext& ct, double k);
// `ct` at noise degree 1 and level `target` (>= its level after one rescale): ct itself when it
// already is, else a new ciphertext stored in `tmp` (no copy when nothing is to be done)
const PhantomCiphertext& AtLevel(const PhantomContext& ctx, const PhantomCiphertext& ct, size_t target,
                                 const std::vector<double>& sf, PhantomCiphertext& tmp);
// AtLevel for many ciphertexts at once (their targets may differ): result k is empty when cts[k]
// already is at targets[k] (use it as it is), else a new ciphertext; those of one target level
// share one batched rescale.  Bit-identical to AtLevel.
std::vector<PhantomCiphertext> AtLevelBatch(const PhantomContext& ctx, const std::vector<const PhantomCiphertext*>& cts,
                                            const std::vector<size_t>& targets, const std::vector<double>& sf);
// EvalAddAutoInplace / EvalSubAuto: level- and scale-aligned add / subtract
void EvalAddAutoInplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b,
                        const std::vector<double>& sf);
void EvalSubAutoInplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b,
                        const std::vector<double>& sf);
// relinearize a 3-polynomial product and rescale it in one key-switch: (c0, c1) + KS(c2) is formed
// P-scaled in the extended basis and divided by P q_last at once (RnsTool::moddown_rescale)
PhantomCiphertext RelinearizeRescale(const PhantomContext& ctx, const PhantomCiphertext& d3, const PhantomRelinKey& rlk);
// the same on raw device buffers: d3 [3][Ql][n] at chain_index -> out [2][Ql - 1][n];
// evk: device array of the relinearization key's digit pointers
void relinearize_rescale_raw(const PhantomContext& ctx, size_t chain_index, const uint64_t* d3, uint64_t* out,
                             const uint64_t* const* evk, hipStream_t s);
// KeySwitchDown followed by a rescale, as one division by P q_last
PhantomCiphertext KeySwitchDownRescale(const PhantomContext& ctx, PhantomCiphertext& ext);
// rescale(relinearize(factor a b + sum_t coeff_t t + constant)) with one key switch: every term
// t (degree 1, at the product's level or above, i.e. with at least its limbs) is brought to the
// product's scale by an integer multiply before the rescale, so it costs no rescale of its own
// (the FLEXIBLEAUTO alignment would rescale it: AdjustToLevel).  a and b: degree 1, same level.
struct ScaledTerm {
  const PhantomCiphertext* ct;
  double coeff;
};
PhantomCiphertext MulAddRescale(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomCiphertext& b,
                                const PhantomRelinKey& rlk, int factor, const std::vector<ScaledTerm>& terms,
                                double constant);
// `count` MulAddRescale products at one level in shared launches: every stage of the key switch
// (modup INTT, digit conversions and NTTs, the moddown-rescale with its fused inner products) runs
// once over all of them.  Bit-identical to calling MulAddRescale on each job.
struct MulAddJob {
  const PhantomCiphertext* a;
  const PhantomCiphertext* b;
  int factor = 1;
  std::vector<ScaledTerm> terms;
  double constant = 0.0;
};
std::vector<PhantomCiphertext> MulAddRescaleBatch(const PhantomContext& ctx, const std::vector<MulAddJob>& jobs,
                                                  const PhantomRelinKey& rlk);
// relinearize + rescale of `count` products d3 + k d3_stride ([3][Ql][n] each) into out[k]
// ([2][Ql - 1][n]); count <= phx::kMaxKsProds
void relinearize_rescale_batch_raw(const PhantomContext& ctx, size_t chain_index, const uint64_t* d3,
                                   size_t d3_stride, size_t count, uint64_t* const* out, const uint64_t* const* evk,
                                   hipStream_t s);
// level-aligned multiply + relinearize + rescale (EvalMultAuto + ModReduce)
PhantomCiphertext EvalMultRescale(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomCiphertext& b,
                                  const PhantomRelinKey& rlk, const std::vector<double>& sf);

// RaiseMod (src/evaluate.cu:2459-2503): limb q0 of a ciphertext -> the full chain Q (chain 1),
// or the leading limbs of chain `chain_index`; centered lift; NTT form in and out.
PhantomCiphertext RaiseMod(const PhantomContext& ctx, const PhantomCiphertext& ct, size_t chain_index = 1);

// ---- hoisted rotations (src/evaluate.cu:3631-3940) ------------------------------------
// EvalFastRotationPrecompute: modup of c1, [beta][size_QlP][n]
DeviceBuffer<uint64_t> EvalFastRotationPrecompute(const PhantomContext& ctx, const PhantomCiphertext& ct);
// EvalFastRotationExt: rotation by `index` slots in the extended basis from shared digits, with
// a fused key (PhantomSecretKey::create_galois_keys_fused); add_first adds P * c0.
PhantomCiphertext EvalFastRotationExt(const PhantomContext& ctx, const PhantomCiphertext& ct,
                                      const PhantomGaloisKey& fused_keys, int index, const uint64_t* digits,
                                      bool add_first);
// the same for an explicit Galois element (conjugation: 2N - 1)
PhantomCiphertext EvalFastAutomorphismExt(const PhantomContext& ctx, const PhantomCiphertext& ct,
                                          const PhantomGaloisKey& fused_keys, uint32_t galois_elt,
                                          const uint64_t* digits, bool add_first);
// Giant step of a hoisted linear transform: acc (+)= rotation by `index` of the extended-basis
// ciphertext `ext` (P-scaled, as EvalFastRotationExt outputs and their plaintext products are).
// Only c1 is brought down to Ql, key switched and permuted; c0 is added in the extended basis
// (one moddown instead of two, and no rounding of c0).  `ext`'s c1 P limbs are clobbered;
// accumulate = false initialises acc.
void EvalRotateExtAccumulate(const PhantomContext& ctx, PhantomCiphertext& ext, const PhantomGaloisKey& fused_keys,
                             int index, PhantomCiphertext& acc, bool accumulate);
// its key switch alone, from digits already computed (RnsTool::moddown_modup of c1, batched over
// the giant steps of a level): acc (+)= rotation of (c0 + KeySwitch(digits)); c0 [QlP][n] is the
// extended ciphertext's first polynomial at chain index `chain`.  acc must be initialised.
void EvalRotateExtAccumulateDigits(const PhantomContext& ctx, size_t chain, const uint64_t* c0,
                                   const uint64_t* digits, const PhantomGaloisKey& fused_keys, int index,
                                   PhantomCiphertext& acc);
// KeySwitchExt: (c0, c1) -> P * (c0, c1) in the extended basis
PhantomCiphertext KeySwitchExt(const PhantomContext& ctx, const PhantomCiphertext& ct);
// KeySwitchDown: extended -> Ql (moddown of both polynomials); `ext` is consumed (its P limbs
// are clobbered)
PhantomCiphertext KeySwitchDown(const PhantomContext& ctx, PhantomCiphertext& ext);
// the reference's const form (include/evaluate.cuh:347): the argument is copied first
PhantomCiphertext KeySwitchDown(const PhantomContext& ctx, const PhantomCiphertext& ext);
// KeySwitchDownFirstElement (include/evaluate.cuh:349, src/evaluate.cu:2875-2892): the moddown of
// the extended-basis ciphertext's first polynomial alone, a one-polynomial ciphertext over Ql
PhantomCiphertext KeySwitchDownFirstElement(const PhantomContext& ctx, const PhantomCiphertext& ext);
// EvalMultExtInPlace / EvalAddExtInPlace over Ql u P
void EvalMultExtInPlace(const PhantomContext& ctx, PhantomCiphertext& ext, const PhantomPlaintext& pt_ext);
void EvalAddExtInPlace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b);
// the value forms (include/evaluate.cuh:458-475)
inline PhantomCiphertext EvalMultExt(const PhantomContext& ctx, const PhantomCiphertext& ext, const PhantomPlaintext& pt) {
  PhantomCiphertext d = ext;
  EvalMultExtInPlace(ctx, d, pt);
  return d;
}
inline PhantomCiphertext EvalAddExt(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomCiphertext& b) {
  PhantomCiphertext d = a;
  EvalAddExtInPlace(ctx, d, b);
  return d;
}
// rotation / conjugation through the hoisted path (one key switch)
PhantomCiphertext EvalRotateFused(const PhantomContext& ctx, const PhantomCiphertext& ct,
                                  const PhantomGaloisKey& fused_keys, int index);
PhantomCiphertext EvalConjFused(const PhantomContext& ctx, const PhantomCiphertext& ct,
                                const PhantomGaloisKey& fused_keys);
// the reference's argument order (include/evaluate.cuh: EvalRotateFused(context, keys, in, out, index),
// EvalConjFused(context, keys, in, out))
inline void EvalRotateFused(const PhantomContext& ctx, const PhantomGaloisKey& fused_keys, const PhantomCiphertext& in,
                            PhantomCiphertext& out, int index) {
  out = EvalRotateFused(ctx, in, fused_keys, index);
}
inline void EvalConjFused(const PhantomContext& ctx, const PhantomGaloisKey& fused_keys, const PhantomCiphertext& in,
                          PhantomCiphertext& out) {
  out = EvalConjFused(ctx, in, fused_keys);
}

// Galois element of a slot rotation (FindAutomorphismIndex2nComplex, src/util.cu:908-935)
uint32_t FindAutomorphismIndex2nComplex(int index, size_t n);

// ---- the reference's FLEXIBLEAUTO surface (include/evaluate.cuh:270-452; host/flexauto.cpp) ----
// sf = getScalingFactorsReal(), sfBig = getScalingFactorsRealBig() (PreComputeScale).  These keep
// the reference's degree bookkeeping: products are left at degree 2 and rescaled lazily.
// ModReduce (src/evaluate.cu:2284-2297): a rescaled copy (levels > 1 rescales that many times;
// the reference rescales the same input repeatedly, i.e. once)
PhantomCiphertext ModReduce(const PhantomContext& ctx, const PhantomCiphertext& ct, size_t levels);
// ModSwitchLevelInPlace (include/evaluate.cuh:304-312): drop `levels` limbs, degree kept
void ModSwitchLevelInPlace(const PhantomContext& ctx, PhantomCiphertext& ct, size_t levels);
// AdjustLevelsAndDepthInPlace (src/evaluate.cu:2611-2779): the lower operand is brought to the
// other's level, degree and scale
void AdjustLevelsAndDepthInPlace(const PhantomContext& ctx, PhantomCiphertext& c1, PhantomCiphertext& c2,
                                 const std::vector<double>& sf, const std::vector<double>& sfBig);
// EvalMultAuto (src/evaluate.cu:2794-2811): adjust, rescale degree-2 operands, multiply + relin;
// the result has degree deg1 + deg2 (not rescaled)
PhantomCiphertext EvalMultAuto(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomCiphertext& b,
                               const PhantomRelinKey& rlk, const std::vector<double>& sf,
                               const std::vector<double>& sfBig);
// EvalMultAutoInplace with a plaintext (src/evaluate.cu:2813-2825) and EvalMultBroadcast (:2827-2854)
void EvalMultAutoInplace(const PhantomContext& ctx, PhantomCiphertext& ct, const PhantomPlaintext& pt,
                         const std::vector<double>& sf, const std::vector<double>& sfBig);
void EvalMultBroadcast(const PhantomContext& ctx, PhantomCiphertext& ct, const PhantomCiphertext& single);
// EvalSquare (src/evaluate.cu:3611-3629): squaring kernel + relin, degree doubled
PhantomCiphertext EvalSquare(const PhantomContext& ctx, const PhantomCiphertext& ct, const PhantomRelinKey& rlk,
                             const std::vector<double>& sf, const std::vector<double>& sfBig);
inline void EvalSquareInPlace(const PhantomContext& ctx, PhantomCiphertext& ct, const PhantomRelinKey& rlk,
                              const std::vector<double>& sf, const std::vector<double>& sfBig) {
  ct = EvalSquare(ctx, ct, rlk, sf, sfBig);
}
// EvalAddAutoInplace / EvalSubAutoInplace with the reference's adjustment (src/evaluate.cu:2856-2873)
void EvalAddAutoInplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b,
                        const std::vector<double>& sf, const std::vector<double>& sfBig);
void EvalSubAutoInplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b,
                        const std::vector<double>& sf, const std::vector<double>& sfBig);
inline PhantomCiphertext EvalAddAuto(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomCiphertext& b,
                                     const std::vector<double>& sf, const std::vector<double>& sfBig) {
  PhantomCiphertext d = a;
  EvalAddAutoInplace(ctx, d, b, sf, sfBig);
  return d;
}
inline PhantomCiphertext EvalSubAuto(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomCiphertext& b,
                                     const std::vector<double>& sf, const std::vector<double>& sfBig) {
  PhantomCiphertext d = a;
  EvalSubAutoInplace(ctx, d, b, sf, sfBig);
  return d;
}
// GetElementForEvalAddOrSub / EvalAddConstInPlace / EvalSubConstInPlace (src/evaluate.cu:2894-2996):
// the constant at scale sf[level]^degree added to c0; operand >= 0 (EvalAddConstInPlaceWrap
// dispatches on the sign, include/evaluate.cuh:425-443)
std::vector<uint64_t> GetElementForEvalAddOrSub(const PhantomContext& ctx, const PhantomCiphertext& ct, double operand,
                                                const std::vector<double>& sf, const std::vector<double>& sfBig);
void EvalAddConstInPlace(const PhantomContext& ctx, PhantomCiphertext& ct, double operand, const std::vector<double>& sf,
                         const std::vector<double>& sfBig);
void EvalSubConstInPlace(const PhantomContext& ctx, PhantomCiphertext& ct, double operand, const std::vector<double>& sf,
                         const std::vector<double>& sfBig);
void EvalAddConstInPlaceWrap(const PhantomContext& ctx, PhantomCiphertext& ct, double operand,
                             const std::vector<double>& sf, const std::vector<double>& sfBig);
inline PhantomCiphertext EvalAddConst(const PhantomContext& ctx, const PhantomCiphertext& ct, double operand,
                                      const std::vector<double>& sf, const std::vector<double>& sfBig) {
  PhantomCiphertext d = ct;
  EvalAddConstInPlaceWrap(ctx, d, operand, sf, sfBig);
  return d;
}
// ConvertToEval / ConvertToCoeff (src/evaluate.cu:2556-2609): NTT / INTT of every polynomial
void ConvertToEval(const PhantomContext& ctx, PhantomCiphertext& ct);
void ConvertToCoeff(const PhantomContext& ctx, PhantomCiphertext& ct);
// EvalChebyshevCoefficients (src/evaluate.cu:3585-3609): degree + 1 coefficients of func on [a, b]
// (coefficient 0 not halved)
std::vector<double> EvalChebyshevCoefficients(const std::function<double(double)>& func, double a, double b,
                                              uint32_t degree);
// EvalChebyshevSeries (src/evaluate.cu:3176-3186): sum c_k T_k((2x - a - b) / (b - a)) with c_0
// halved.  Degree < 5: the reference's linear method (EvalChebyshevSeriesLinear, :3188-3262);
// otherwise the reference's Paterson-Stockmeyer split (EvalChebyshevSeriesPS, :3264-3535, and
// InnerEvalChebyshevPS, :2998-3174; host/chebyshev_ps.cpp), the same operation sequence through
// the FLEXIBLEAUTO helpers above, so the result's level, degree and scale are the reference's.
// (The bootstrap's EvalMod uses its own fused evaluator, host/bootstrap.cpp.)
PhantomCiphertext EvalChebyshevSeries(const PhantomContext& ctx, const PhantomRelinKey& rlk, const PhantomCiphertext& x,
                                      const std::vector<double>& coeffs, double a, double b,
                                      const std::vector<double>& sf, const std::vector<double>& sfBig);
PhantomCiphertext EvalChebyshevSeriesLinear(const PhantomContext& ctx, const PhantomRelinKey& rlk,
                                            const PhantomCiphertext& x, const std::vector<double>& coeffs, double a,
                                            double b, const std::vector<double>& sf, const std::vector<double>& sfBig);
PhantomCiphertext EvalChebyshevSeriesPS(const PhantomContext& ctx, const PhantomRelinKey& rlk, const PhantomCiphertext& x,
                                        const std::vector<double>& coeffs, double a, double b,
                                        const std::vector<double>& sf, const std::vector<double>& sfBig);
// the reference's [-1, 1] test of the series interval (src/evaluate.cu:3208): signed differences
bool ChebyshevUnitInterval(double a, double b);
// EvalLinearWSumMutable (include/evaluate.cuh:371, src/evaluate.cu:3537-3583): sum w_i ct_i after
// bringing every ct_i to the deepest one's level and degree (the operands are adjusted in place)
PhantomCiphertext EvalLinearWSumMutable(const PhantomContext& ctx, std::vector<PhantomCiphertext*>& cts,
                                        const std::vector<double>& w, const std::vector<double>& sf,
                                        const std::vector<double>& sfBig);
// the reference's argument type (shared pointers, adjusted in place the same way)
PhantomCiphertext EvalLinearWSumMutable(const PhantomContext& ctx, std::vector<std::shared_ptr<PhantomCiphertext>>& cts,
                                        const std::vector<double>& w, const std::vector<double>& sf,
                                        const std::vector<double>& sfBig);
// the Paterson-Stockmeyer host helpers of src/util.cu:15-312
namespace ps {
struct Division {
  std::vector<double> q, r;
};
uint32_t Degree(const std::vector<double>& c);  // last non-zero index (0 when all are zero)
uint32_t GetDepthByDegree(size_t degree);        // degrees 5 .. 2031
uint32_t GetMultiplicativeDepthByCoeffVector(const std::vector<double>& vec, bool isNormalized);
std::vector<uint32_t> ComputeDegreesPS(uint32_t n);  // {k, m}
Division LongDivisionChebyshev(const std::vector<double>& f, const std::vector<double>& g);
Division LongDivisionPoly(const std::vector<double>& f, const std::vector<double>& g);  // power basis
}  // namespace ps
// EvalChebyshevFunction (include/evaluate.cuh:381-388)
inline PhantomCiphertext EvalChebyshevFunction(const std::function<double(double)>& func, const PhantomContext& ctx,
                                               const PhantomRelinKey& rlk, const PhantomCiphertext& ct, double a,
                                               double b, uint32_t degree, const std::vector<double>& sf,
                                               const std::vector<double>& sfBig) {
  return EvalChebyshevSeries(ctx, rlk, ct, EvalChebyshevCoefficients(func, a, b, degree), a, b, sf, sfBig);
}

}  // namespace phantom
