// bootstrap.h — CKKS bootstrapping (FHECKKSRNS, include/bootstrap.cuh + src/bootstrap.cu of the
// reference): ModRaise -> CoeffToSlot -> conjugate split -> EvalMod (Chebyshev series of a scaled
// cosine + double-angle iterations) -> SlotToCoeff, full packing (slots = N/2), FLEXIBLEAUTO
// scaling, hoisted baby-step/giant-step linear transforms in the extended basis.
//
// The linear maps are this engine's own factorisation of the canonical-embedding matrix U
// (U[j][k] = zeta^(5^j k), zeta = exp(2 pi i / 2N), k < N/2): a radix-2 decimation-in-time
// recursion whose stage s (block size m = 2^s) is a slot-domain butterfly with twiddles
// zeta_m^(5^j) and rotations by +-m/2.  CoeffToSlot applies the inverse stages top-down and
// leaves the coefficients in bit-reversed slot order; SlotToCoeff applies the stages bottom-up
// from that order, so no permutation is ever evaluated.  `levelBudget` groups the log2(N/2)
// stages into that many levels (reference: bootstrap.cu:181-560, GetCollapsedFFTParams).
#pragma once

#include <complex>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "ciphertext.h"
#include "ckks_eval.h"
#include "context.h"
#include "encoder.h"
#include "keys.h"
#include "../csrc/ckks.h"

namespace phantom {

namespace boot {
using cvec = std::vector<std::complex<double>>;
// a slot-domain linear map as diagonals: (T v)[p] = sum_a diag_a[p] v[p + a]  (a mod slots)
using DiagMap = std::map<int, cvec>;

// stage s (1 <= s <= log2 slots) of U's factorisation, or its inverse
DiagMap stage(size_t slots, int s, bool inverse);
// A * B (B applied first)
DiagMap compose(const DiagMap& A, const DiagMap& B, size_t slots);
// a map T on n slots applied to every n-block of an S-slot vector independently (S a multiple of
// n): each diagonal of T becomes the within-block offsets it really is, so the result is correct
// on inputs that are not n-periodic.  out_mask (period 2n) scales output slot p, in_mask (period
// 2n) input slot q; null = 1.
DiagMap lift_blocks(const DiagMap& T, size_t n, size_t S, const cvec* out_mask, const cvec* in_mask);
// apply a DiagMap to a vector (tests)
cvec apply(const DiagMap& T, const cvec& v);
// Chebyshev interpolation coefficients of f on [-1, 1] (p(y) = sum_k c_k T_k(y), c_0 not halved)
std::vector<double> chebyshev_coefficients(double (*f)(double, const double*), const double* args, int degree);
// the EvalMod target before the double-angle iterations: (2 pi)^(-2^-r) cos(2 pi (K y - 1/4) / 2^r)
double scaled_cosine(double y, const double* args /* {K, r} */);
}  // namespace boot

// device copies of the Chebyshev leaf constant tables, keyed by content (they depend only on
// the levels and scales the evaluation reaches, the same for every bootstrap)
class LeafTableCache {
 public:
  const uint64_t* get(const std::vector<uint64_t>& table, hipStream_t s);

 private:
  std::mutex mu_;
  std::map<std::vector<uint64_t>, DeviceBuffer<uint64_t>> tables_;
};

struct LevelWork;  // one linear-transform level's working buffers (bootstrap.cpp)

class FHECKKSRNS {
 public:
  explicit FHECKKSRNS(PhantomCKKSEncoder& encoder);

  // EvalBootstrapSetup (bootstrap.cu:15-181, include/bootstrap.cuh:98-101): linear-transform
  // plaintexts and EvalMod constants for `slots` slots (0: N/2, full packing; a power of two below
  // N/2: sparse packing).  `sf` are the FLEXIBLEAUTO scaling factors (PreComputeScale).  dim1:
  // baby-step sizes {CoeffToSlot, SlotToCoeff} of the baby-step giant-step evaluation (0: chosen
  // per level).  Setups for several slot counts coexist (the reference's m_bootPrecomMap).
  void EvalBootstrapSetup(const PhantomContext& cc, const std::vector<uint32_t>& levelBudget, double scale,
                          const std::vector<double>& sf, uint32_t correctionFactor = 0, uint32_t slots = 0,
                          const std::vector<uint32_t>& dim1 = {0, 0});
  // the reference's argument list (bootstrap.cu:15-18).  scalingFactorsRealBig must be the
  // FLEXIBLEAUTO squares of scalingFactorsReal (ciphertext.h:357-365; PreComputeScale makes them
  // so): other values throw std::invalid_argument instead of being ignored, and the factors are
  // kept (scaling_factors_big()).  precompute = false sets up the level structure (what
  // EvalBootstrapKeyGen needs, as the reference's m_paramsEnc / m_paramsDec) and defers the
  // linear-transform plaintexts to the first EvalBootstrap of that slot count (the reference
  // skips them, bootstrap.cu:87, and would then bootstrap with empty transforms).
  void EvalBootstrapSetup(const PhantomContext& cc, const std::vector<uint32_t>& levelBudget, double scale,
                          const std::vector<double>& sf, const std::vector<double>& sf_big,
                          const std::vector<uint32_t>& dim1 = {0, 0}, uint32_t slots = 0,
                          uint32_t correctionFactor = 0, bool precompute = true);
  // EvalBootstrapKeyGen / EvalMultKeyGen (bootstrap.cu:566-841): fused rotation keys for the
  // baby/giant steps, the sparse partial sums and conjugation, and the relinearization key.
  void EvalBootstrapKeyGen(PhantomSecretKey& sk, const PhantomContext& cc, uint32_t numSlots = 0);
  void EvalMultKeyGen(PhantomSecretKey& sk, const PhantomContext& cc);
  // fused rotation keys for further slot rotations (e.g. FindLinearTransformRotationIndices for
  // EvalLinearTransform); keys already held are kept
  void EvalRotationKeyGen(PhantomSecretKey& sk, const PhantomContext& cc, const std::vector<int32_t>& indices);
  // EvalBootstrap (bootstrap.cu:843-1129); the input needs at least two limbs.  numSlots: the
  // setup to use (0: N/2).  numIterations > 1: iterative bootstrapping (bootstrap.cu:856-900):
  // bootstrap, scale the residual error up by 2^precision, bootstrap it and subtract.
  PhantomCiphertext EvalBootstrap(const PhantomCiphertext& ct, const PhantomContext& cc, uint32_t numSlots = 0,
                                  uint32_t numIterations = 1, uint32_t precision = 0) const;
  // EvalBootstrapBatch's default lockstep group (a run-time choice: the group argument below,
  // phantom_boot_run_grouped at the C-ABI)
  static constexpr size_t kBootGroup = 8;
  static_assert(kBootGroup >= 1 && kBootGroup <= 8, "lockstep groups hold 1 to phx::kLtGroupMax ciphertexts");
  // a batch of independent bootstraps, `lanes` at a time side by side (each on its own thread
  // and stream lane, PhantomContext::kLanes at most), each lane `group` ciphertexts at a time in
  // lockstep (1..8; groups of 8 on 3 lanes: 56.8/s holding 86 GiB, groups of 4 on 4 lanes: 55.6/s
  // holding 79 GiB, profiles/r05/c5_pool/); the results are ordered
  // on cc.stream()
  std::vector<PhantomCiphertext> EvalBootstrapBatch(const std::vector<PhantomCiphertext>& in,
                                                    const PhantomContext& cc, int lanes, uint32_t numSlots = 0,
                                                    size_t group = kBootGroup) const;

  // stages, exposed for tests and the benchmark (full packing setup unless numSlots is given)
  PhantomCiphertext EvalCoeffsToSlots(const PhantomCiphertext& ct, const PhantomContext& cc,
                                      uint32_t numSlots = 0) const;
  PhantomCiphertext EvalSlotsToCoeffs(const PhantomCiphertext& ct, const PhantomContext& cc,
                                      uint32_t numSlots = 0) const;
  PhantomCiphertext EvalChebyshevSeries(const PhantomCiphertext& ct, const PhantomContext& cc,
                                        const std::vector<double>& coeffs) const;
  void ApplyDoubleAngleIterations(PhantomCiphertext& ct, const PhantomContext& cc, uint32_t numIter) const;
  // ModRaise input preparation (AdjustCiphertext, bootstrap.cu:1131-1155) + RaiseMod
  PhantomCiphertext RaiseWithCorrection(const PhantomCiphertext& ct, const PhantomContext& cc) const;

  // ---- the reference's rotation-index / precompute / evaluate surface (include/bootstrap.cuh:116-175)
  // Find*RotationIndices (bootstrap.cu:610-820): the slot rotations whose keys the transforms of
  // a setup read (M = 2N), sorted, without 0 and M/4.  They describe this engine's level structure
  // (baby steps j stride, giant steps g i stride per level, plus the sparse partial sums / fold).
  std::vector<int32_t> FindBootstrapRotationIndices(uint32_t slots, uint32_t M) const;
  std::vector<int32_t> FindCoeffsToSlotsRotationIndices(uint32_t slots, uint32_t M) const;
  std::vector<int32_t> FindSlotsToCoeffsRotationIndices(uint32_t slots, uint32_t M) const;
  // a dense slots x slots linear transform evaluated by baby steps g = dim (0: the smallest power of
  // two with g^2 >= slots) and giant steps g i: rotations 1 .. g-1 and g, 2g, ..
  std::vector<int32_t> FindLinearTransformRotationIndices(uint32_t slots, uint32_t M, uint32_t dim = 0) const;
  // EvalLinearTransformPrecompute (include/bootstrap.cuh:128-131; declared but never defined in the
  // reference): the diagonals of A (times scale), pre-rotated for the baby-step giant-step
  // evaluation, encoded in the extended basis Ql u P at chain 1 + L (L = limbs dropped)
  std::vector<std::shared_ptr<PhantomPlaintext>> EvalLinearTransformPrecompute(
      const PhantomContext& cc, const std::vector<std::vector<std::complex<double>>>& A, double scale = 1,
      uint32_t L = 0) const;
  // the two-matrix (sparse) form: declared by the reference without a definition either; throws
  std::vector<std::shared_ptr<PhantomPlaintext>> EvalLinearTransformPrecompute(
      const PhantomContext& cc, const std::vector<std::vector<std::complex<double>>>& A,
      const std::vector<std::vector<std::complex<double>>>& B, uint32_t orientation = 0, double scale = 1,
      uint32_t L = 0) const;
  // A(ct) for the plaintexts of EvalLinearTransformPrecompute (the reference's EvalLinearTransform,
  // commented out in include/bootstrap.cuh:152): one hoisted modup, g rotations, b giant steps
  PhantomCiphertext EvalLinearTransform(const std::vector<std::shared_ptr<PhantomPlaintext>>& A,
                                        const PhantomCiphertext& ct, const PhantomContext& cc) const;
  // EvalCoeffsToSlotsPrecompute / EvalSlotsToCoeffsPrecompute (bootstrap.cu:183-560): the level
  // plaintexts of the homomorphic encoding / decoding of the setup for rotGroup.size() slots, with
  // `scale` (times i when flag_i) folded in, at the levels L selects (the reference's lEnc / lDec:
  // chain 1 + size_Q - L - levelBudget; 0 = chain 1).  A must be the 2N-th roots of unity
  // (ksiPows, A[j] = exp(2 pi i j / 2N)) and rotGroup the powers 5^j mod 2N: this engine factors the
  // same canonical embedding into its own slot-domain butterfly stages, so the
  // plaintext sets are that factorisation's [level][diagonal], not the reference's collapsed-FFT
  // coefficients.  Requires EvalBootstrapSetup for that slot count.
  std::vector<std::vector<std::shared_ptr<PhantomPlaintext>>> EvalCoeffsToSlotsPrecompute(
      const PhantomContext& cc, const std::vector<std::complex<double>>& A, const std::vector<uint32_t>& rotGroup,
      const std::vector<double>& sf, bool flag_i, double scale = 1, uint32_t L = 0) const;
  std::vector<std::vector<std::shared_ptr<PhantomPlaintext>>> EvalSlotsToCoeffsPrecompute(
      const PhantomContext& cc, const std::vector<std::complex<double>>& A, const std::vector<uint32_t>& rotGroup,
      const std::vector<double>& sf, bool flag_i, double scale = 1, uint32_t L = 0) const;
  // EvalCoeffsToSlots / EvalSlotsToCoeffs with those plaintext sets (bootstrap.cu:1157-1655)
  PhantomCiphertext EvalCoeffsToSlots(const std::vector<std::vector<std::shared_ptr<PhantomPlaintext>>>& A,
                                      const PhantomCiphertext& ctxt, const PhantomContext& cc,
                                      uint32_t numSlots = 0) const;
  PhantomCiphertext EvalSlotsToCoeffs(const std::vector<std::vector<std::shared_ptr<PhantomPlaintext>>>& A,
                                      const PhantomCiphertext& ctxt, const PhantomContext& cc,
                                      uint32_t numSlots = 0) const;
  // GetMultKey / GetGaloisKey (include/bootstrap.cuh:169-175): the relinearization key and the
  // fused rotation keys the bootstrap uses
  const PhantomRelinKey& GetMultKey() const { return mul_key_; }
  const PhantomGaloisKey& GetGaloisKey() const { return galois_keys_; }

  // GetBootstrapDepth (bootstrap.cu:595-604): the reference's level budget, levelBudget[0] +
  // levelBudget[1] + GetMultiplicativeDepthByCoeffVector(88) (8, util.cu:44-58) + R (6) = 18 for
  // {2, 2}.  This engine's own evaluation needs one level less (the Chebyshev recursion folds the
  // affine map, GetBootstrapDepthTight = 17); by default a bootstrap still lands on the
  // reference's output level (the raise starts one level down), so a caller's level bookkeeping
  // after EvalBootstrap is the reference's.  UseTightLevels(true) before EvalBootstrapSetup keeps
  // the extra level instead.
  static uint32_t GetBootstrapDepth(const std::vector<uint32_t>& levelBudget);
  static uint32_t GetBootstrapDepthTight(const std::vector<uint32_t>& levelBudget);
  void UseTightLevels(bool tight) { tight_levels_ = tight; }
  // rotations (slot offsets) whose keys a bootstrap with `numSlots` slots needs
  std::vector<int> rotation_indices(uint32_t numSlots = 0) const;
  // chain index of a bootstrap's output
  size_t output_chain_index(uint32_t numSlots = 0, uint32_t numIterations = 1) const;
  // the same from the parameters alone (no context, no setup): ModRaise lands on chain
  // 1 + raise level, then CoeffToSlot, EvalMod and SlotToCoeff each consume their depth
  static size_t OutputChainIndex(const std::vector<uint32_t>& levelBudget, uint32_t log_slots,
                                 uint32_t numIterations = 1, bool tight = false);
  uint32_t correction_factor() const { return correction_; }
  const std::vector<double>& eval_mod_coefficients() const { return cheb_; }
  const std::vector<double>& scaling_factors() const { return sf_; }
  const std::vector<double>& scaling_factors_big() const { return sf_big_; }
  // whether the linear-transform plaintexts of a slot count are encoded (false between a
  // precompute = false setup and the first bootstrap)
  bool precomputed(uint32_t numSlots = 0) const;

  static constexpr uint32_t K_UNIFORM = 512;  // bound on |I| of the raised plaintext t = m + q0 I
  static constexpr uint32_t R_UNIFORM = 6;    // double-angle iterations
  static constexpr int kChebDegree = 88;      // bootstrap.cuh:232-255 (89 coefficients)

 private:
  // one level of a linear transform: diagonals (u - center) * stride, u < D, evaluated as
  // baby steps j < g (hoisted rotations) and giant steps i < b
  struct LTLevel {
    int stride = 1, center = 0, D = 0, g = 1, b = 1;
    size_t chain = 1;
    std::vector<std::unique_ptr<PhantomPlaintext>> pts;  // [D], pre-rotated by -g i stride; null = zero
    DeviceBuffer<const uint64_t*> d_pts;                // [b][g] device pointer table (zero-padded)
    DeviceBuffer<uint64_t> zero;                        // the zero plaintext absent diagonals point at
  };
  // the precomputation of one slot count (the reference's CKKSBootstrapPrecom)
  // the arguments of one direction's build_levels, kept for a deferred encoding
  struct LevelArgs {
    std::vector<int> sizes;
    double constant = 1.0;
    size_t first_chain = 1;
    uint32_t dim1 = 0;
    bool times_i = false;  // the constant is i * constant (EvalCoeffsToSlotsPrecompute's flag_i)
  };
  struct Precom {
    uint32_t slots = 0;
    std::vector<LTLevel> enc, dec;
    bool encoded = true;  // false: level structure only (precompute = false)
    LevelArgs enc_args, dec_args;
  };
  void setup(const PhantomContext& cc, const std::vector<uint32_t>& levelBudget, const std::vector<double>& sf,
             uint32_t correctionFactor, uint32_t slots, const std::vector<uint32_t>& dim1, bool precompute);
  // encode = false: the levels' structure (g, b, stride, center, chain) without their plaintexts
  void build_levels(const PhantomContext& cc, bool encode_dir, const LevelArgs& args, uint32_t slots,
                    std::vector<LTLevel>& out, bool encode) const;
  const Precom& precom(uint32_t numSlots, const PhantomContext& cc) const;
  PhantomCiphertext apply_level(const PhantomContext& cc, const PhantomCiphertext& ct, const LTLevel& lv) const;
  void level_babies(const PhantomContext& cc, const PhantomCiphertext& in, const LTLevel& lv, LevelWork& w,
                    bool launch = true, bool alloc_babies = true) const;
  phx::LtArgs level_lt_args(const PhantomContext& cc, const LTLevel& lv, LevelWork& w) const;
  PhantomCiphertext level_giants(const PhantomContext& cc, const LTLevel& lv, LevelWork& w) const;
  std::vector<PhantomCiphertext> level_giants_group(const PhantomContext& cc, const LTLevel& lv,
                                                    std::vector<LevelWork>& w) const;
  // apply_level of 2..8 ciphertexts in lockstep: their baby steps and inner products each in one
  // launch that reads the level's keys / plaintexts about once for all; each result equals apply_level's
  std::vector<PhantomCiphertext> apply_level_group(const PhantomContext& cc,
                                                   const std::vector<const PhantomCiphertext*>& in,
                                                   const LTLevel& lv) const;
  // the reference-signature precompute / evaluate pair (above): one direction's levels built from
  // a caller's roots, and the level structure re-attached to a caller's plaintext set
  std::vector<std::vector<std::shared_ptr<PhantomPlaintext>>> precompute_dir(
      const PhantomContext& cc, bool encode_dir, const std::vector<std::complex<double>>& A,
      const std::vector<uint32_t>& rotGroup, bool flag_i, double scale, uint32_t L) const;
  PhantomCiphertext apply_dir(const std::vector<std::vector<std::shared_ptr<PhantomPlaintext>>>& A,
                              const PhantomCiphertext& ct, const PhantomContext& cc, uint32_t numSlots,
                              bool encode_dir) const;
  void attach(const PhantomContext& cc, LTLevel& lv, const std::vector<std::shared_ptr<PhantomPlaintext>>& pts) const;
  // the baby-step giant-step shape of a level from its diagonal map (n ring slots, offsets multiples
  // of `stride`; dim1 = 0: g^2 >= 2 D)
  static void lt_shape(LTLevel& lv, const boot::DiagMap& T, size_t n, uint32_t dim1, int stride);
  // encode a level's diagonals (pre-rotated by -g i stride) in the extended basis at lv.chain
  void encode_level(const PhantomContext& cc, LTLevel& lv, const boot::DiagMap& T) const;
  std::vector<int32_t> dir_rotations(uint32_t slots, uint32_t M, bool encode_dir) const;
  PhantomCiphertext eval_mod(const PhantomCiphertext& ct, const PhantomContext& cc) const;
  // the series / double angle / EvalMod on several ciphertexts in lockstep (one level and scale):
  // their products share batched key switches (the real and imaginary halves of EvalMod)
  std::vector<PhantomCiphertext> eval_mod_lanes(std::vector<PhantomCiphertext> in, const PhantomContext& cc) const;
  std::vector<PhantomCiphertext> chebyshev_lanes(std::vector<PhantomCiphertext> in, const PhantomContext& cc,
                                                 const std::vector<double>& coeffs) const;
  void double_angle_lanes(std::vector<PhantomCiphertext>& v, const PhantomContext& cc, uint32_t numIter) const;
  PhantomCiphertext bootstrap_once(const PhantomCiphertext& ct, const PhantomContext& cc, const Precom& pc) const;
  // bootstrap_once of 2..8 ciphertexts in lockstep (full packing): grouped linear-transform levels,
  // EvalMod on 2 x group lanes; each result equals bootstrap_once's, bit for bit
  std::vector<PhantomCiphertext> bootstrap_group(const std::vector<const PhantomCiphertext*>& in,
                                                 const PhantomContext& cc, const Precom& pc) const;

  PhantomCKKSEncoder& encoder_;
  std::vector<double> sf_, sf_big_;
  std::vector<uint32_t> budget_;
  mutable std::mutex precom_mu_;  // deferred encodings
  uint32_t correction_ = 0;
  bool tight_levels_ = false;
  size_t raise_level_ = 0;  // the level ModRaise lands on (reference layout: the spare level)
  std::map<uint32_t, Precom> precom_;
  std::vector<double> cheb_;
  mutable LeafTableCache leaf_tables_;
  // per linear-transform level: the device table of its baby steps (phx::KsBatchEntry as raw
  // words) and the host copy it was uploaded from (re-uploaded when keys or tables move)
  mutable std::mutex baby_mu_;
  mutable std::map<const void*, std::pair<std::vector<uint64_t>, DeviceBuffer<uint64_t>>> baby_tables_;
  const void* baby_table(const PhantomContext& cc, const LTLevel& lv, size_t QlP) const;
  PhantomRelinKey mul_key_;
  PhantomGaloisKey galois_keys_;  // fused keys
  // fingerprint of the secret the Galois keys were made from: keys of earlier setups (other slot
  // counts) are kept only while the secret stays the same; a new secret replaces them all, as the
  // reference's EvalBootstrapKeyGen replaces its key set (bootstrap.cu:824-836)
  uint64_t galois_owner_ = 0;
  void claim_galois_keys(const PhantomSecretKey& sk);
};

}  // namespace phantom
