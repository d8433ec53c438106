// bootstrapping_example — the reference's bootstrapping/bootstrapping_example.cu
// (SimpleBootstrapExample, lines 69-200) on this engine, plus staged checks of the pieces.
//
// usage: bootstrapping_example [ops|boot|batch] [log_n] [iterations] [lanes]
//   ops  : encode/encrypt/decrypt, const-mult drain, hoisted rotation, conjugation, multiply,
//          ModRaise; precision of each against the plaintext computation
//   boot : full bootstrap of 2^(log_n - 1) uniform reals in [1, 5] (the example's input),
//          levelBudget {2, 2}, scale 2^59, Q = {60, 29 x 59}, P = 10 x 60
//   batch: `iterations` independent bootstraps, `lanes` at a time side by side (C5 on one GPU)
//   tail : `iterations` fresh ciphertexts under each of `keys` fresh keys (4th argument, default 1),
//          each bootstrapped; per ciphertext the precision, the raised plaintext's overflow I
//          (t = m + q0 I, from decrypting RaiseWithCorrection's output mod q0 and q1) and the
//          output error in the coefficient domain, so a low-precision outlier can be traced to
//          the coefficients that carry its error
// Prints one JSON object per check; exit status 0 iff every check meets its bound.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../host/bootstrap.h"
#include "../host/ckks_eval.h"
#include "../host/encoder.h"
#include "../host/evaluate.h"
#include "../host/keys.h"
#include "../host/modulus.h"
#include "../host/traffic.h"
#include "../csrc/ckks.h"
#include "../csrc/rns.h"
#include "../csrc/ntt.h"

using namespace phantom;
using namespace phantom::arith;

static bool g_ok = true;

// bootstrapping_example.cu:17-41
static double compute_bit_precision(const std::vector<double>& ref, const std::vector<double>& actual) {
  double sum = 0.0;
  int cnt = 0;
  for (size_t i = 0; i < ref.size(); ++i) {
    if (std::abs(ref[i]) < 1e-20) continue;
    double rel = std::abs(ref[i] - actual[i]) / std::abs(ref[i]);
    if (rel < 1e-40) rel = 1e-40;
    sum += -std::log2(rel);
    ++cnt;
  }
  return cnt ? sum / cnt : 0.0;
}

// NaN-propagating max |a - b|; also prints the first slots of a and b
static double max_abs_err(const std::vector<std::complex<double>>& a, const std::vector<std::complex<double>>& b) {
  double m = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    const double e = std::abs(a[i] - b[i]);
    if (!(e <= m)) m = e;  // NaN sticks
  }
  std::printf("{\"sample\": [[%.6f, %.6f], [%.6f, %.6f]], \"want\": [[%.6f, %.6f], [%.6f, %.6f]]}\n", a[0].real(),
              a[0].imag(), a[1].real(), a[1].imag(), b[0].real(), b[0].imag(), b[1].real(), b[1].imag());
  return m;
}

static std::vector<std::complex<double>> decrypt_decode(const PhantomContext& ctx, PhantomSecretKey& sk,
                                                        const PhantomCKKSEncoder& enc, const PhantomCiphertext& ct) {
  PhantomPlaintext pt;
  sk.decrypt(ctx, ct, pt);
  std::vector<std::complex<double>> z;
  enc.decode(ctx, pt, z);
  return z;
}

static void report(const char* name, double err, double bound, size_t chain) {
  const bool ok = err <= bound;
  g_ok &= ok;
  std::printf("{\"check\": \"%s\", \"max_abs_err\": %.3e, \"bound\": %.1e, \"chain_index\": %zu, \"ok\": %s}\n", name,
              err, bound, chain, ok ? "true" : "false");
  std::fflush(stdout);
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "boot";
  // concurrent bootstraps use up to 16 streams: give them their own hardware queues (read once,
  // at HIP initialisation, which has not happened yet)
  if (mode == "batch") setenv("GPU_MAX_HW_QUEUES", "16", 0);
  const int log_n = argc > 2 ? std::atoi(argv[2]) : 16;
  const int iters = argc > 3 ? std::atoi(argv[3]) : 3;
  const size_t N = size_t(1) << log_n, slots = N / 2;

  // parameters of SimpleBootstrapExample (bootstrapping_example.cu:76-116)
  const std::vector<uint32_t> levelBudget = {2, 2};
  const int depth = 29, special = 10;
  std::vector<int> bits;
  for (int i = 0; i < depth + 1 + special; ++i) bits.push_back(i == 0 ? 60 : (i < depth + 1 ? 59 : 60));
  EncryptionParameters parms(scheme_type::ckks);
  parms.set_poly_modulus_degree(N);
  parms.set_special_modulus_size(special);
  parms.set_coeff_modulus(CoeffModulus::Create(N, bits));
  const double scale = std::pow(2.0, 59);

  double t0 = now_ms();
  PhantomContext ctx(parms);
  // "tail" draws fresh OS-entropy keys
  // (TAIL_KEY_SEED=s: seeded keys s, s + 1, .. instead, so that two library builds see the same
  // keys and ciphertexts: tools/diag_centred.sh)
  const char* tail_seed = std::getenv("TAIL_KEY_SEED");
  const uint64_t key_seed = mode == "tail" ? (tail_seed ? std::strtoull(tail_seed, nullptr, 0) : 0) : 0x5EED;
  PhantomSecretKey sk = key_seed ? PhantomSecretKey::for_testing(ctx, key_seed) : PhantomSecretKey(ctx);
  PhantomCKKSEncoder enc(ctx);
  const std::vector<double> sf = precompute_scaling_factors(ctx, scale);
  std::printf("{\"stage\": \"context+keys\", \"ms\": %.1f, \"N\": %zu, \"limbs_Q\": %zu, \"limbs_P\": %zu}\n",
              now_ms() - t0, N, ctx.size_Q(), ctx.size_P());

  std::mt19937_64 rng(0xB007);
  std::uniform_real_distribution<double> dis(1.0, 5.0);
  std::vector<double> x(slots);
  for (auto& v : x) v = dis(rng);
  std::vector<std::complex<double>> xz(x.begin(), x.end());

  // encode + encrypt at chain 1 with the FLEXIBLEAUTO scale of level 0
  PhantomPlaintext pt;
  enc.encode(ctx, x, sf[0], pt, 1);
  PhantomCiphertext ct;
  sk.encrypt_symmetric(ctx, pt, ct);
  report("encrypt_decrypt", max_abs_err(decrypt_decode(ctx, sk, enc, ct), xz), 1e-6, ct.chain_index());

  if (mode == "dbg") {
    {  // rescale only
      PhantomCiphertext r = ct;
      EvalModReduceInPlace(ctx, r, 1);
      report("dbg_rescale", max_abs_err(decrypt_decode(ctx, sk, enc, r), xz), 1e-6, r.chain_index());
    }
    {  // mod switch only
      PhantomCiphertext r = mod_switch_to_next(ctx, ct);
      report("dbg_modswitch", max_abs_err(decrypt_decode(ctx, sk, enc, r), xz), 1e-6, r.chain_index());
    }
    {  // const mult by 1 (degree 2, no rescale)
      PhantomCiphertext r = ct;
      EvalMultConstInplace(ctx, r, 1.0, sf);
      report("dbg_constmult", max_abs_err(decrypt_decode(ctx, sk, enc, r), xz), 1e-6, r.chain_index());
      EvalModReduceInPlace(ctx, r, 1);
      report("dbg_constmult_rescale", max_abs_err(decrypt_decode(ctx, sk, enc, r), xz), 1e-6, r.chain_index());
    }
    {  // tensor only (3 components), decrypt with s^2
      PhantomCiphertext r = ct;
      multiply_inplace(ctx, r, r);
      std::vector<std::complex<double>> want(slots);
      for (size_t j = 0; j < slots; ++j) want[j] = x[j] * x[j];
      report("dbg_tensor", max_abs_err(decrypt_decode(ctx, sk, enc, r), want), 1e-6, r.chain_index());
      PhantomRelinKey rlk = sk.gen_relinkey(ctx);
      relinearize_inplace(ctx, r, rlk);
      report("dbg_relin", max_abs_err(decrypt_decode(ctx, sk, enc, r), want), 1e-6, r.chain_index());
    }
    {  // square via EvalMultRescale
      PhantomRelinKey rlk = sk.gen_relinkey(ctx);
      PhantomCiphertext r = EvalMultRescale(ctx, ct, ct, rlk, sf);
      std::vector<std::complex<double>> want(slots);
      for (size_t j = 0; j < slots; ++j) want[j] = x[j] * x[j];
      report("dbg_square_rescale", max_abs_err(decrypt_decode(ctx, sk, enc, r), want), 1e-5, r.chain_index());
    }
    std::vector<std::complex<double>> want(slots);
    for (size_t j = 0; j < slots; ++j) want[j] = xz[(j + 1) % slots];
    {  // key residue check: b_i + a_i * enc must be small outside digit i's primes
      auto check_key = [&](const PhantomKSwitchKey& k, const uint64_t* enc_key, const char* name) {
        const size_t QP = ctx.size_QP();
        DeviceBuffer<uint64_t> t(QP * N, nullptr);
        for (size_t i = 0; i < k.dnum(); ++i) {
          const uint64_t* b = k.digit(i);
          const uint64_t* a = b + QP * N;
          (void)phx::poly_mul_add(a, enc_key, b, t.get(), ctx.mod_QP(), N, QP, nullptr);
          (void)phx::ntt_inverse(ctx.gpu_rns_tables(), t.get(), t.get(), phx::LimbMap::contiguous((int)QP, 0), nullptr,
                                 nullptr, nullptr);
          std::vector<uint64_t> h = t.download(nullptr);
          uint64_t worst = 0;
          size_t worst_l = 0;
          for (size_t l = 0; l < QP; ++l) {
            if (l >= i * ctx.size_P() && l < (i + 1) * ctx.size_P()) continue;
            const uint64_t q = ctx.key_moduli()[l];
            for (size_t c = 0; c < N; c += 97) {
              const uint64_t v = h[l * N + c], m = std::min(v, q - v);
              if (m > worst) { worst = m; worst_l = l; }
            }
          }
          std::printf("{\"key\": \"%s\", \"digit\": %zu, \"worst_offdigit_residue\": %llu, \"limb\": %zu}\n", name, i,
                      (unsigned long long)worst, worst_l);
        }
      };
      PhantomRelinKey rk = sk.gen_relinkey(ctx);
      check_key(rk, sk.secret_key_array(), "relin");
      PhantomGaloisKey g = sk.create_galois_keys(ctx, {5});
      check_key(g.get(5), sk.secret_key_array(), "galois5");
      PhantomRelinKey rk2 = sk.gen_relinkey(ctx);
      check_key(rk2, sk.secret_key_array(), "relin_again");
    }
    {  // standard Galois key rotation by 1
      PhantomGaloisKey g = sk.create_galois_keys(ctx, {FindAutomorphismIndex2nComplex(1, N)});
      PhantomCiphertext r = ct;
      rotate_inplace(ctx, r, 1, g);
      report("dbg_rotate_std", max_abs_err(decrypt_decode(ctx, sk, enc, r), want), 1e-6, r.chain_index());
    }
    {  // fused key rotation by 1, step by step
      PhantomGaloisKey g = sk.create_galois_keys_fused(ctx, {FindAutomorphismIndex2nComplex(1, N)});
      DeviceBuffer<uint64_t> d = EvalFastRotationPrecompute(ctx, ct);
      PhantomCiphertext e0 = KeySwitchExt(ctx, ct);
      PhantomCiphertext back = KeySwitchDown(ctx, e0);
      report("dbg_ksext_down", max_abs_err(decrypt_decode(ctx, sk, enc, back), xz), 1e-6, back.chain_index());
      PhantomCiphertext e = EvalFastRotationExt(ctx, ct, g, 1, d.get(), true);
      PhantomCiphertext r = KeySwitchDown(ctx, e);
      report("dbg_rotate_fused", max_abs_err(decrypt_decode(ctx, sk, enc, r), want), 1e-6, r.chain_index());
    }
    for (size_t lv = 0; lv + 2 < ctx.size_Q(); ++lv) {  // drain, every level
      PhantomCiphertext& d = ct;
      EvalMultConstInplace(ctx, d, 1.0, sf);
      EvalModReduceInPlace(ctx, d, 1);
      std::printf("{\"drain_level\": %zu, \"scale\": %.6e, \"sf\": %.6e}\n", level_of(d), d.scale(), sf[level_of(d)]);
      report("dbg_drain", max_abs_err(decrypt_decode(ctx, sk, enc, d), xz), 1e-4, d.chain_index());
    }
    return g_ok ? 0 : 1;
  }

  if (mode == "flex") {
    // the reference's FLEXIBLEAUTO surface (include/evaluate.cuh:270-452) with the ciphertext's
    // PreComputeScale factors, as bootstrapping_example.cu:146-148 obtains them
    PhantomRelinKey rlk = sk.gen_relinkey(ctx);
    ct.PreComputeScale(ctx, scale);
    const std::vector<double> sfR = ct.getScalingFactorsReal(), sfB = ct.getScalingFactorsRealBig();
    auto want_of = [&](auto f) {
      std::vector<std::complex<double>> w(slots);
      for (size_t j = 0; j < slots; ++j) w[j] = f(x[j]);
      return w;
    };
    const auto sq = want_of([](double v) { return v * v; });
    PhantomCiphertext m = EvalMultAuto(ctx, ct, ct, rlk, sfR, sfB);
    report("flex_mult_auto", max_abs_err(decrypt_decode(ctx, sk, enc, m), sq), 1e-5, m.chain_index());
    PhantomCiphertext s2 = EvalSquare(ctx, ct, rlk, sfR, sfB);
    report("flex_square", max_abs_err(decrypt_decode(ctx, sk, enc, s2), sq), 1e-5, s2.chain_index());
    const bool degs = m.GetNoiseScaleDeg() == 2 && s2.GetNoiseScaleDeg() == 2;
    report("flex_degrees", degs ? 0.0 : 1.0, 0.5, m.chain_index());
    // same level, degrees 2 and 1; then across levels (rescaled product + fresh input)
    PhantomCiphertext a1 = EvalAddAuto(ctx, m, ct, sfR, sfB);
    const auto sq_plus = want_of([](double v) { return v * v + v; });
    report("flex_add_auto_degree", max_abs_err(decrypt_decode(ctx, sk, enc, a1), sq_plus), 1e-5, a1.chain_index());
    PhantomCiphertext r1 = ModReduce(ctx, m, 1);
    PhantomCiphertext a2 = EvalAddAuto(ctx, ct, r1, sfR, sfB);
    report("flex_add_auto_levels", max_abs_err(decrypt_decode(ctx, sk, enc, a2), sq_plus), 1e-5, a2.chain_index());
    PhantomCiphertext d2 = EvalSubAuto(ctx, r1, ct, sfR, sfB);
    report("flex_sub_auto_levels", max_abs_err(decrypt_decode(ctx, sk, enc, d2), want_of([](double v) { return v * v - v; })),
           1e-5, d2.chain_index());
    PhantomCiphertext c1 = EvalAddConst(ctx, ct, -2.5, sfR, sfB);
    report("flex_add_const", max_abs_err(decrypt_decode(ctx, sk, enc, c1), want_of([](double v) { return v - 2.5; })), 1e-6,
           c1.chain_index());
    PhantomCiphertext c2 = EvalAddConst(ctx, m, 3.0, sfR, sfB);
    report("flex_add_const_degree2", max_abs_err(decrypt_decode(ctx, sk, enc, c2), want_of([](double v) { return v * v + 3.0; })),
           1e-5, c2.chain_index());
    PhantomCiphertext mc = EvalMultConst(ctx, m, 0.25, sfR);  // lazily rescales m first
    report("flex_mult_const_lazy", max_abs_err(decrypt_decode(ctx, sk, enc, mc), want_of([](double v) { return 0.25 * v * v; })),
           1e-5, mc.chain_index());
    {
      PhantomPlaintext pp;
      std::vector<double> half(slots, 0.5);
      enc.encode(ctx, half, scale, pp, 1);
      PhantomCiphertext mp = ct;
      EvalMultAutoInplace(ctx, mp, pp, sfR, sfB);
      report("flex_mult_plain_auto", max_abs_err(decrypt_decode(ctx, sk, enc, mp), want_of([](double v) { return 0.5 * v; })),
             1e-5, mp.chain_index());
    }
    // Chebyshev series on [1, 5]: degree 4 (the linear method) and 30 (Paterson-Stockmeyer),
    // against the host value of the same interpolant; levels consumed reported
    for (uint32_t deg : {4u, 30u}) {
      auto f = [](double t) { return std::sin(t) / t; };
      const std::vector<double> co = EvalChebyshevCoefficients(f, 1.0, 5.0, deg);
      PhantomCiphertext cs = EvalChebyshevFunction(f, ctx, rlk, ct, 1.0, 5.0, deg, sfR, sfB);
      const auto host = want_of([&](double v) {
        const double y = (2.0 * v - 6.0) / 4.0;
        double t0 = 1.0, t1 = y, acc = co[0] / 2 + co[1] * y;
        for (size_t k = 2; k < co.size(); ++k) {
          const double t2 = 2.0 * y * t1 - t0;
          acc += co[k] * t2;
          t0 = t1;
          t1 = t2;
        }
        return acc;
      });
      const size_t used = cs.chain_index() - ct.chain_index() + (cs.GetNoiseScaleDeg() > 1 ? 1 : 0);
      std::printf("{\"chebyshev_degree\": %u, \"levels_used\": %zu}\n", deg, used);
      report(deg == 4 ? "flex_chebyshev_linear" : "flex_chebyshev_ps", max_abs_err(decrypt_decode(ctx, sk, enc, cs), host),
             1e-4, cs.chain_index());
    }
    std::printf("{\"done\": \"flex\", \"ok\": %s}\n", g_ok ? "true" : "false");
    return g_ok ? 0 : 1;
  }

  if (mode == "refapi") {
    // the reference-signature FHECKKSRNS surface (include/bootstrap.cuh:116-175) at a small ring:
    // rotation-index finders, CoeffsToSlots / SlotsToCoeffs through the precompute + evaluate pair,
    // the dense linear transform, GetMultKey / GetGaloisKey, and the evaluator's
    // KeySwitchDownFirstElement / EvalMultExt / EvalAddExt value forms
    ct.PreComputeScale(ctx, scale);
    const std::vector<double> sfR = ct.getScalingFactorsReal(), sfB = ct.getScalingFactorsRealBig();
    FHECKKSRNS boot(enc);
    std::vector<uint32_t> budget = levelBudget;
    boot.EvalBootstrapSetup(ctx, budget, scale, sfR, sfB);
    boot.EvalMultKeyGen(sk, ctx);
    boot.EvalBootstrapKeyGen(sk, ctx, static_cast<uint32_t>(slots));
    const uint32_t M = static_cast<uint32_t>(2 * N);
    std::vector<int32_t> all = boot.FindBootstrapRotationIndices(static_cast<uint32_t>(slots), M);
    std::vector<int> own = boot.rotation_indices();
    std::sort(own.begin(), own.end());
    const bool idx_ok = std::vector<int>(all.begin(), all.end()) == own &&
                        std::is_sorted(all.begin(), all.end()) && !all.empty();
    report("refapi_rotation_indices", idx_ok ? 0.0 : 1.0, 0.5, 0);
    report("refapi_get_keys", (&boot.GetMultKey() != nullptr && boot.GetGaloisKey().has(
                                  FindAutomorphismIndex2nComplex(all.front(), N))) ? 0.0 : 1.0, 0.5, 0);
    // ksiPows and rotGroup as EvalBootstrapSetup computes them (bootstrap.cu:92-107)
    std::vector<std::complex<double>> ksi(M + 1);
    for (uint32_t j = 0; j < M; ++j) ksi[j] = std::polar(1.0, 2.0 * M_PI * j / M);
    ksi[M] = ksi[0];
    std::vector<uint32_t> rot(slots);
    for (size_t j = 0, g5 = 1; j < slots; ++j, g5 = g5 * 5 % M) rot[j] = static_cast<uint32_t>(g5);
    // lEnc = L0 - levelBudget - 1: the encoding starts at chain 2; the decoding right after it
    const uint32_t L0 = static_cast<uint32_t>(ctx.size_Q());
    auto ctsPre = boot.EvalCoeffsToSlotsPrecompute(ctx, ksi, rot, sfR, false, 1.0, L0 - budget[0] - 1);
    auto stcPre = boot.EvalSlotsToCoeffsPrecompute(ctx, ksi, rot, sfR, false, 1.0, L0 - budget[0] - 1 - budget[1]);
    PhantomCiphertext in2 = ct;
    EvalMultConstInplace(ctx, in2, 1.0, sfR);  // at chain 2
    EvalModReduceInPlace(ctx, in2, 1);
    PhantomCiphertext slotsCt = boot.EvalCoeffsToSlots(ctsPre, in2, ctx);
    PhantomCiphertext back = boot.EvalSlotsToCoeffs(stcPre, slotsCt, ctx);
    report("refapi_cts_stc_roundtrip", max_abs_err(decrypt_decode(ctx, sk, enc, back), xz), 1e-6, back.chain_index());
    // the coefficient-domain view: CtS puts the message polynomial's coefficients (scaled by 1 /
    // its encoding scale) into the slots, bit-reversed; their norm equals the message's
    {
      const auto cv = decrypt_decode(ctx, sk, enc, slotsCt);
      double e_slots = 0, e_msg = 0;
      for (size_t j = 0; j < slots; ++j) {
        e_slots += std::norm(cv[j]);
        e_msg += x[j] * x[j];
      }
      // Parseval for the canonical embedding: sum |z_j|^2 = (N / 2) sum |c_k|^2 over the N coefficients,
      // and the slots hold c_lo + i c_hi: sum |slot|^2 = sum |c_k|^2
      report("refapi_cts_parseval", std::fabs(e_slots * static_cast<double>(slots) - e_msg) / e_msg, 1e-6,
             slotsCt.chain_index());
    }
    // KeySwitchDownFirstElement / EvalMultExt / EvalAddExt on a P-scaled extended ciphertext
    {
      PhantomCiphertext ext = KeySwitchExt(ctx, ct);
      PhantomCiphertext two = EvalAddExt(ctx, ext, ext);
      PhantomCiphertext down = KeySwitchDown(ctx, static_cast<const PhantomCiphertext&>(two));
      std::vector<std::complex<double>> want2(slots);
      for (size_t j = 0; j < slots; ++j) want2[j] = 2.0 * x[j];
      report("refapi_add_ext_keyswitch_down", max_abs_err(decrypt_decode(ctx, sk, enc, down), want2), 1e-6,
             down.chain_index());
      PhantomCiphertext first = KeySwitchDownFirstElement(ctx, two);
      PhantomCiphertext full = KeySwitchDown(ctx, static_cast<const PhantomCiphertext&>(two));
      const auto a = first.to_host(ctx.stream()), b = full.to_host(ctx.stream());
      const bool same = a.size() * 2 == b.size() && std::equal(a.begin(), a.end(), b.begin());
      report("refapi_keyswitch_down_first_element", same && first.size() == 1 ? 0.0 : 1.0, 0.5, first.chain_index());
      PhantomPlaintext half;
      std::vector<double> hv(slots, 0.5);
      enc.encode_ext(ctx, std::vector<std::complex<double>>(hv.begin(), hv.end()), scale, half, ct.chain_index());
      PhantomCiphertext prod = EvalMultExt(ctx, ext, half);
      PhantomCiphertext pd = KeySwitchDown(ctx, static_cast<const PhantomCiphertext&>(prod));
      EvalModReduceInPlace(ctx, pd, 1);
      std::vector<std::complex<double>> wanth(slots);
      for (size_t j = 0; j < slots; ++j) wanth[j] = 0.5 * x[j];
      report("refapi_mult_ext", max_abs_err(decrypt_decode(ctx, sk, enc, pd), wanth), 1e-6, pd.chain_index());
    }
    // a dense slots x slots transform: A[p][q] = cos(p + 2q) / slots + i sin(3p - q) / slots
    if (slots <= 2048) {  // one level of g <= 32 baby and b <= 64 giant steps (csrc/ckks.h kLtMaxG, kLtMaxB)
      std::vector<std::vector<std::complex<double>>> A(slots, std::vector<std::complex<double>>(slots));
      for (size_t p = 0; p < slots; ++p)
        for (size_t q = 0; q < slots; ++q)
          A[p][q] = std::complex<double>(std::cos(double(p + 2 * q)), std::sin(3.0 * p - double(q))) / double(slots);
      boot.EvalRotationKeyGen(sk, ctx, boot.FindLinearTransformRotationIndices(static_cast<uint32_t>(slots), M));
      auto ltPre = boot.EvalLinearTransformPrecompute(ctx, A, 1.0, 0);
      PhantomCiphertext lt = boot.EvalLinearTransform(ltPre, ct, ctx);
      std::vector<std::complex<double>> want(slots);
      for (size_t p = 0; p < slots; ++p)
        for (size_t q = 0; q < slots; ++q) want[p] += A[p][q] * x[q];
      report("refapi_linear_transform", max_abs_err(decrypt_decode(ctx, sk, enc, lt), want), 1e-6, lt.chain_index());
    }
    // MulAddRescaleBatch (the EvalMod products' shared launches) equals MulAddRescale per job, bit
    // for bit: factors 1 / 2 / 3, zero / one / two terms, with and without a constant, 11 jobs
    // (more than one launch of the batched tensor kernel)
    {
      PhantomCiphertext c2 = ct;
      EvalMultConstInplace(ctx, c2, 0.5, sfR);
      EvalModReduceInPlace(ctx, c2, 1);
      PhantomCiphertext c1 = c2;
      EvalMultConstInplace(ctx, c1, 1.5, sfR);
      EvalModReduceInPlace(ctx, c1, 1);  // one level below c2
      PhantomCiphertext c3 = c2;
      EvalMultConstInplace(ctx, c3, 1.0, sfR);
      EvalModReduceInPlace(ctx, c3, 1);
      const PhantomRelinKey& rk = boot.GetMultKey();
      std::vector<MulAddJob> jobs;
      for (int k = 0; k < 11; ++k) {
        MulAddJob j{&c1, k % 2 ? &c3 : &c1, 1 + k % 3, {}, 0.0};
        if (k % 4 >= 1) j.terms.push_back({&c2, k % 2 ? -1.0 : 0.75});
        if (k % 4 == 3) j.terms.push_back({&c1, 2.0});
        if (k % 5 >= 2) j.constant = k % 2 ? -1.0 : 0.25;
        jobs.push_back(std::move(j));
      }
      const std::vector<PhantomCiphertext> got = MulAddRescaleBatch(ctx, jobs, rk);
      bool same = got.size() == jobs.size();
      for (size_t k = 0; same && k < jobs.size(); ++k) {
        const PhantomCiphertext want = MulAddRescale(ctx, *jobs[k].a, *jobs[k].b, rk, jobs[k].factor, jobs[k].terms,
                                                     jobs[k].constant);
        same = want.to_host(ctx.stream()) == got[k].to_host(ctx.stream()) && want.scale() == got[k].scale() &&
               want.chain_index() == got[k].chain_index();
      }
      report("refapi_muladd_batch_bitexact", same ? 0.0 : 1.0, 0.5, got.empty() ? 0 : got[0].chain_index());
    }
    // a second secret: EvalMultKeyGen / EvalBootstrapKeyGen replace the first secret's keys
    // (bootstrap.cu:824-841), so a ciphertext under the new secret bootstraps correctly
    {
      const size_t nkeys = boot.GetGaloisKey().size();
      PhantomSecretKey sk2(ctx);
      boot.EvalMultKeyGen(sk2, ctx);
      boot.EvalBootstrapKeyGen(sk2, ctx, static_cast<uint32_t>(slots));
      PhantomPlaintext p2;
      enc.encode(ctx, x, ct.scale(), p2, ct.chain_index());
      PhantomCiphertext c2;
      sk2.encrypt_symmetric(ctx, p2, c2);
      PhantomCiphertext r2 = boot.EvalBootstrap(c2, ctx);
      const double err = max_abs_err(decrypt_decode(ctx, sk2, enc, r2), xz);
      report("refapi_rekey_bootstrap", boot.GetGaloisKey().size() <= nkeys ? err : 1.0, 0.05, r2.chain_index());
    }
    std::printf("{\"done\": \"refapi\", \"ok\": %s}\n", g_ok ? "true" : "false");
    return g_ok ? 0 : 1;
  }
  if (mode == "ltpair") {
    // the linear-transform inner products of two ciphertexts: two lt_bsgs launches against one
    // lt_bsgs_group launch (the plaintexts shared through L2), at the CoeffToSlot level shape
    // (Ql = 30, P = 10, g = 32, b = 8); outputs compared bit for bit
    const size_t QlP = ctx.size_Q() + ctx.size_P(), words = 2 * QlP * N;
    const int g = 32, b = 8;
    hipStream_t s = ctx.stream();
    phx::ChaChaKey key{};
    for (int i = 0; i < 8; ++i) key.k[i] = 0x1234567u * (i + 1);
    uint64_t nonce = 1;
    std::vector<DeviceBuffer<uint64_t>> babies, pts;
    for (int c = 0; c < 2 * g; ++c) {
      babies.emplace_back(words, s);
      PHX_CHECK(phx::sample_uniform(babies.back().get(), ctx.mod_QP().q, ctx.mod_QP().barrett, N, QlP, key, nonce++, s));
      PHX_CHECK(phx::sample_uniform(babies.back().get() + QlP * N, ctx.mod_QP().q, ctx.mod_QP().barrett, N, QlP, key,
                                    nonce++, s));
    }
    std::vector<const uint64_t*> ptr_host;
    for (int k = 0; k < g * b; ++k) {
      pts.emplace_back(QlP * N, s);
      PHX_CHECK(phx::sample_uniform(pts.back().get(), ctx.mod_QP().q, ctx.mod_QP().barrett, N, QlP, key, nonce++, s));
      ptr_host.push_back(pts.back().get());
    }
    DeviceBuffer<const uint64_t*> ptr_dev(ptr_host.size(), s);
    PHX_CHECK(hipMemcpy(ptr_dev.get(), ptr_host.data(), ptr_host.size() * sizeof(void*), hipMemcpyHostToDevice));
    phx::LtArgs la[2];
    for (int c = 0; c < 2; ++c) {
      la[c].g = g;
      la[c].b = b;
      la[c].Ql = static_cast<int>(ctx.size_Q());
      la[c].P = static_cast<int>(ctx.size_P());
      la[c].size_Q = static_cast<int>(ctx.size_Q());
      la[c].pts = ptr_dev.get();
      la[c].q = ctx.mod_QP().q;
      la[c].barrett = ctx.mod_QP().barrett;
      la[c].q60 = below_2_60(ctx.key_moduli());
    }
    // the group form takes contiguous babies / inner sums: one buffer per ciphertext
    DeviceBuffer<uint64_t> bcat0(static_cast<size_t>(g) * words, s), bcat1(static_cast<size_t>(g) * words, s);
    for (int j = 0; j < g; ++j) {
      PHX_CHECK(hipMemcpyAsync(bcat0.get() + j * words, babies[j].get(), words * 8, hipMemcpyDeviceToDevice, s));
      PHX_CHECK(hipMemcpyAsync(bcat1.get() + j * words, babies[g + j].get(), words * 8, hipMemcpyDeviceToDevice, s));
    }
    for (int j = 0; j < g; ++j) {
      la[0].baby[j] = bcat0.get() + j * words;
      la[1].baby[j] = bcat1.get() + j * words;
    }
    DeviceBuffer<uint64_t> ocat1(static_cast<size_t>(2 * b) * words, s), ocat2(static_cast<size_t>(2 * b) * words, s);
    phx::LtGroupArgs pa;
    pa.pts = ptr_dev.get();
    pa.q = ctx.mod_QP().q;
    pa.barrett = ctx.mod_QP().barrett;
    pa.g = g;
    pa.b = b;
    pa.Ql = la[0].Ql;
    pa.P = la[0].P;
    pa.size_Q = la[0].size_Q;
    pa.q60 = la[0].q60;
    pa.count = 2;
    pa.baby_stride = words;
    pa.giant_stride = words;
    for (int c = 0; c < 2; ++c) {
      pa.baby0[c] = c ? bcat1.get() : bcat0.get();
      pa.acc[c] = ocat2.get() + static_cast<size_t>(c) * b * words;
      pa.giant1[c] = pa.acc[c] + words;
    }
    auto run = [&](bool pair) {
      if (pair) {
        PHX_CHECK(phx::lt_bsgs_group(pa, N, s));
      } else {
        for (int c = 0; c < 2; ++c) {
          for (int i = 0; i < b; ++i) la[c].out[i] = ocat1.get() + (static_cast<size_t>(c) * b + i) * words;
          PHX_CHECK(phx::lt_bsgs(la[c], N, s));
        }
      }
    };
    hipEvent_t e0, e1;
    PHX_CHECK(hipEventCreate(&e0));
    PHX_CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; ++rep)
      for (bool pair : {false, true}) {
        run(pair);  // warm
        PHX_CHECK(hipEventRecord(e0, s));
        for (int it = 0; it < 5; ++it) run(pair);
        PHX_CHECK(hipEventRecord(e1, s));
        PHX_CHECK(hipEventSynchronize(e1));
        float ms = 0;
        PHX_CHECK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"ltpair\": \"%s\", \"ms_per_pair\": %.3f}\n", pair ? "pair" : "two", ms / 5);
      }
    const bool same = ocat1.download(s) == ocat2.download(s);
    report("ltpair_bitexact", same ? 0.0 : 1.0, 0.5, 0);
    return g_ok ? 0 : 1;
  }
  if (mode == "chebdepth") {
    // EvalChebyshevSeries through the reference's Paterson-Stockmeyer (host/chebyshev_ps.cpp) for
    // every degree 5..119 on three intervals: levels consumed (a pending rescale counts) against
    // the reference's GetDepthByDegree (src/util.cu:44-71), and the decrypted value against the
    // host evaluation of the same interpolant
    PhantomRelinKey rlk = sk.gen_relinkey(ctx);
    ct.PreComputeScale(ctx, scale);
    const std::vector<double> sfR = ct.getScalingFactorsReal(), sfB = ct.getScalingFactorsRealBig();
    const int dmin = argc > 4 ? std::atoi(argv[4]) : 5, dmax = argc > 5 ? std::atoi(argv[5]) : 119;
    struct Iv {
      double a, b, shift;  // inputs x + shift (x in [1, 5]) lie inside [a, b]
    };
    for (const Iv iv : {Iv{-1.0, 1.0, -3.0}, Iv{0.0, 5.0, 0.0}, Iv{-8.0, 3.0, -4.0}}) {
      std::vector<double> xs(slots);
      for (size_t j = 0; j < slots; ++j) xs[j] = iv.shift == -3.0 ? (x[j] - 3.0) / 2.0 : x[j] + iv.shift;
      PhantomPlaintext px;
      enc.encode(ctx, xs, sf[0], px, 1);
      PhantomCiphertext cx;
      sk.encrypt_symmetric(ctx, px, cx);
      auto f = [](double t) { return 1.0 / (1.0 + t * t); };
      for (int deg = dmin; deg <= dmax; ++deg) {
        const std::vector<double> co = EvalChebyshevCoefficients(f, iv.a, iv.b, static_cast<uint32_t>(deg));
        PhantomCiphertext cs = EvalChebyshevSeries(ctx, rlk, cx, co, iv.a, iv.b, sfR, sfB);
        std::vector<std::complex<double>> host(slots);
        for (size_t j = 0; j < slots; ++j) {
          const double y = (2.0 * xs[j] - iv.a - iv.b) / (iv.b - iv.a);
          double t0 = 1.0, t1 = y, acc = co[0] / 2 + co[1] * y;
          for (size_t k = 2; k < co.size(); ++k) {
            const double t2 = 2.0 * y * t1 - t0;
            acc += co[k] * t2;
            t0 = t1;
            t1 = t2;
          }
          host[j] = acc;
        }
        const size_t used = cs.chain_index() - cx.chain_index() + (cs.GetNoiseScaleDeg() > 1 ? 1 : 0);
        const double err = max_abs_err(decrypt_decode(ctx, sk, enc, cs), host);
        std::printf("{\"cheb\": %d, \"a\": %g, \"b\": %g, \"levels_used\": %zu, \"depth_by_degree\": %u, "
                    "\"degree_out\": %zu, \"max_abs_err\": %.3e}\n",
                    deg, iv.a, iv.b, used, ps::GetDepthByDegree(static_cast<size_t>(deg)), cs.GetNoiseScaleDeg(), err);
      }
    }
    std::printf("{\"done\": \"chebdepth\", \"ok\": true}\n");
    return 0;
  }
  if (mode == "ops") {
    PhantomGaloisKey gk = sk.create_galois_keys_fused(
        ctx, {FindAutomorphismIndex2nComplex(1, N), FindAutomorphismIndex2nComplex(-3, N), static_cast<uint32_t>(2 * N - 1)});
    PhantomRelinKey rlk = sk.gen_relinkey(ctx);
    // rotation by 1 and -3 through the hoisted path
    for (int r : {1, -3}) {
      PhantomCiphertext rc = EvalRotateFused(ctx, ct, gk, r);
      std::vector<std::complex<double>> want(slots);
      for (size_t j = 0; j < slots; ++j) want[j] = xz[(j + slots + r) % slots];
      report(r == 1 ? "rotate_1" : "rotate_-3", max_abs_err(decrypt_decode(ctx, sk, enc, rc), want), 1e-6, rc.chain_index());
    }
    // conjugation of (x + i x)
    {
      std::vector<std::complex<double>> zc(slots);
      for (size_t j = 0; j < slots; ++j) zc[j] = {x[j], 0.5 * x[j]};
      PhantomPlaintext pc;
      enc.encode(ctx, zc, sf[0], pc, 1);
      PhantomCiphertext cc;
      sk.encrypt_symmetric(ctx, pc, cc);
      PhantomCiphertext cj = EvalConjFused(ctx, cc, gk);
      std::vector<std::complex<double>> want(slots);
      for (size_t j = 0; j < slots; ++j) want[j] = std::conj(zc[j]);
      report("conjugate", max_abs_err(decrypt_decode(ctx, sk, enc, cj), want), 1e-6, cj.chain_index());
    }
    // multiply + relinearize + rescale (FLEXIBLEAUTO)
    {
      PhantomCiphertext sq = EvalMultRescale(ctx, ct, ct, rlk, sf);
      std::vector<std::complex<double>> want(slots);
      for (size_t j = 0; j < slots; ++j) want[j] = x[j] * x[j];
      report("square_rescale", max_abs_err(decrypt_decode(ctx, sk, enc, sq), want), 1e-5, sq.chain_index());
      // add across levels (AdjustToLevel path)
      PhantomCiphertext s2 = sq;
      EvalAddAutoInplace(ctx, s2, ct, sf);
      for (size_t j = 0; j < slots; ++j) want[j] += x[j];
      report("add_auto_levels", max_abs_err(decrypt_decode(ctx, sk, enc, s2), want), 1e-5, s2.chain_index());
    }
    // monomial X^(N/2) multiplies the slots by i
    {
      PhantomCiphertext m = ct;
      MultByMonomialInPlace(ctx, m, static_cast<uint32_t>(N / 2));
      std::vector<std::complex<double>> want(slots);
      for (size_t j = 0; j < slots; ++j) want[j] = std::complex<double>(0, x[j]);
      report("monomial_i", max_abs_err(decrypt_decode(ctx, sk, enc, m), want), 1e-6, m.chain_index());
    }
    // const-mult drain to 2 limbs, then raise: the raised ciphertext decrypts to m + q0 I whose
    // slots are not small, but its q0 residue must still decrypt to the message
    {
      PhantomCiphertext d = ct;
      for (size_t i = 0; i + 2 < ctx.size_Q(); ++i) {
        EvalMultConstInplace(ctx, d, 1.0, sf);
        EvalModReduceInPlace(ctx, d, 1);
      }
      report("drain_const_mult", max_abs_err(decrypt_decode(ctx, sk, enc, d), xz), 1e-4, d.chain_index());
    }
    // save / load in the reference's byte formats: a ciphertext and the keys round-trip bit
    // for bit, and a rotation with the reloaded key and secret key still decrypts
    {
      std::stringstream cs, ks, gs, ss;
      ct.save(cs);
      PhantomCiphertext c2;
      c2.load(ctx, cs);
      const bool same_ct = c2.to_host(ctx.stream()) == ct.to_host(ctx.stream()) && c2.scale() == ct.scale() &&
                           c2.chain_index() == ct.chain_index();
      rlk.save(ctx, ks);
      PhantomRelinKey rlk2;
      rlk2.load(ctx, ks);
      bool same_key = rlk2.dnum() == rlk.dnum();
      for (size_t i = 0; same_key && i < rlk.dnum(); ++i) {
        std::vector<uint64_t> ha(2 * ctx.size_QP() * N), hb(ha.size());
        PHX_CHECK(hipMemcpy(ha.data(), rlk.digit(i), ha.size() * 8, hipMemcpyDeviceToHost));
        PHX_CHECK(hipMemcpy(hb.data(), rlk2.digit(i), hb.size() * 8, hipMemcpyDeviceToHost));
        same_key = ha == hb;
      }
      gk.save_with_elements(ctx, gs);  // fused keys: no reference format exists
      PhantomGaloisKey gk2;
      gk2.load_with_elements(ctx, gs);
      sk.save(ctx, ss);
      PhantomSecretKey sk2 = PhantomSecretKey::load(ctx, ss);
      PhantomCiphertext rc = EvalRotateFused(ctx, c2, gk2, 1);
      std::vector<std::complex<double>> want(slots);
      for (size_t j = 0; j < slots; ++j) want[j] = xz[(j + 1) % slots];
      const double err = max_abs_err(decrypt_decode(ctx, sk2, enc, rc), want);
      report("save_load", (same_ct && same_key && sk2.coefficients() == sk.coefficients()) ? err : 1.0, 1e-6,
             rc.chain_index());
    }
    std::printf("{\"done\": \"ops\", \"ok\": %s}\n", g_ok ? "true" : "false");
    return g_ok ? 0 : 1;
  }

  // drain levels as the example does (25 x EvalMultConstInplace(ct, 1), lines 150-153)
  for (int i = 0; i < 25; ++i) {
    EvalMultConstInplace(ctx, ct, 1.0, sf);
    EvalModReduceInPlace(ctx, ct, 1);
  }
  report("drained_input", max_abs_err(decrypt_decode(ctx, sk, enc, ct), xz), 1e-4, ct.chain_index());

  FHECKKSRNS boot(enc);
  t0 = now_ms();
  if (mode == "deferred") {
    // the reference's argument list (bootstrap.cu:15-18) with precompute = false: the level
    // structure now, the linear-transform plaintexts at the first EvalBootstrap.  A
    // scalingFactorsRealBig that is not the squares of scalingFactorsReal is refused.
    std::vector<double> sf_big(sf.size() - 1);
    for (size_t k = 0; k < sf_big.size(); ++k) sf_big[k] = sf[k] * sf[k];
    bool threw = false;
    try {
      std::vector<double> bad = sf_big;
      bad[3] *= 1.5;
      FHECKKSRNS b2(enc);
      b2.EvalBootstrapSetup(ctx, levelBudget, scale, sf, bad);
    } catch (const std::invalid_argument&) {
      threw = true;
    }
    report("sf_big_mismatch_refused", threw ? 0.0 : 1.0, 0.5, 0);
    boot.EvalBootstrapSetup(ctx, levelBudget, scale, sf, sf_big, {0, 0}, 0, 0, false);
    report("deferred_not_encoded", boot.precomputed() ? 1.0 : 0.0, 0.5, 0);
    report("sf_big_kept", boot.scaling_factors_big() == sf_big ? 0.0 : 1.0, 0.5, 0);
  } else {
    boot.EvalBootstrapSetup(ctx, levelBudget, scale, sf);
  }
  PHX_CHECK(hipDeviceSynchronize());
  const double setup_ms = now_ms() - t0;
  t0 = now_ms();
  boot.EvalMultKeyGen(sk, ctx);
  boot.EvalBootstrapKeyGen(sk, ctx);
  PHX_CHECK(hipDeviceSynchronize());
  const double keygen_ms = now_ms() - t0;
  std::printf("{\"stage\": \"setup\", \"setup_ms\": %.1f, \"keygen_ms\": %.1f, \"rotation_keys\": %zu, "
              "\"bootstrap_depth\": %u, \"correction\": %u}\n",
              setup_ms, keygen_ms, boot.rotation_indices().size() + 1, FHECKKSRNS::GetBootstrapDepth(levelBudget),
              boot.correction_factor());
  std::fflush(stdout);

  if (mode == "tail") {
    // decrypt `c` and return its first two limbs in coefficient form (q0, q1 residues)
    DeviceBuffer<uint64_t> tmp(2 * N, nullptr);
    auto coeffs2 = [&](const PhantomPlaintext& p) {
      PHX_CHECK(hipMemcpy(tmp.get(), p.data(), 2 * N * sizeof(uint64_t), hipMemcpyDeviceToDevice));
      PHX_CHECK(phx::ntt_inverse(ctx.gpu_rns_tables(), tmp.get(), tmp.get(), phx::LimbMap::contiguous(2, 0), nullptr,
                                 nullptr, nullptr));
      return tmp.download(nullptr);
    };
    const uint64_t q0 = ctx.key_moduli()[0], q1 = ctx.key_moduli()[1];
    auto centered = [](uint64_t v, uint64_t q) { return v > q / 2 ? (__int128)v - (__int128)q : (__int128)v; };
    const int K = FHECKKSRNS::K_UNIFORM;
    __int128 q0inv = 1;  // q0^-1 mod q1 (Fermat)
    for (__int128 b = q0 % q1, e = q1 - 2; e > 0; e >>= 1, b = b * b % q1)
      if (e & 1) q0inv = q0inv * b % q1;
    double worst_bits = 1e9, sum_bits = 0;
    const int nkeys = argc > 4 ? std::max(1, std::atoi(argv[4])) : 1;
    for (int key = 0; key < nkeys; ++key) {
    if (key > 0) {
      sk = key_seed ? PhantomSecretKey::for_testing(ctx, key_seed + key) : PhantomSecretKey(ctx);
      boot.EvalMultKeyGen(sk, ctx);
      boot.EvalBootstrapKeyGen(sk, ctx);
    }
    {  // the secret's value at the first slot's root, s(zeta) with zeta = e^(i pi / N): the rounding
       // bias of a rescale / moddown, -1/2 per coefficient of c0 and c1, sums to (1 + s(zeta)) / (zeta - 1)
       // in that slot and to far less in any other
      std::complex<double> sz = 0;
      const auto& sc = sk.coefficients();
      for (size_t k = 0; k < N; ++k) sz += static_cast<double>(sc[k]) * std::polar(1.0, M_PI * static_cast<double>(k) / N);
      std::printf("{\"key\": %d, \"s_zeta\": [%.2f, %.2f], \"hamming\": %zu}\n", key, sz.real(), sz.imag(),
                  static_cast<size_t>(std::count_if(sc.begin(), sc.end(), [](int8_t v) { return v != 0; })));
    }
    // TAIL_ONLY_I0=1: bootstrap only ciphertexts whose slot 0 has overflow I = 0 in coefficient 0
    // or N/2 (the ~1.3% that expose the slot-0 offset), drawing up to 400 per kept one
    const bool only_i0 = std::getenv("TAIL_ONLY_I0") != nullptr;
    for (int it = 0, tries = 0; it < std::max(1, iters); ++it) {
      std::vector<double> xt(slots);
      for (auto& v : xt) v = dis(rng);
      PhantomPlaintext pin;
      enc.encode(ctx, xt, ct.scale(), pin, ct.chain_index());
      PhantomCiphertext cin;
      sk.encrypt_symmetric(ctx, pin, cin);
      // the overflow of the raised plaintext t = c0 + c1 s = t0 + q0 I (|t| << q0 q1 / 2): t0 the
      // centered residue mod q0, I = (t1 - t0) q0^-1 mod q1, centered (CRT of the first two limbs)
      PhantomPlaintext praw;
      sk.decrypt(ctx, boot.RaiseWithCorrection(cin, ctx), praw);
      const std::vector<uint64_t> r = coeffs2(praw);
      std::vector<int> I(N);
      int max_i = 0;
      size_t arg_i = 0;
      for (size_t k = 0; k < N; ++k) {
        const __int128 t0 = centered(r[k], q0);
        const __int128 d = ((__int128)r[N + k] - t0 % (__int128)q1 + 2 * (__int128)q1) % (__int128)q1;
        I[k] = static_cast<int>(centered(static_cast<uint64_t>(d * q0inv % (__int128)q1), q1));
        if (std::abs(I[k]) > max_i) { max_i = std::abs(I[k]); arg_i = k; }
      }
      if (only_i0 && I[0] != 0 && I[N / 2] != 0) {
        if (++tries > 400 * std::max(1, iters)) break;
        --it;
        continue;
      }
      PhantomCiphertext o = boot.EvalBootstrap(cin, ctx);
      // the same input bootstrapped again must give the same ciphertext bit for bit (the
      // computation is deterministic; a difference would be a race)
      PhantomCiphertext o2 = boot.EvalBootstrap(cin, ctx);
      PHX_CHECK(hipDeviceSynchronize());  // the context's streams do not synchronise with hipMemcpy
      const size_t words = o.size() * o.coeff_modulus_size() * N;
      std::vector<uint64_t> h1(words), h2(words);
      PHX_CHECK(hipMemcpy(h1.data(), o.data(), words * 8, hipMemcpyDeviceToHost));
      PHX_CHECK(hipMemcpy(h2.data(), o2.data(), words * 8, hipMemcpyDeviceToHost));
      const bool repeat_equal = h1 == h2;
      g_ok &= repeat_equal;
      std::vector<std::complex<double>> z = decrypt_decode(ctx, sk, enc, o);
      std::vector<double> res(slots);
      for (size_t j = 0; j < slots; ++j) res[j] = z[j].real();
      const double bits = compute_bit_precision(xt, res);
      worst_bits = std::min(worst_bits, bits);
      sum_bits += bits;
      // output error per coefficient, in units of the output scale
      PhantomPlaintext pout, pref;
      sk.decrypt(ctx, o, pout);
      enc.encode(ctx, xt, o.scale(), pref, o.chain_index());
      const std::vector<uint64_t> a = coeffs2(pout), b = coeffs2(pref);
      std::vector<double> e(N);
      double ss = 0;
      for (size_t k = 0; k < N; ++k) {
        const uint64_t d = a[k] >= b[k] ? a[k] - b[k] : a[k] + q0 - b[k];
        e[k] = static_cast<double>(centered(d, q0)) / o.scale();
        ss += e[k] * e[k];
      }
      std::vector<size_t> idx(N);
      for (size_t k = 0; k < N; ++k) idx[k] = k;
      std::partial_sort(idx.begin(), idx.begin() + 4, idx.end(),
                        [&](size_t u, size_t v) { return std::abs(e[u]) > std::abs(e[v]); });
      // mean |e| by the distance d of I to the nearest multiple of 32, where the double-angle
      // steps amplify an error of the series most (64 / |sin(pi (I + f - 1/4) / 32)|); bands
      // d = 0, 1, 2-3, 4-7, 8-16; coefficients 0 and N/2 (slot 0 of CoeffToSlot) left out
      double band_sum[9] = {0}, band_n[9] = {0};
      for (size_t k = 1; k < N; ++k) {
        if (k == N / 2) continue;
        const int r = ((I[k] % 32) + 32) % 32, d = std::min(r, 32 - r);
        const int bnd = d == 0 ? 0 : d == 1 ? 1 : d <= 3 ? 2 : d <= 7 ? 3 : 4;
        band_sum[bnd] += std::abs(e[k]);
        band_n[bnd] += 1;
      }
      // coefficients with I = 0 other than 0 and N/2: the double-angle steps amplify their error most
      double z_sum = 0, z_max = 0, z_n = 0;
      for (size_t k = 1; k < N; ++k) {
        if (k == N / 2 || I[k] != 0) continue;
        z_sum += std::abs(e[k]);
        z_max = std::max(z_max, std::abs(e[k]));
        z_n += 1;
      }
      // the same message under a second, independent encryption
      PhantomCiphertext cin2;
      sk.encrypt_symmetric(ctx, pin, cin2);
      PhantomCiphertext o3 = boot.EvalBootstrap(cin2, ctx);
      PhantomPlaintext pout3;
      sk.decrypt(ctx, o3, pout3);
      const std::vector<uint64_t> a3 = coeffs2(pout3);
      const uint64_t d3 = a3[0] >= b[0] ? a3[0] - b[0] : a3[0] + q0 - b[0];
      const double e0_reenc = static_cast<double>(centered(d3, q0)) / o3.scale();
      std::ostringstream top, bands;
      for (int t = 0; t < 4; ++t)
        top << (t ? ", " : "") << "[" << idx[t] << ", " << e[idx[t]] << ", " << I[idx[t]] << "]";
      for (int bnd = 0; bnd < 5; ++bnd)
        bands << (bnd ? ", " : "") << (band_n[bnd] ? band_sum[bnd] / band_n[bnd] : 0.0);
      const double rms = std::sqrt(ss / N);
      std::printf("{\"key\": %d, \"tail\": %d, \"repeat_equal\": %s, \"avg_bits\": %.3f, \"I0\": %d, \"e0\": %.4e, "
                  "\"e0_reencrypted\": %.4e, \"I_half\": %d, \"e_half\": %.4e, \"I_zero_others\": [%.0f, %.3e, %.3e], \"max_abs_I\": %d, \"argmax_I\": %zu, \"err_rms\": %.3e, "
                  "\"top_err_share\": %.4f, \"top_err\": [%s], \"mean_err_by_I_mod32_band\": [%s]}\n",
                  key, it, repeat_equal ? "true" : "false", bits, I[0], e[0], e0_reenc, I[N / 2], e[N / 2], z_n, z_n ? z_sum / z_n : 0.0, z_max, max_i, arg_i, rms, e[idx[0]] * e[idx[0]] / ss, top.str().c_str(), bands.str().c_str());
      std::fflush(stdout);
    }
    }
    std::printf("{\"stage\": \"tail\", \"keys\": %d, \"ciphertexts_per_key\": %d, \"K\": %d, \"min_avg_bits\": %.3f, "
                "\"mean_avg_bits\": %.3f}\n",
                nkeys, std::max(1, iters), K, worst_bits, sum_bits / (nkeys * std::max(1, iters)));
    return g_ok ? 0 : 1;
  }

  if (mode == "prof") {
    // kernel-trace windows for rocprofv3 (tools/prof_windows.py cuts the trace at idle gaps of more
    // than 20 ms): warm-up, then exactly ONE warm bootstrap, then ONE lockstep group of `iters`
    // (default 4) bootstraps on one lane, each between device synchronisations and 100 ms sleeps
    const size_t group = static_cast<size_t>(std::max(2, std::min(iters, 8)));
    std::vector<PhantomCiphertext> batch(group);
    for (size_t i = 0; i < group; ++i) {
      std::vector<double> xi(slots);
      for (auto& v : xi) v = dis(rng);
      PhantomPlaintext p;
      enc.encode(ctx, xi, ct.scale(), p, ct.chain_index());
      sk.encrypt_symmetric(ctx, p, batch[i]);
    }
    auto gap = [] {
      PHX_CHECK(hipDeviceSynchronize());
      const double t = now_ms();
      while (now_ms() - t < 100.0) {
      }
    };
    for (int w = 0; w < 2; ++w) (void)boot.EvalBootstrap(ct, ctx);
    (void)boot.EvalBootstrapBatch(batch, ctx, 1, 0, group);
    gap();
    double a = now_ms();
    PhantomCiphertext one = boot.EvalBootstrap(ct, ctx);
    PHX_CHECK(hipDeviceSynchronize());
    const double ms1 = now_ms() - a;
    gap();
    a = now_ms();
    std::vector<PhantomCiphertext> outs = boot.EvalBootstrapBatch(batch, ctx, 1, 0, group);
    PHX_CHECK(hipDeviceSynchronize());
    const double msg = now_ms() - a;
    gap();
    std::printf("{\"stage\": \"prof\", \"single_ms\": %.2f, \"group\": %zu, \"group_ms\": %.2f}\n", ms1, group, msg);
    return 0;
  }

  if (mode == "batch") {
    // C5 on one GPU: `iters` independent bootstraps, `lanes` of them side by side
    const int lanes = argc > 4 ? std::atoi(argv[4]) : 2;
    const size_t group = argc > 5 ? static_cast<size_t>(std::atoi(argv[5])) : 4;  // lockstep group per lane
    // distinct inputs: fresh encryptions of fresh messages at the drained input's level and scale
    std::vector<PhantomCiphertext> batch(static_cast<size_t>(std::max(1, iters)));
    std::vector<std::vector<double>> xs(batch.size());
    for (size_t i = 0; i < batch.size(); ++i) {
      xs[i].resize(slots);
      for (auto& v : xs[i]) v = dis(rng);
      PhantomPlaintext p;
      enc.encode(ctx, xs[i], ct.scale(), p, ct.chain_index());
      sk.encrypt_symmetric(ctx, p, batch[i]);
    }
    std::vector<PhantomCiphertext> warm = boot.EvalBootstrapBatch(
        std::vector<PhantomCiphertext>(batch.begin(), batch.begin() + std::min<size_t>(batch.size(), lanes)), ctx,
        lanes, 0, group);
    PHX_CHECK(hipDeviceSynchronize());
    const double a = now_ms();
    std::vector<PhantomCiphertext> outs = boot.EvalBootstrapBatch(batch, ctx, lanes, 0, group);
    PHX_CHECK(hipDeviceSynchronize());
    const double ms = now_ms() - a;
    double worst = 1e9;
    for (size_t i = 0; i < outs.size(); ++i) {
      std::vector<std::complex<double>> z = decrypt_decode(ctx, sk, enc, outs[i]);
      std::vector<double> res(slots);
      for (size_t j = 0; j < slots; ++j) res[j] = z[j].real();
      worst = std::min(worst, compute_bit_precision(xs[i], res));
    }
    // the batch (lanes, `group` bootstraps in lockstep per lane) equals bootstrapping one at a time,
    // bit for bit (the first 8: at least one whole group)
    bool same = true;
    for (size_t i = 0; i < std::min<size_t>(outs.size(), 8); ++i) {
      const PhantomCiphertext one = boot.EvalBootstrap(batch[i], ctx);
      same &= one.to_host(ctx.stream()) == outs[i].to_host(ctx.stream()) && one.scale() == outs[i].scale() &&
              one.chain_index() == outs[i].chain_index();
    }
    report("batch_equals_single_bitexact", same ? 0.0 : 1.0, 0.5, outs.empty() ? 0 : outs[0].chain_index());
    std::printf("{\"stage\": \"batch\", \"bootstraps\": %zu, \"lanes\": %d, \"group\": %zu, \"ms_total\": %.2f, "
                "\"bootstraps_per_s\": %.3f, \"min_avg_bits\": %.2f}\n",
                outs.size(), lanes, group, ms, 1e3 * outs.size() / ms, worst);
    g_ok &= worst > 9.85;
    std::printf("{\"done\": \"batch\", \"ok\": %s}\n", g_ok ? "true" : "false");
    return g_ok ? 0 : 1;
  }

  PhantomCiphertext out;
  std::vector<double> times, host_times;  // host_times: until EvalBootstrap returns (enqueue side)
  uint64_t tk = 0, tp = 0, tc = 0;
  for (int it = 0; it < std::max(1, iters); ++it) {
    PHX_CHECK(hipDeviceSynchronize());
    auto& tr = traffic::counters();
    const uint64_t k0 = tr.keys, p0 = tr.plaintexts, c0 = tr.ciphertexts;
    const double a = now_ms();
    out = boot.EvalBootstrap(ct, ctx);
    tk = tr.keys - k0;
    tp = tr.plaintexts - p0;
    tc = tr.ciphertexts - c0;
    host_times.push_back(now_ms() - a);
    PHX_CHECK(hipDeviceSynchronize());
    times.push_back(now_ms() - a);
  }
  std::sort(host_times.begin(), host_times.end());
  std::vector<std::complex<double>> z = decrypt_decode(ctx, sk, enc, out);
  std::vector<double> res(slots);
  for (size_t j = 0; j < slots; ++j) res[j] = z[j].real();
  const double bits_avg = compute_bit_precision(x, res);
  const double err = max_abs_err(z, xz);
  std::sort(times.begin(), times.end());
  const size_t levels_after = ctx.size_Q() - out.chain_index();  // remaining levels (limbs - 1)
  double total = 0;
  for (double t : times) total += t;
  std::printf("{\"stage\": \"bootstrap\", \"ms_total\": %.2f, \"ms_median\": %.2f, \"ms_min\": %.2f, \"host_ms_median\": %.2f, \"runs\": %zu, \"avg_bits\": %.2f, "
              "\"max_abs_err\": %.3e, \"chain_in\": %zu, \"chain_out\": %zu, \"levels_after\": %zu, "
              "\"alg_bytes\": {\"keys\": %llu, \"plaintexts\": %llu, \"ciphertexts\": %llu}}\n",
              total, times[times.size() / 2], times[0], host_times[host_times.size() / 2], times.size(), bits_avg, err,
              ct.chain_index(), out.chain_index(),
              levels_after, (unsigned long long)tk, (unsigned long long)tp, (unsigned long long)tc);
  g_ok &= bits_avg > 9.85;
  if (mode == "deferred") report("deferred_encoded_by_bootstrap", boot.precomputed() ? 0.0 : 1.0, 0.5, out.chain_index());
  std::printf("{\"done\": \"boot\", \"ok\": %s}\n", g_ok ? "true" : "false");
  return g_ok ? 0 : 1;
}
