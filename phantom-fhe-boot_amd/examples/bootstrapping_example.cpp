// bootstrapping_example — the reference's bootstrapping/bootstrapping_example.cu
// (SimpleBootstrapExample, lines 69-200) on this engine, plus staged checks of the pieces.
//
// usage: bootstrapping_example [ops|boot] [log_n] [iterations]
//   ops  : encode/encrypt/decrypt, const-mult drain, hoisted rotation, conjugation, multiply,
//          ModRaise; precision of each against the plaintext computation
//   boot : full bootstrap of 2^(log_n - 1) uniform reals in [1, 5] (the example's input),
//          levelBudget {2, 2}, scale 2^59, Q = {60, 29 x 59}, P = 10 x 60
// Prints one JSON object per check; exit status 0 iff every check meets its bound.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <complex>
#include <cstdio>
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

static double max_abs_err(const std::vector<std::complex<double>>& a, const std::vector<std::complex<double>>& b) {
  double m = 0;
  for (size_t i = 0; i < a.size(); ++i) m = std::max(m, std::abs(a[i] - b[i]));
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
  PhantomSecretKey sk(ctx, 0x5EED);
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
  boot.EvalBootstrapSetup(ctx, levelBudget, scale, sf);
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

  PhantomCiphertext out;
  std::vector<double> times;
  for (int it = 0; it < std::max(1, iters); ++it) {
    PHX_CHECK(hipDeviceSynchronize());
    const double a = now_ms();
    out = boot.EvalBootstrap(ct, ctx);
    PHX_CHECK(hipDeviceSynchronize());
    times.push_back(now_ms() - a);
  }
  std::vector<std::complex<double>> z = decrypt_decode(ctx, sk, enc, out);
  std::vector<double> res(slots);
  for (size_t j = 0; j < slots; ++j) res[j] = z[j].real();
  const double bits_avg = compute_bit_precision(x, res);
  const double err = max_abs_err(z, xz);
  std::sort(times.begin(), times.end());
  const size_t levels_after = ctx.size_Q() - out.chain_index();  // remaining levels (limbs - 1)
  std::printf("{\"stage\": \"bootstrap\", \"ms_median\": %.2f, \"ms_min\": %.2f, \"runs\": %zu, \"avg_bits\": %.2f, "
              "\"max_abs_err\": %.3e, \"chain_in\": %zu, \"chain_out\": %zu, \"levels_after\": %zu}\n",
              times[times.size() / 2], times[0], times.size(), bits_avg, err, ct.chain_index(), out.chain_index(),
              levels_after);
  g_ok &= bits_avg > 8.0;
  std::printf("{\"done\": \"boot\", \"ok\": %s}\n", g_ok ? "true" : "false");
  return g_ok ? 0 : 1;
}
