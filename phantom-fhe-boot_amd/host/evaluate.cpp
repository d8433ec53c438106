#include "evaluate.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <stdexcept>

#include "../csrc/rns.h"
#include "numth.h"
#include "traffic.h"

namespace phantom {

bool ks_epilogue_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("PHX_KS_EPI");
    return !(e && e[0] == '0');
  }();
  return on;
}

void keyswitch_raw(const PhantomContext& ctx, size_t chain_index, uint64_t* ct, const uint64_t* c2,
                   const uint64_t* const* evk, hipStream_t s) {
  if (ctx.size_P() == 0) throw std::invalid_argument("key switching requires special primes");
  if (chain_index < 1 || chain_index >= ctx.total_parm_size()) throw std::invalid_argument("invalid chain index");
  const size_t n = ctx.poly_degree();
  // levelsDropped = chain_index - 1 (src/eval_key_switch.cu:145-148)
  const RnsTool& rt = ctx.get_context_data(chain_index).gpu_rns_tool();
  const size_t size_Ql = rt.size_Ql(), size_QlP = size_Ql + ctx.size_P(), beta = rt.beta();
  uint64_t* t_mod_up = rt.workspace().get(s, Workspace::kKsModup, beta * size_QlP * n);
  rt.modup(t_mod_up, c2, ctx.gpu_rns_tables(), s);
  uint64_t* cx = rt.workspace().get(s, Workspace::kKsCx, 2 * size_QlP * n);
  // the inner product is formed inside the moddown: its P limbs in the INTT(P) prologue, its Ql
  // limbs in the finish's epilogue (ntt.h ntt_inverse_ks, NttEpilogue::ks_beta), so no limb of it
  // makes an HBM round trip (PHX_KS_EPI=0: the whole inner product in one kernel, as before)
  const bool fuse = ks_epilogue_enabled() && beta <= (size_t)phx::kMaxKsBeta && n >= 1024;
  if (!fuse)
    hip_ok(phx::keyswitch_inner_prod(t_mod_up, evk, cx, ctx.mod_QP().q, ctx.mod_QP().barrett, n, size_Ql,
                                     ctx.size_Q(), ctx.size_P(), beta, s),
           "keyswitch inner product");
  traffic::keys(traffic::limb_bytes(beta * 2 * size_QlP, n));
  traffic::ciphertexts(traffic::limb_bytes(5 * size_Ql, n));  // c2 + (c0, c1) read, (c0, c1) written
  rt.moddown_add(ct, cx, true, ctx.gpu_rns_tables(), s, 2, fuse ? t_mod_up : nullptr, fuse ? evk : nullptr);
}

void keyswitch_inplace(const PhantomContext& ctx, PhantomCiphertext& ct, const uint64_t* c2,
                       const uint64_t* const* evk) {
  keyswitch_raw(ctx, ct.chain_index(), ct.data(), c2, evk, ctx.stream());
}

static void check_same(const PhantomCiphertext& a, const PhantomCiphertext& b) {
  if (a.chain_index() != b.chain_index()) throw std::invalid_argument("encrypted1 and encrypted2 parameter mismatch");
  if (a.is_ntt_form() != b.is_ntt_form()) throw std::invalid_argument("NTT form mismatch");
}

// are_same_scale / are_close (src/evaluate.cu:89-92, include/host/common.h:342-345)
template <typename A, typename B>
static bool same_scale(const A& a, const B& b) {
  const double s1 = a.scale(), s2 = b.scale();
  const double f = std::max({std::fabs(s1), std::fabs(s2), 1.0});
  return std::fabs(s1 - s2) < 1e-6 * f;
}

void add_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b) {
  check_same(a, b);
  if (a.size() != b.size()) throw std::invalid_argument("poly number mismatch");
  if (a.GetNoiseScaleDeg() != b.GetNoiseScaleDeg()) throw std::invalid_argument("noise mismatch");
  const size_t n = ctx.poly_degree(), L = a.coeff_modulus_size();
  hip_ok(phx::poly_add(a.data(), b.data(), a.data(), ctx.mod_QP(), n, L, ctx.stream(), a.size()), "add");
  traffic::ciphertexts(traffic::limb_bytes(3 * a.size() * L, n));
}

void sub_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b, bool negate) {
  check_same(a, b);
  if (a.size() != b.size()) throw std::invalid_argument("poly number mismatch");
  if (a.GetNoiseScaleDeg() != b.GetNoiseScaleDeg()) throw std::invalid_argument("noise mismatch");
  const size_t n = ctx.poly_degree(), L = a.coeff_modulus_size();
  uint64_t* x = a.data();
  const uint64_t* y = b.data();
  if (negate) hip_ok(phx::poly_sub(y, x, x, ctx.mod_QP(), n, L, ctx.stream(), a.size()), "sub");
  else hip_ok(phx::poly_sub(x, y, x, ctx.mod_QP(), n, L, ctx.stream(), a.size()), "sub");
  traffic::ciphertexts(traffic::limb_bytes(3 * a.size() * L, n));
}

void negate_inplace(const PhantomContext& ctx, PhantomCiphertext& a) {
  const size_t n = ctx.poly_degree(), L = a.coeff_modulus_size();
  hip_ok(phx::poly_negate(a.data(), a.data(), ctx.mod_QP(), n, L, ctx.stream(), a.size()), "negate");
}

void add_many(const PhantomContext& ctx, const std::vector<PhantomCiphertext>& v, PhantomCiphertext& dst) {
  if (v.empty()) throw std::invalid_argument("encrypteds cannot be empty");
  for (const auto& c : v) {
    if (&c == &dst) throw std::invalid_argument("encrypteds must be different from destination");
    if (c.chain_index() != v[0].chain_index()) throw std::invalid_argument("encrypteds parameter mismatch");
    if (c.is_ntt_form() != v[0].is_ntt_form()) throw std::invalid_argument("NTT form mismatch");
    if (!same_scale(c, v[0])) throw std::invalid_argument("scale mismatch");
    if (c.size() != v[0].size()) throw std::invalid_argument("poly number mismatch");
  }
  const size_t n = ctx.poly_degree(), L = v[0].coeff_modulus_size(), polys = v[0].size();
  hipStream_t s = ctx.stream();
  dst.resize(ctx, v[0].chain_index(), polys, s, false);
  dst.set_ntt_form(v[0].is_ntt_form());
  dst.set_scale(v[0].scale());
  dst.set_correction_factor(v[0].correction_factor());
  dst.SetNoiseScaleDeg(v[0].GetNoiseScaleDeg());
  for (size_t i0 = 0; i0 < v.size(); i0 += phx::kAddManyMax) {
    phx::AddManyArgs a;
    a.count = static_cast<int>(std::min<size_t>(phx::kAddManyMax, v.size() - i0));
    a.accumulate = i0 > 0;
    for (int k = 0; k < a.count; ++k) a.in[k] = v[i0 + k].data();
    hip_ok(phx::poly_add_many(a, dst.data(), ctx.mod_QP(), n, L, s, polys, L * n), "add_many");
  }
  traffic::ciphertexts(traffic::limb_bytes((v.size() + 1) * polys * L, n));
}

static void check_plain(const PhantomCiphertext& a, const PhantomPlaintext& p) {
  if (!a.is_ntt_form()) throw std::invalid_argument("CKKS encrypted must be in NTT form");
  if (a.chain_index() != p.chain_index()) throw std::invalid_argument("encrypted and plain parameter mismatch");
  if (!same_scale(a, p)) throw std::invalid_argument("scale mismatch");
}

void add_plain_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomPlaintext& p) {
  check_plain(a, p);
  hip_ok(phx::poly_add(a.data(), p.data(), a.data(), ctx.mod_QP(), ctx.poly_degree(), a.coeff_modulus_size(),
                       ctx.stream()),
         "add_plain");
}

void sub_plain_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomPlaintext& p) {
  check_plain(a, p);
  hip_ok(phx::poly_sub(a.data(), p.data(), a.data(), ctx.mod_QP(), ctx.poly_degree(), a.coeff_modulus_size(),
                       ctx.stream()),
         "sub_plain");
}

void multiply_plain_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomPlaintext& p) {
  if (a.chain_index() != p.chain_index()) throw std::invalid_argument("encrypted and plain parameter mismatch");
  const size_t n = ctx.poly_degree(), L = a.coeff_modulus_size();
  hip_ok(phx::poly_mul(a.data(), p.data(), a.data(), ctx.mod_QP(), n, L, ctx.stream(), a.size(), 0),
         "multiply_plain");
  a.set_scale(a.scale() * p.scale());
}

PhantomCiphertext multiply(const PhantomContext& ctx, const PhantomCiphertext& a, const PhantomCiphertext& b) {
  check_same(a, b);
  if (!a.is_ntt_form()) throw std::invalid_argument("encrypted1 and encrypted2 must be in NTT form");
  if (a.size() != 2 || b.size() != 2) throw std::invalid_argument("only size-2 ciphertexts are supported");
  if (a.GetNoiseScaleDeg() != b.GetNoiseScaleDeg()) throw std::invalid_argument("noise mismatch");
  const size_t n = ctx.poly_degree(), L = a.coeff_modulus_size();
  hipStream_t s = ctx.stream();
  // the tensor product goes straight into a fresh 3-polynomial buffer: no copy of a
  PhantomCiphertext d;
  d.resize(ctx, a.chain_index(), 3, s, false);
  if (&a == &b)  // bgv_ckks_multiply's square branch (src/evaluate.cu:443-450)
    hip_ok(phx::tensor_square_2x2(a.data(), d.data(), ctx.mod_QP(), n, L, s), "tensor square");
  else
    hip_ok(phx::tensor_prod_2x2(a.data(), b.data(), d.data(), ctx.mod_QP(), n, L, s), "tensor");
  d.set_ntt_form(true);
  d.set_scale(a.scale() * b.scale());
  d.set_correction_factor(a.correction_factor());
  d.SetNoiseScaleDeg(a.GetNoiseScaleDeg());
  return d;
}

void multiply_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b) {
  if (!same_scale(a, b)) throw std::invalid_argument("scale mismatch");  // src/evaluate.cu:1191-1192
  a = multiply(ctx, a, b);
}

void multiply_and_relin_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b,
                                const PhantomRelinKey& rlk) {
  if (a.chain_index() != b.chain_index()) throw std::invalid_argument("encrypted1 and encrypted2 parameter mismatch");
  if (a.is_ntt_form() != b.is_ntt_form()) throw std::invalid_argument("NTT form mismatch");
  if (a.size() != b.size()) throw std::invalid_argument("poly number mismatch");
  if (a.GetNoiseScaleDeg() != b.GetNoiseScaleDeg()) throw std::invalid_argument("noise mismatch");
  a = multiply(ctx, a, b);
  relinearize_inplace(ctx, a, rlk);
}

void relinearize_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomRelinKey& rlk) {
  if (a.size() != 3) throw std::invalid_argument("destination_size must be 3");
  if (!a.is_ntt_form()) throw std::invalid_argument("CKKS encrypted must be in NTT form");
  const size_t n = ctx.poly_degree(), L = a.coeff_modulus_size();
  keyswitch_inplace(ctx, a, a.data() + 2 * L * n, rlk.public_keys_ptr());
  a.resize(2, L, n, ctx.stream());
}

PhantomCiphertext rescale_to_next(const PhantomContext& ctx, const PhantomCiphertext& a) {
  if (a.chain_index() + 1 >= ctx.total_parm_size()) throw std::invalid_argument("end of modulus switching chain reached");
  const RnsTool& rt = ctx.get_context_data(a.chain_index()).gpu_rns_tool();
  PhantomCiphertext d;
  d.resize(ctx, a.chain_index() + 1, a.size(), ctx.stream(), false);
  rt.rescale_ntt(a.data(), d.data(), a.size(), ctx.gpu_rns_tables(), ctx.stream());
  d.set_ntt_form(a.is_ntt_form());
  d.set_scale(a.scale() / static_cast<double>(rt.base_Ql().back()));
  d.SetNoiseScaleDeg(a.GetNoiseScaleDeg());
  return d;
}

PhantomCiphertext mod_switch_to(const PhantomContext& ctx, const PhantomCiphertext& a, size_t chain_index) {
  if (chain_index >= ctx.total_parm_size()) throw std::invalid_argument("end of modulus switching chain reached");
  if (chain_index < a.chain_index()) throw std::invalid_argument("cannot switch to higher level modulus");
  const size_t n = ctx.poly_degree(), L = a.coeff_modulus_size();
  PhantomCiphertext d;
  d.resize(ctx, chain_index, a.size(), ctx.stream(), false);
  const size_t Ld = d.coeff_modulus_size();
  // every polynomial's leading Ld limbs in one strided copy
  PHX_CHECK(hipMemcpy2DAsync(d.data(), Ld * n * sizeof(uint64_t), a.data(), L * n * sizeof(uint64_t),
                             Ld * n * sizeof(uint64_t), a.size(), hipMemcpyDeviceToDevice, ctx.stream()));
  d.set_scale(a.scale());
  d.set_ntt_form(a.is_ntt_form());
  d.set_correction_factor(a.correction_factor());
  d.SetNoiseScaleDeg(a.GetNoiseScaleDeg());
  return d;
}

PhantomCiphertext mod_switch_to_next(const PhantomContext& ctx, const PhantomCiphertext& a) {
  return mod_switch_to(ctx, a, a.chain_index() + 1);
}

void mod_switch_to_inplace(const PhantomContext& ctx, PhantomCiphertext& a, size_t chain_index) {
  if (chain_index < a.chain_index()) throw std::invalid_argument("cannot switch to higher level modulus");
  if (chain_index > a.chain_index()) a = mod_switch_to(ctx, a, chain_index);
}

void mod_switch_to_next_inplace(const PhantomContext& ctx, PhantomPlaintext& plain) {
  if (plain.chain_index() + 1 >= ctx.total_parm_size()) throw std::invalid_argument("end of modulus switching chain reached");
  const size_t next = plain.chain_index() + 1, n = ctx.poly_degree();
  PhantomPlaintext d;
  d.resize(ctx, next, ctx.stream());
  PHX_CHECK(hipMemcpyAsync(d.data(), plain.data(), d.coeff_modulus_size() * n * sizeof(uint64_t),
                           hipMemcpyDeviceToDevice, ctx.stream()));
  d.set_scale(plain.scale());
  d.SetNoiseScaleDeg(plain.GetNoiseScaleDeg());
  plain = std::move(d);
}

void mod_switch_to_inplace(const PhantomContext& ctx, PhantomPlaintext& plain, size_t chain_index) {
  if (plain.chain_index() > chain_index) throw std::invalid_argument("cannot switch to higher level modulus");
  if (chain_index >= ctx.total_parm_size()) throw std::invalid_argument("end of modulus switching chain reached");
  if (plain.chain_index() == chain_index) return;
  // one copy of the leading limbs instead of a copy per dropped limb
  const size_t n = ctx.poly_degree();
  PhantomPlaintext d;
  d.resize(ctx, chain_index, ctx.stream());
  PHX_CHECK(hipMemcpyAsync(d.data(), plain.data(), d.coeff_modulus_size() * n * sizeof(uint64_t),
                           hipMemcpyDeviceToDevice, ctx.stream()));
  d.set_scale(plain.scale());
  d.SetNoiseScaleDeg(plain.GetNoiseScaleDeg());
  plain = std::move(d);
}

void apply_galois_inplace(const PhantomContext& ctx, PhantomCiphertext& a, uint32_t elt, const PhantomGaloisKey& keys) {
  if (a.size() != 2) throw std::invalid_argument("encrypted size must be 2");
  const size_t n = ctx.poly_degree(), L = a.coeff_modulus_size();
  hipStream_t s = ctx.stream();
  const uint32_t* perm = ctx.galois_perm(elt);
  DeviceBuffer<uint64_t> temp(L * n, s);
  uint64_t* c0 = a.data();
  uint64_t* c1 = a.data() + L * n;
  hip_ok(phx::galois_ntt(c0, temp.get(), perm, n, L, s), "galois c0");
  PHX_CHECK(hipMemcpyAsync(c0, temp.get(), L * n * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
  hip_ok(phx::galois_ntt(c1, temp.get(), perm, n, L, s), "galois c1");
  PHX_CHECK(hipMemsetAsync(c1, 0, L * n * sizeof(uint64_t), s));
  keyswitch_inplace(ctx, a, temp.get(), keys.get(elt).public_keys_ptr());
}

// non-adjacent form of `value` (naf, include/host/numth.h:17-35): signed powers of two
static std::vector<int> naf(int value) {
  std::vector<int> res;
  const bool sign = value < 0;
  value = std::abs(value);
  for (int i = 0; value; ++i) {
    const int zi = (value & 1) ? 2 - (value & 3) : 0;
    value = (value - zi) >> 1;
    if (zi) res.push_back((sign ? -zi : zi) * (1 << i));
  }
  return res;
}

void rotate_inplace(const PhantomContext& ctx, PhantomCiphertext& a, int step, const PhantomGaloisKey& keys) {
  const size_t n = ctx.poly_degree();
  const uint32_t elt = galois_elt_from_step(step, n);
  if (keys.has(elt)) {
    apply_galois_inplace(ctx, a, elt, keys);
    return;
  }
  // rotate_internal (src/evaluate.cu:1877-1914): compose from the non-adjacent form
  const std::vector<int> parts = naf(step);
  if (parts.size() == 1) throw std::invalid_argument("Galois key not present");
  for (int t : parts)
    if (static_cast<size_t>(std::abs(t)) != (n >> 1)) rotate_inplace(ctx, a, t, keys);
}

void hoisting_inplace(const PhantomContext& ctx, PhantomCiphertext& ct, const PhantomGaloisKey& keys,
                      const std::vector<int>& steps) {
  if (ct.size() > 2) throw std::invalid_argument("ciphertext size must be 2");
  if (steps.empty()) throw std::invalid_argument("hoisting needs at least one step");
  if (ctx.size_P() == 0) throw std::invalid_argument("key switching requires special primes");
  const size_t n = ctx.poly_degree(), L = ct.coeff_modulus_size();
  const RnsTool& rt = ctx.get_context_data(ct.chain_index()).gpu_rns_tool();
  const size_t QlP = L + ctx.size_P(), beta = rt.beta();
  hipStream_t s = ctx.stream();
  std::vector<const PhantomKSwitchKey*> ks;
  std::vector<const uint32_t*> perms;
  for (int step : steps) {
    const uint32_t elt = galois_elt_from_step(step, n);
    if (!keys.has(elt)) throw std::logic_error("Galois key not present in hoisting");
    ks.push_back(&keys.get(elt));
    perms.push_back(ctx.galois_perm(elt));
  }
  // modup of c1 once; every step permutes the digits and accumulates its inner product
  DeviceBuffer<uint64_t> digits(beta * QlP * n, s), rot(beta * QlP * n, s), acc_c0(L * n, s), t_c0(L * n, s);
  DeviceBuffer<uint64_t> acc_cx(2 * QlP * n, s), t_cx(2 * QlP * n, s);
  rt.modup(digits.get(), ct.data() + L * n, ctx.gpu_rns_tables(), s);
  const phx::ModView mql = rt.mod_Ql(), mqlp = rt.mod_QlP();
  for (size_t i = 0; i < steps.size(); ++i) {
    uint64_t* c0_dst = i ? t_c0.get() : acc_c0.get();
    uint64_t* cx_dst = i ? t_cx.get() : acc_cx.get();
    hip_ok(phx::galois_ntt(ct.data(), c0_dst, perms[i], n, L, s), "hoisting c0 automorphism");
    hip_ok(phx::galois_ntt(digits.get(), rot.get(), perms[i], n, beta * QlP, s), "hoisting digit automorphism");
    hip_ok(phx::keyswitch_inner_prod(rot.get(), ks[i]->public_keys_ptr(), cx_dst, ctx.mod_QP().q,
                                     ctx.mod_QP().barrett, n, L, ctx.size_Q(), ctx.size_P(), beta, s),
           "hoisting inner product");
    traffic::keys(traffic::limb_bytes(beta * 2 * QlP, n));
    if (i) {
      hip_ok(phx::poly_add(acc_c0.get(), t_c0.get(), acc_c0.get(), mql, n, L, s), "hoisting c0 sum");
      hip_ok(phx::poly_add(acc_cx.get(), t_cx.get(), acc_cx.get(), mqlp, n, QlP, s, 2), "hoisting cx sum");
    }
  }
  // ct = (acc_c0, 0) + moddown(acc_cx)
  PHX_CHECK(hipMemcpyAsync(ct.data(), acc_c0.get(), L * n * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
  PHX_CHECK(hipMemsetAsync(ct.data() + L * n, 0, L * n * sizeof(uint64_t), s));
  rt.moddown_add(ct.data(), acc_cx.get(), true, ctx.gpu_rns_tables(), s, 2);
}

}  // namespace phantom
