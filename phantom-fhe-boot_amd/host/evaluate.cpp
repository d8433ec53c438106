#include "evaluate.h"

#include <cmath>
#include <map>
#include <mutex>
#include <stdexcept>

#include "../csrc/rns.h"
#include "numth.h"
#include "traffic.h"

namespace phantom {

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
  hip_ok(phx::keyswitch_inner_prod(t_mod_up, evk, cx, ctx.mod_QP().q, ctx.mod_QP().barrett, n, size_Ql,
                                   ctx.size_Q(), ctx.size_P(), beta, s),
         "keyswitch inner product");
  traffic::keys(traffic::limb_bytes(beta * 2 * size_QlP, n));
  traffic::ciphertexts(traffic::limb_bytes(5 * size_Ql, n));  // c2 + (c0, c1) read, (c0, c1) written
  rt.moddown_add(ct, cx, true, ctx.gpu_rns_tables(), s, 2);
}

void keyswitch_inplace(const PhantomContext& ctx, PhantomCiphertext& ct, const uint64_t* c2,
                       const uint64_t* const* evk) {
  keyswitch_raw(ctx, ct.chain_index(), ct.data(), c2, evk, ctx.stream());
}

static void check_same(const PhantomCiphertext& a, const PhantomCiphertext& b) {
  if (a.chain_index() != b.chain_index()) throw std::invalid_argument("encrypted1 and encrypted2 parameter mismatch");
  if (a.is_ntt_form() != b.is_ntt_form()) throw std::invalid_argument("NTT form mismatch");
}

void add_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b) {
  check_same(a, b);
  if (a.size() != b.size()) throw std::invalid_argument("poly number mismatch");
  const size_t n = ctx.poly_degree(), L = a.coeff_modulus_size();
  hip_ok(phx::poly_add(a.data(), b.data(), a.data(), ctx.mod_QP(), n, L, ctx.stream(), a.size()), "add");
  traffic::ciphertexts(traffic::limb_bytes(3 * a.size() * L, n));
}

void sub_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b, bool negate) {
  check_same(a, b);
  if (a.size() != b.size()) throw std::invalid_argument("poly number mismatch");
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

void add_plain_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomPlaintext& p) {
  if (a.chain_index() != p.chain_index()) throw std::invalid_argument("encrypted and plain parameter mismatch");
  hip_ok(phx::poly_add(a.data(), p.data(), a.data(), ctx.mod_QP(), ctx.poly_degree(), a.coeff_modulus_size(),
                       ctx.stream()),
         "add_plain");
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
  const size_t n = ctx.poly_degree(), L = a.coeff_modulus_size();
  hipStream_t s = ctx.stream();
  // the tensor product goes straight into a fresh 3-polynomial buffer: no copy of a
  PhantomCiphertext d;
  d.resize(ctx, a.chain_index(), 3, s, false);
  hip_ok(phx::tensor_prod_2x2(a.data(), b.data(), d.data(), ctx.mod_QP(), n, L, s), "tensor");
  d.set_ntt_form(true);
  d.set_scale(a.scale() * b.scale());
  d.set_correction_factor(a.correction_factor());
  d.SetNoiseScaleDeg(a.GetNoiseScaleDeg());
  return d;
}

void multiply_inplace(const PhantomContext& ctx, PhantomCiphertext& a, const PhantomCiphertext& b) {
  a = multiply(ctx, a, b);
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

void rotate_inplace(const PhantomContext& ctx, PhantomCiphertext& a, int step, const PhantomGaloisKey& keys) {
  apply_galois_inplace(ctx, a, galois_elt_from_step(step, ctx.poly_degree()), keys);
}

}  // namespace phantom
