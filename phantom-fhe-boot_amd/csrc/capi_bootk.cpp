// capi_bootk.cpp — C-ABI of the bootstrap's own kernels (declared in include/phantom_amd.h), on
// raw device buffers, so each can be checked bit for bit against the CPU oracle: the hoisted
// linear transforms' inner sums (lt_bsgs), EvalFastRotationExt with its fused epilogue
// (one fused kernel, keyswitch_rotate), the giant-step rotate-and-accumulate, KeySwitchExt, the tensor product with
// MulAddRescale's linear epilogue (tensor_lin), the Chebyshev leaves (leaf_combine) and the
// per-limb scalar kernels.  Host arrays of device pointers and of per-limb residues are copied into
// the kernels' argument blocks or small device tables here (set-up cost, not on the hot path).
#include <cstring>
#include <vector>

#include "../host/buffer.h"
#include "../host/capi_internal.h"
#include "../host/ckks_eval.h"
#include "../host/context.h"
#include "../host/numth.h"
#include "ckks.h"
#include "phantom_amd.h"
#include "rns.h"

using phantom::capi::fail;
using phantom::capi::from_hip;

const phantom::PhantomContext& phantom_capi_context(const phantom_context* c);
const uint64_t* const* phantom_capi_key_array(const phantom_context* c, const uint64_t* const* host, size_t dnum,
                                              size_t need);

namespace {

const phantom::RnsTool& tool_at(const phantom::PhantomContext& pc, size_t chain) {
  if (chain < 1 || chain >= pc.total_parm_size()) throw std::invalid_argument("invalid chain index");
  return pc.get_context_data(chain).gpu_rns_tool();
}

// per-limb residues (reduced mod the chain's primes) + Shoup quotients as kernel arguments
phx::LimbScalars scalars(const phantom::PhantomContext& pc, size_t chain, const uint64_t* v) {
  const auto& mods = pc.get_context_data(chain).moduli();
  if (mods.size() > static_cast<size_t>(phx::kMaxScalarLimbs)) throw std::invalid_argument("too many limbs");
  phx::LimbScalars c;
  for (size_t l = 0; l < mods.size(); ++l) {
    c.v[l] = v[l] % mods[l];
    c.vs[l] = phantom::arith::shoup(c.v[l], mods[l]);
  }
  return c;
}

}  // namespace

extern "C" {

int phantom_lt_bsgs(const phantom_context* ctx, size_t chain_index, const uint64_t* const* babies, size_t g,
                    const uint64_t* const* pts, size_t b, uint64_t* const* outs, hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& pc = phantom_capi_context(ctx);
    const auto& rt = tool_at(pc, chain_index);
    if (!babies || !pts || !outs) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    if (g < 1 || g > static_cast<size_t>(phx::kLtMaxG) || (g & (g - 1)) || b < 1 || b > static_cast<size_t>(phx::kLtMaxB))
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "baby steps must be a power of two <= 32, giant steps <= 64");
    phx::LtArgs a;
    a.g = static_cast<int>(g);
    a.b = static_cast<int>(b);
    a.Ql = static_cast<int>(rt.size_Ql());
    a.P = static_cast<int>(pc.size_P());
    a.size_Q = static_cast<int>(pc.size_Q());
    a.q = pc.mod_QP().q;
    a.barrett = pc.mod_QP().barrett;
    a.q60 = phantom::below_2_60(pc.key_moduli());
    for (size_t j = 0; j < g; ++j) a.baby[j] = babies[j];
    for (size_t i = 0; i < b; ++i) a.out[i] = outs[i];
    phantom::DeviceBuffer<const uint64_t*> table;
    table.upload(std::vector<const uint64_t*>(pts, pts + g * b), stream);
    a.pts = table.get();
    const hipError_t e = phx::lt_bsgs(a, pc.poly_degree(), stream);
    PHX_CHECK(hipStreamSynchronize(stream));  // the pointer table is freed on return
    return from_hip(e);
  });
}

int phantom_keyswitch_ext(const phantom_context* ctx, size_t chain_index, const uint64_t* ct, uint64_t* out,
                          hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& pc = phantom_capi_context(ctx);
    const auto& rt = tool_at(pc, chain_index);
    const size_t n = pc.poly_degree(), Ql = rt.size_Ql(), QlP = Ql + pc.size_P();
    PHX_CHECK(hipMemsetAsync(out, 0, 2 * QlP * n * sizeof(uint64_t), stream));
    for (size_t i = 0; i < 2; ++i) {
      const hipError_t e = phx::mul_scalar_add(ct + i * Ql * n, rt.bigP_mod_q(), rt.bigP_mod_q_shoup(), nullptr,
                                               out + i * QlP * n, pc.mod_QP().q, n, Ql, stream);
      if (e != hipSuccess) return from_hip(e);
    }
    return PHANTOM_OK;
  });
}

int phantom_fast_rotation_ext(const phantom_context* ctx, size_t chain_index, const uint64_t* ct,
                              const uint64_t* digits, const uint64_t* const* key_digits, size_t dnum,
                              uint32_t galois_elt, int add_first, uint64_t* out, hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& pc = phantom_capi_context(ctx);
    const auto& rt = tool_at(pc, chain_index);
    const size_t n = pc.poly_degree(), Ql = rt.size_Ql(), QlP = Ql + pc.size_P();
    const uint64_t* const* evk = phantom_capi_key_array(ctx, key_digits, dnum, rt.beta());
    phx::KsRotateArgs g;
    g.digits = digits;
    g.evk = evk;
    g.qp = pc.mod_QP().q;
    g.qp_barrett = pc.mod_QP().barrett;
    g.c0 = ct;
    g.pmod = rt.bigP_mod_q();
    g.pmod_shoup = rt.bigP_mod_q_shoup();
    g.out = out;
    g.perm = pc.galois_perm(galois_elt);
    g.ql = static_cast<uint32_t>(Ql);
    g.qlp = static_cast<uint32_t>(QlP);
    g.size_q = static_cast<uint32_t>(pc.size_Q());
    g.size_p = static_cast<uint32_t>(pc.size_P());
    g.beta = static_cast<uint32_t>(rt.beta());
    return from_hip(phx::keyswitch_rotate(g, add_first ? 1 : 0, n, stream));
  });
}

int phantom_fast_rotation_ext_batch(const phantom_context* ctx, size_t chain_index, const uint64_t* ct,
                                    const uint64_t* digits, const uint64_t* const* const* key_digits, size_t dnum,
                                    const uint32_t* galois_elts, size_t count, uint64_t* const* outs,
                                    hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (count == 0) return PHANTOM_OK;
    if (!ct || !digits || !key_digits || !galois_elts || !outs) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    const auto& pc = phantom_capi_context(ctx);
    const auto& rt = tool_at(pc, chain_index);
    const size_t n = pc.poly_degree(), Ql = rt.size_Ql(), QlP = Ql + pc.size_P();
    std::vector<phx::KsBatchEntry> e(count);
    for (size_t k = 0; k < count; ++k) {
      if (!outs[k]) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null output");
      if (key_digits[k]) {
        e[k].evk = phantom_capi_key_array(ctx, key_digits[k], dnum, rt.beta());
        e[k].perm = pc.galois_perm(galois_elts[k]);
        e[k].binv = pc.galois_block_inv(galois_elts[k]);
      }
      e[k].out_off = outs[k] - outs[0];
    }
    phantom::DeviceBuffer<phx::KsBatchEntry> table;
    table.upload(e, stream);
    phx::KsRotateBatchArgs a;
    a.digits = digits;
    a.entries = table.get();
    a.count = static_cast<uint32_t>(count);
    a.qp = pc.mod_QP().q;
    a.qp_barrett = pc.mod_QP().barrett;
    a.ct = ct;
    a.pmod = rt.bigP_mod_q();
    a.pmod_shoup = rt.bigP_mod_q_shoup();
    a.out = outs[0];
    a.ql = static_cast<uint32_t>(Ql);
    a.qlp = static_cast<uint32_t>(QlP);
    a.size_q = static_cast<uint32_t>(pc.size_Q());
    a.size_p = static_cast<uint32_t>(pc.size_P());
    a.beta = static_cast<uint32_t>(rt.beta());
    return from_hip(phx::keyswitch_rotate_batch(a, n, stream));
  });
}

int phantom_rotate_ext_accumulate(const phantom_context* ctx, size_t chain_index, uint64_t* ext,
                                  const uint64_t* const* key_digits, size_t dnum, uint32_t galois_elt, uint64_t* acc,
                                  int accumulate, hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& pc = phantom_capi_context(ctx);
    const auto& rt = tool_at(pc, chain_index);
    const size_t n = pc.poly_degree(), Ql = rt.size_Ql(), QlP = Ql + pc.size_P();
    const uint64_t* const* evk = phantom_capi_key_array(ctx, key_digits, dnum, rt.beta());
    phantom::DeviceBuffer<uint64_t> digits(rt.beta() * QlP * n, stream);
    rt.moddown_modup(digits.get(), ext + QlP * n, pc.gpu_rns_tables(), stream);
    phx::KsRotateArgs g;
    g.digits = digits.get();
    g.evk = evk;
    g.qp = pc.mod_QP().q;
    g.qp_barrett = pc.mod_QP().barrett;
    g.c0 = ext;
    g.out = acc;
    g.perm = pc.galois_perm(galois_elt);
    g.ql = static_cast<uint32_t>(Ql);
    g.qlp = static_cast<uint32_t>(QlP);
    g.size_q = static_cast<uint32_t>(pc.size_Q());
    g.size_p = static_cast<uint32_t>(pc.size_P());
    g.beta = static_cast<uint32_t>(rt.beta());
    g.accumulate = accumulate != 0;
    return from_hip(phx::keyswitch_rotate(g, 2, n, stream));
  });
}

int phantom_lt_bsgs_group(const phantom_context* ctx, size_t chain_index, size_t group,
                          const uint64_t* const* babies, size_t baby_stride, size_t g, const uint64_t* const* pts,
                          size_t b, uint64_t* const* acc, uint64_t* const* giants, size_t giant_stride,
                          hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& pc = phantom_capi_context(ctx);
    const auto& rt = tool_at(pc, chain_index);
    if (!babies || !pts || !acc || (b > 1 && !giants)) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    if (group < 2 || group > static_cast<size_t>(phx::kLtGroupMax))
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "group must hold 2 to 8 ciphertexts");
    if (g != 32 || b < 1 || b > 8) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "grouped inner sums need g = 32, b <= 8");
    const size_t ext_words = 2 * (rt.size_Ql() + pc.size_P()) * pc.poly_degree();
    if (baby_stride < ext_words || (b > 1 && giant_stride < ext_words))
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "stride below one extended-basis ciphertext");
    phx::LtGroupArgs a;
    a.g = static_cast<int>(g);
    a.b = static_cast<int>(b);
    a.Ql = static_cast<int>(rt.size_Ql());
    a.P = static_cast<int>(pc.size_P());
    a.size_Q = static_cast<int>(pc.size_Q());
    a.q = pc.mod_QP().q;
    a.barrett = pc.mod_QP().barrett;
    a.q60 = phantom::below_2_60(pc.key_moduli());
    a.count = static_cast<int>(group);
    a.baby_stride = baby_stride;
    a.giant_stride = giant_stride;
    for (size_t c = 0; c < group; ++c) {
      if (!babies[c] || !acc[c] || (b > 1 && !giants[c])) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
      a.baby0[c] = babies[c];
      a.acc[c] = acc[c];
      a.giant1[c] = b > 1 ? giants[c] : acc[c];
    }
    phantom::DeviceBuffer<const uint64_t*> table;
    table.upload(std::vector<const uint64_t*>(pts, pts + g * b), stream);
    a.pts = table.get();
    const hipError_t e = phx::lt_bsgs_group(a, pc.poly_degree(), stream);
    PHX_CHECK(hipStreamSynchronize(stream));  // the pointer table is freed on return
    return from_hip(e);
  });
}

int phantom_fast_rotation_ext_batch_group(const phantom_context* ctx, size_t chain_index, size_t group,
                                          const uint64_t* const* cts, const uint64_t* const* digits,
                                          const uint64_t* const* const* key_digits, size_t dnum,
                                          const uint32_t* galois_elts, size_t count, uint64_t* const* outs,
                                          hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (count == 0) return PHANTOM_OK;
    if (!cts || !digits || !key_digits || !galois_elts || !outs) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    if (group < 2 || group > static_cast<size_t>(phx::kKsGroupMax))
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "group must hold 2 to 8 ciphertexts");
    const auto& pc = phantom_capi_context(ctx);
    const auto& rt = tool_at(pc, chain_index);
    const size_t n = pc.poly_degree(), Ql = rt.size_Ql(), QlP = Ql + pc.size_P();
    std::vector<phx::KsBatchEntry> e(count);
    for (size_t k = 0; k < count; ++k) {
      if (key_digits[k]) {
        e[k].evk = phantom_capi_key_array(ctx, key_digits[k], dnum, rt.beta());
        e[k].perm = pc.galois_perm(galois_elts[k]);
        e[k].binv = pc.galois_block_inv(galois_elts[k]);
      }
    }
    for (size_t c = 0; c < group; ++c) {
      if (!cts[c] || !digits[c]) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
      for (size_t k = 0; k < count; ++k) {
        uint64_t* const o = outs[c * count + k];
        if (!o) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null output");
        const int64_t off = o - outs[c * count];
        if (c == 0) e[k].out_off = off;
        else if (off != e[k].out_off)
          return fail(PHANTOM_ERR_INVALID_ARGUMENT, "every ciphertext's outputs must sit at the same offsets");
      }
    }
    phantom::DeviceBuffer<phx::KsBatchEntry> table;
    table.upload(e, stream);
    phx::KsRotateBatchGroupArgs ga;
    ga.count = static_cast<int>(group);
    for (size_t c = 0; c < group; ++c) {
      phx::KsRotateBatchArgs& a = ga.a[c];
      a.digits = digits[c];
      a.entries = table.get();
      a.count = static_cast<uint32_t>(count);
      a.qp = pc.mod_QP().q;
      a.qp_barrett = pc.mod_QP().barrett;
      a.ct = cts[c];
      a.pmod = rt.bigP_mod_q();
      a.pmod_shoup = rt.bigP_mod_q_shoup();
      a.out = outs[c * count];
      a.ql = static_cast<uint32_t>(Ql);
      a.qlp = static_cast<uint32_t>(QlP);
      a.size_q = static_cast<uint32_t>(pc.size_Q());
      a.size_p = static_cast<uint32_t>(pc.size_P());
      a.beta = static_cast<uint32_t>(rt.beta());
      a.q60 = phantom::below_2_60(pc.key_moduli());
    }
    const hipError_t err = phx::keyswitch_rotate_batch_group(ga, n, stream);
    PHX_CHECK(hipStreamSynchronize(stream));  // the entry table is freed on return
    return from_hip(err);
  });
}

int phantom_rotate_ext_accumulate_group(const phantom_context* ctx, size_t chain_index, size_t group,
                                        uint64_t* const* ext, const uint64_t* const* key_digits, size_t dnum,
                                        uint32_t galois_elt, uint64_t* const* acc, int accumulate,
                                        hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (!ext || !acc) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    if (group < 2 || group > static_cast<size_t>(phx::kKsGroupMax))
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "group must hold 2 to 8 ciphertexts");
    const auto& pc = phantom_capi_context(ctx);
    const auto& rt = tool_at(pc, chain_index);
    const size_t n = pc.poly_degree(), Ql = rt.size_Ql(), QlP = Ql + pc.size_P();
    const uint64_t* const* evk = phantom_capi_key_array(ctx, key_digits, dnum, rt.beta());
    const size_t dwords = rt.beta() * QlP * n;
    phantom::DeviceBuffer<uint64_t> digits(group * dwords, stream);
    phx::KsRotateGroupArgs ga;
    ga.count = static_cast<int>(group);
    for (size_t c = 0; c < group; ++c) {
      if (!ext[c] || !acc[c]) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
      rt.moddown_modup(digits.get() + c * dwords, ext[c] + QlP * n, pc.gpu_rns_tables(), stream);
      phx::KsRotateArgs& g = ga.a[c];
      g.digits = digits.get() + c * dwords;
      g.evk = evk;
      g.qp = pc.mod_QP().q;
      g.qp_barrett = pc.mod_QP().barrett;
      g.c0 = ext[c];
      g.out = acc[c];
      g.perm = pc.galois_perm(galois_elt);
      g.ql = static_cast<uint32_t>(Ql);
      g.qlp = static_cast<uint32_t>(QlP);
      g.size_q = static_cast<uint32_t>(pc.size_Q());
      g.size_p = static_cast<uint32_t>(pc.size_P());
      g.beta = static_cast<uint32_t>(rt.beta());
      g.accumulate = accumulate != 0;
    }
    return from_hip(phx::keyswitch_rotate_group(ga, 2, n, stream));
  });
}

int phantom_tensor_lin(const phantom_context* ctx, size_t chain_index, const uint64_t* ct1, const uint64_t* ct2,
                       uint64_t* out, const uint64_t* f, const uint64_t* t, size_t t_stride, const uint64_t* c,
                       hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& pc = phantom_capi_context(ctx);
    const auto& rt = tool_at(pc, chain_index);
    phx::TensorLinArgs a;
    a.ct1 = ct1;
    a.ct2 = ct2;
    a.out = out;
    a.q = pc.mod_QP().q;
    a.barrett = pc.mod_QP().barrett;
    if (f) {
      a.scale = true;
      a.f = scalars(pc, chain_index, f);
    }
    if (t && c) {
      a.t = t;
      a.t_stride = t_stride;
      a.c = scalars(pc, chain_index, c);
    }
    return from_hip(phx::tensor_lin(a, pc.poly_degree(), rt.size_Ql(), stream));
  });
}

int phantom_tensor_lin_batch(const phantom_context* ctx, size_t chain_index, size_t count, const uint64_t* const* ct1,
                             const uint64_t* const* ct2, uint64_t* const* out, const uint64_t* factors,
                             const uint64_t* const* t, size_t t_stride, const uint64_t* const* c,
                             const uint64_t* const* consts, hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& pc = phantom_capi_context(ctx);
    const auto& rt = tool_at(pc, chain_index);
    const size_t L = rt.size_Ql();
    if (!ct1 || !ct2 || !out || !factors) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    if (count < 1 || count > static_cast<size_t>(phx::kTensorBatchMax) ||
        count * 2 * L > static_cast<size_t>(phx::kTensorBatchLimbWords))
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "too many jobs for one launch at this level");
    const auto& mods = rt.base_Ql();
    phx::TensorLinBatchArgs a;
    a.q = pc.mod_QP().q;
    a.barrett = pc.mod_QP().barrett;
    a.L = static_cast<uint32_t>(L);
    a.count = static_cast<uint32_t>(count);
    for (size_t k = 0; k < count; ++k) {
      phx::TensorLinJob& J = a.job[k];
      J.ct1 = ct1[k];
      J.ct2 = ct2[k];
      J.out = out[k];
      J.factor = factors[k];
      J.t = t ? t[k] : nullptr;
      J.t_stride = J.t ? t_stride : 0;
      J.has_const = consts && consts[k] ? 1 : 0;
      uint64_t* cl = a.limb + k * 2 * L;
      if (J.t) {
        if (!c || !c[k]) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "a term needs its constants");
        for (size_t l = 0; l < L; ++l) cl[l] = c[k][l] % mods[l];
      }
      if (J.has_const)
        for (size_t l = 0; l < L; ++l) cl[L + l] = consts[k][l] % mods[l];
    }
    return from_hip(phx::tensor_lin_batch(a, pc.poly_degree(), stream));
  });
}

int phantom_lin_comb(const phantom_context* ctx, size_t chain_index, uint64_t* d, size_t d_polys, const uint64_t* ca,
                     const uint64_t* t, size_t t_polys, size_t t_stride, const uint64_t* cb, hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& pc = phantom_capi_context(ctx);
    const auto& rt = tool_at(pc, chain_index);
    if (!cb) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null term constants");
    const phx::LimbScalars b = scalars(pc, chain_index, cb);
    phx::LimbScalars a;
    if (ca) a = scalars(pc, chain_index, ca);
    return from_hip(phx::lin_comb_v(d, d_polys, ca ? &a : nullptr, t, t_polys, t_stride, b, pc.mod_QP().q,
                                    pc.poly_degree(), rt.size_Ql(), stream));
  });
}

int phantom_mul_scalar(const phantom_context* ctx, size_t chain_index, const uint64_t* in, size_t in_stride,
                       const uint64_t* c, const uint64_t* acc, uint64_t* out, size_t polys, hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& pc = phantom_capi_context(ctx);
    const auto& rt = tool_at(pc, chain_index);
    if (!c) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null constants");
    return from_hip(phx::mul_scalar_v(in, scalars(pc, chain_index, c), out, pc.mod_QP().q, pc.poly_degree(),
                                      rt.size_Ql(), stream, polys, in_stride, acc));
  });
}

int phantom_leaf_combine(const phantom_context* ctx, size_t chain_index, const uint64_t* const* in,
                         const size_t* in_stride, size_t K, const uint64_t* coef, const uint64_t* cadd,
                         uint64_t* const* out, size_t M, hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& pc = phantom_capi_context(ctx);
    const auto& rt = tool_at(pc, chain_index);
    if (!in || !in_stride || !coef || !cadd || !out) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    if (K < 1 || K > static_cast<size_t>(phx::kLeafMaxK) || M < 1 || M > static_cast<size_t>(phx::kLeafMaxM))
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "leaf count out of range");
    const size_t L = rt.size_Ql();
    const auto& mods = pc.get_context_data(chain_index).moduli();
    // device table [values][shoup][cadd] as the kernel reads it (FHECKKSRNS::eval_leaves layout)
    std::vector<uint64_t> tab(2 * M * K * L + M * L);
    for (size_t m = 0; m < M; ++m)
      for (size_t k = 0; k < K; ++k)
        for (size_t l = 0; l < L; ++l) {
          const uint64_t v = coef[(m * K + k) * L + l] % mods[l];
          tab[(m * K + k) * L + l] = v;
          tab[M * K * L + (m * K + k) * L + l] = phantom::arith::shoup(v, mods[l]);
        }
    for (size_t i = 0; i < M * L; ++i) tab[2 * M * K * L + i] = cadd[i] % mods[i % L];
    phantom::DeviceBuffer<uint64_t> d;
    d.upload(tab, stream);
    phx::LeafArgs a;
    a.K = static_cast<int>(K);
    a.M = static_cast<int>(M);
    a.L = static_cast<int>(L);
    a.q = pc.mod_QP().q;
    a.barrett = pc.mod_QP().barrett;
    a.coef = d.get();
    a.cadd = d.get() + 2 * M * K * L;
    for (size_t k = 0; k < K; ++k) {
      a.in[k] = in[k];
      a.in_stride[k] = in_stride[k];
    }
    for (size_t m = 0; m < M; ++m) a.out[m] = out[m];
    const hipError_t e = phx::leaf_combine(a, pc.poly_degree(), stream);
    PHX_CHECK(hipStreamSynchronize(stream));  // the table is freed on return
    return from_hip(e);
  });
}

}  // extern "C"
