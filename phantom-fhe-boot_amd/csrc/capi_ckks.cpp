// capi_ckks.cpp — C-ABI entry points for context-level CKKS evaluation on raw device buffers
// (declared in include/phantom_amd.h).  Thin wrappers over the C++ façade in host/.
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "../host/buffer.h"
#include "../host/capi_internal.h"
#include "../host/ckks_eval.h"
#include "../host/context.h"
#include "../host/evaluate.h"
#include "../host/numth.h"
#include "../host/rns_tool.h"
#include "../host/serialize.h"
#include "phantom_amd.h"
#include "rns.h"

struct phantom_context {
  std::unique_ptr<phantom::PhantomContext> ctx;
  std::mutex mu;
  static constexpr size_t kMaxKeyArrays = 256;
  std::map<std::vector<const uint64_t*>, phantom::DeviceBuffer<const uint64_t*>> key_ptrs;  // cached device arrays

  const uint64_t* const* device_key_array(const uint64_t* const* host, size_t dnum, size_t need) {
    if (!host || dnum < need) throw std::invalid_argument("not enough key-switching key digits");
    std::vector<const uint64_t*> v(host, host + dnum);
    std::lock_guard<std::mutex> lk(mu);
    auto it = key_ptrs.find(v);
    if (it == key_ptrs.end()) {
      // bounded: callers that reallocate their keys would otherwise grow the cache forever.
      // Enqueued inner products may still read the arrays, so drain the device first.
      if (key_ptrs.size() >= kMaxKeyArrays) {
        (void)hipDeviceSynchronize();
        key_ptrs.clear();
      }
      phantom::DeviceBuffer<const uint64_t*> d;
      d.upload(v, nullptr);
      it = key_ptrs.emplace(v, std::move(d)).first;
    }
    return it->second.get();
  }
};

using phantom::capi::fail;
using phantom::capi::from_hip;

const phantom::PhantomContext& phantom_capi_context(const phantom_context* c) {
  if (!c || !c->ctx) throw std::invalid_argument("null context");
  return *c->ctx;
}

const uint64_t* const* phantom_capi_key_array(const phantom_context* c, const uint64_t* const* host, size_t dnum,
                                              size_t need) {
  if (!c) throw std::invalid_argument("null context");
  return const_cast<phantom_context*>(c)->device_key_array(host, dnum, need);
}

namespace {
const phantom::RnsTool& tool(const phantom_context* c, size_t chain_index) {
  if (!c) throw std::invalid_argument("null context");
  if (chain_index < 1 || chain_index >= c->ctx->total_parm_size()) throw std::invalid_argument("invalid chain index");
  return c->ctx->get_context_data(chain_index).gpu_rns_tool();
}
}  // namespace

extern "C" {

int phantom_context_create(size_t n, const uint64_t* moduli, size_t count, size_t special, phantom_context** out) {
  PHX_CAPI_GUARD({
    if (!moduli || !out) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    phantom::EncryptionParameters p(phantom::scheme_type::ckks);
    p.set_poly_modulus_degree(n);
    std::vector<phantom::arith::Modulus> m;
    for (size_t i = 0; i < count; ++i) m.emplace_back(moduli[i]);
    p.set_coeff_modulus(m);
    p.set_special_modulus_size(special);
    auto c = std::make_unique<phantom_context>();
    c->ctx = std::make_unique<phantom::PhantomContext>(p, nullptr);
    *out = c.release();
    return PHANTOM_OK;
  });
}

int phantom_context_destroy(phantom_context* ctx) {
  if (ctx) (void)hipDeviceSynchronize();
  delete ctx;
  return PHANTOM_OK;
}

int phantom_context_set_unbiased_moddown(phantom_context* ctx, int on) {
  PHX_CAPI_GUARD({
    if (!ctx) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null context");
    ctx->ctx->set_unbiased_moddown(on != 0);
    return PHANTOM_OK;
  });
}

size_t phantom_context_coeff_modulus_size(const phantom_context* ctx, size_t chain_index) {
  if (!ctx || chain_index >= ctx->ctx->total_parm_size()) return 0;
  return ctx->ctx->get_context_data(chain_index).coeff_modulus_size();
}

int phantom_multiply(const phantom_context* ctx, size_t chain_index, const uint64_t* ct1, const uint64_t* ct2,
                     uint64_t* out, hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& rt = tool(ctx, chain_index);
    return from_hip(phx::tensor_prod_2x2(ct1, ct2, out, ctx->ctx->mod_QP(), ctx->ctx->poly_degree(), rt.size_Ql(),
                                         stream));
  });
}

int phantom_square(const phantom_context* ctx, size_t chain_index, const uint64_t* ct, uint64_t* out,
                   hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& rt = tool(ctx, chain_index);
    return from_hip(phx::tensor_square_2x2(ct, out, ctx->ctx->mod_QP(), ctx->ctx->poly_degree(), rt.size_Ql(), stream));
  });
}

int phantom_keyswitch(const phantom_context* ctx, size_t chain_index, uint64_t* ct, const uint64_t* c2,
                      const uint64_t* const* key_digits, size_t dnum, hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& rt = tool(ctx, chain_index);
    auto* c = const_cast<phantom_context*>(ctx);
    const uint64_t* const* evk = c->device_key_array(key_digits, dnum, rt.beta());
    phantom::keyswitch_raw(*ctx->ctx, chain_index, ct, c2, evk, stream);
    return from_hip(hipGetLastError());
  });
}

int phantom_relinearize(const phantom_context* ctx, size_t chain_index, uint64_t* ct,
                        const uint64_t* const* key_digits, size_t dnum, hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& rt = tool(ctx, chain_index);
    const size_t L = rt.size_Ql(), n = ctx->ctx->poly_degree();
    return phantom_keyswitch(ctx, chain_index, ct, ct + 2 * L * n, key_digits, dnum, stream);
  });
}

int phantom_relinearize_rescale(const phantom_context* ctx, size_t chain_index, const uint64_t* ct3, uint64_t* out,
                                const uint64_t* const* key_digits, size_t dnum, hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& rt = tool(ctx, chain_index);
    auto* c = const_cast<phantom_context*>(ctx);
    const uint64_t* const* evk = c->device_key_array(key_digits, dnum, rt.beta());
    phantom::relinearize_rescale_raw(*ctx->ctx, chain_index, ct3, out, evk, stream);
    return from_hip(hipGetLastError());
  });
}

int phantom_relinearize_rescale_batch(const phantom_context* ctx, size_t chain_index, const uint64_t* ct3,
                                      size_t ct3_stride, size_t count, uint64_t* out, size_t out_stride,
                                      const uint64_t* const* key_digits, size_t dnum, hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& rt = tool(ctx, chain_index);
    const size_t n = ctx->ctx->poly_degree(), L = rt.size_Ql();
    if (!ct3 || !out || count < 1 || count > static_cast<size_t>(phx::kMaxKsProds))
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "bad batch (1 <= count <= 16)");
    if (count > 1 && (ct3_stride < 3 * L * n || out_stride < 2 * (L - 1) * n))
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "batch strides overlap");
    // not in place: the finish reads c0 / c1 of every ct3 ([3][L][n]) while it writes the outputs
    // ([2][L-1][n]) in another layout, so an output range must not meet an input range
    const uintptr_t in0 = reinterpret_cast<uintptr_t>(ct3), out0 = reinterpret_cast<uintptr_t>(out);
    const uintptr_t in1 = in0 + ((count - 1) * ct3_stride + 3 * L * n) * sizeof(uint64_t);
    const uintptr_t out1 = out0 + ((count - 1) * out_stride + 2 * (L - 1) * n) * sizeof(uint64_t);
    if (out0 < in1 && in0 < out1) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "output overlaps the input (not in place)");
    auto* c = const_cast<phantom_context*>(ctx);
    const uint64_t* const* evk = c->device_key_array(key_digits, dnum, rt.beta());
    std::vector<uint64_t*> outs(count);
    for (size_t k = 0; k < count; ++k) outs[k] = out + k * out_stride;
    phantom::relinearize_rescale_batch_raw(*ctx->ctx, chain_index, ct3, ct3_stride, count, outs.data(), evk, stream);
    return from_hip(hipGetLastError());
  });
}

int phantom_modup(const phantom_context* ctx, size_t chain_index, const uint64_t* c2, uint64_t* t_mod_up,
                  hipStream_t stream) {
  PHX_CAPI_GUARD({
    tool(ctx, chain_index).modup(t_mod_up, c2, ctx->ctx->gpu_rns_tables(), stream);
    return from_hip(hipGetLastError());
  });
}

int phantom_keyswitch_inner_prod(const phantom_context* ctx, size_t chain_index, const uint64_t* t_mod_up,
                                 const uint64_t* const* key_digits, size_t dnum, uint64_t* cx, hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& rt = tool(ctx, chain_index);
    auto* c = const_cast<phantom_context*>(ctx);
    const uint64_t* const* evk = c->device_key_array(key_digits, dnum, rt.beta());
    const auto& pc = *ctx->ctx;
    return from_hip(phx::keyswitch_inner_prod(t_mod_up, evk, cx, pc.mod_QP().q, pc.mod_QP().barrett, pc.poly_degree(),
                                              rt.size_Ql(), pc.size_Q(), pc.size_P(), rt.beta(), stream));
  });
}

int phantom_fast_bconv(const uint64_t* ibase, size_t ibase_size, const uint64_t* obase, size_t obase_size,
                       const uint64_t* src, uint64_t* dst, size_t n, int prescale, hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (!ibase || !obase || !src || !dst || ibase_size == 0 || obase_size == 0 || n == 0 || n % 2 != 0)
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "fast_bconv: empty or odd-sized input");
    phantom::DeviceBaseConverter conv;
    conv.init(std::vector<uint64_t>(ibase, ibase + ibase_size), std::vector<uint64_t>(obase, obase + obase_size), stream);
    const hipError_t e = phx::bconv(conv.args(src, dst, prescale != 0), n, stream);
    if (e != hipSuccess) return from_hip(e);
    // the converter's tables are freed on return
    return from_hip(hipStreamSynchronize(stream));
  });
}

struct phantom_bconv {
  phantom::DeviceBaseConverter conv;
};

int phantom_bconv_create(const uint64_t* ibase, size_t ibase_size, const uint64_t* obase, size_t obase_size,
                         hipStream_t stream, phantom_bconv** out) {
  PHX_CAPI_GUARD({
    if (!ibase || !obase || !out || ibase_size == 0 || obase_size == 0)
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "bconv_create: empty base");
    auto h = std::make_unique<phantom_bconv>();
    h->conv.init(std::vector<uint64_t>(ibase, ibase + ibase_size), std::vector<uint64_t>(obase, obase + obase_size),
                 stream);
    PHX_CHECK(hipStreamSynchronize(stream));
    *out = h.release();
    return PHANTOM_OK;
  });
}

int phantom_bconv_run(const phantom_bconv* conv, const uint64_t* src, uint64_t* dst, size_t n, int prescale,
                      hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (!conv || !src || !dst || n == 0 || n % 2 != 0)
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "bconv_run: null handle or odd-sized input");
    const hipError_t e = phx::bconv(conv->conv.args(src, dst, prescale != 0), n, stream);
    return from_hip(e != hipSuccess ? e : hipGetLastError());
  });
}

int phantom_bconv_destroy(phantom_bconv* conv) {
  delete conv;
  return PHANTOM_OK;
}

int phantom_moddown_from_ntt(const phantom_context* ctx, size_t chain_index, uint64_t* cx_i, uint64_t* out,
                             hipStream_t stream) {
  PHX_CAPI_GUARD({
    tool(ctx, chain_index).moddown_add(out, cx_i, false, ctx->ctx->gpu_rns_tables(), stream);
    return from_hip(hipGetLastError());
  });
}

int phantom_moddown_modup(const phantom_context* ctx, size_t chain_index, uint64_t* cx_i, uint64_t* t_mod_up,
                          hipStream_t stream) {
  PHX_CAPI_GUARD({
    tool(ctx, chain_index).moddown_modup(t_mod_up, cx_i, ctx->ctx->gpu_rns_tables(), stream);
    return from_hip(hipGetLastError());
  });
}

int phantom_moddown_modup_batch(const phantom_context* ctx, size_t chain_index, uint64_t* cx, size_t count,
                                size_t cx_stride, uint64_t* t_mod_up, hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (!cx || !t_mod_up || count == 0) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "empty batch");
    tool(ctx, chain_index).moddown_modup(t_mod_up, cx, ctx->ctx->gpu_rns_tables(), stream, count, cx_stride);
    return from_hip(hipGetLastError());
  });
}

int phantom_moddown_rescale(const phantom_context* ctx, size_t chain_index, uint64_t* cx, uint64_t* out, size_t polys,
                            hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& rt = tool(ctx, chain_index);
    if (rt.size_Ql() < 2) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "end of modulus switching chain reached");
    rt.moddown_rescale(out, cx, ctx->ctx->gpu_rns_tables(), stream, polys);
    return from_hip(hipGetLastError());
  });
}

int phantom_galois_key_serialize(size_t n, size_t size_QP, size_t dnum, size_t count, const uint64_t* host_keys,
                                 uint8_t* out, size_t capacity, size_t* written) {
  PHX_CAPI_GUARD({
    if (!written || (count && !host_keys)) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    if (dnum > 64) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "dnum too large");
    const size_t digit = phantom::ser::checked_words(2, size_QP, n);
    const size_t need = 8 + count * (8 + dnum * (phantom::ser::kCiphertextHeaderBytes + digit * sizeof(uint64_t)));
    *written = need;
    if (!out || capacity < need) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "output buffer too small");
    std::ostringstream os;
    phantom::ser::write_u64(os, count);
    for (size_t k = 0; k < count; ++k) {
      std::vector<const uint64_t*> d;
      for (size_t i = 0; i < dnum; ++i) d.push_back(host_keys + (k * dnum + i) * digit);
      phantom::ser::write_kswitch_key(os, n, size_QP, d);
    }
    const std::string b = os.str();
    std::memcpy(out, b.data(), b.size());
    return PHANTOM_OK;
  });
}

int phantom_ciphertext_serialize(const phantom_ct_header* h, const uint64_t* host_data, uint8_t* out, size_t capacity,
                                 size_t* written) {
  PHX_CAPI_GUARD({
    if (!h || !written) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    phantom::ser::CiphertextHeader c;
    c.chain_index = h->chain_index;
    c.size = h->size;
    c.poly_modulus_degree = h->poly_modulus_degree;
    c.coeff_modulus_size = h->coeff_modulus_size;
    c.scale = h->scale;
    c.correction_factor = h->correction_factor;
    c.noise_scale_deg = h->noise_scale_deg;
    c.is_ntt_form = h->is_ntt_form != 0;
    c.is_asymmetric = h->is_asymmetric != 0;
    const size_t need = phantom::ser::kCiphertextHeaderBytes + c.words() * sizeof(uint64_t);
    *written = need;
    if (!out || capacity < need) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "output buffer too small");
    if (c.words() && !host_data) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null data");
    std::ostringstream os;
    phantom::ser::write_ciphertext(os, c, host_data);
    const std::string b = os.str();
    std::memcpy(out, b.data(), b.size());
    return PHANTOM_OK;
  });
}

int phantom_ciphertext_deserialize(const uint8_t* in, size_t len, phantom_ct_header* h, uint64_t* host_data,
                                   size_t capacity_words, size_t* words) {
  PHX_CAPI_GUARD({
    if (!in || !h || !words) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    if (len < phantom::ser::kCiphertextHeaderBytes) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "serialized object truncated");
    phantom::ser::CiphertextHeader c;
    std::vector<uint64_t> v;
    try {
      // the payload must be in the buffer: check the header's word count against len first
      std::istringstream hs(std::string(reinterpret_cast<const char*>(in), phantom::ser::kCiphertextHeaderBytes));
      phantom::ser::read_ciphertext_header(hs, c);
      if (c.words() > (len - phantom::ser::kCiphertextHeaderBytes) / sizeof(uint64_t))
        return fail(PHANTOM_ERR_INVALID_ARGUMENT, "serialized object truncated");
      std::istringstream is(std::string(reinterpret_cast<const char*>(in), len));
      phantom::ser::read_ciphertext(is, c, v);
    } catch (const std::runtime_error& e) {
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, e.what());
    }
    h->chain_index = c.chain_index;
    h->size = c.size;
    h->poly_modulus_degree = c.poly_modulus_degree;
    h->coeff_modulus_size = c.coeff_modulus_size;
    h->scale = c.scale;
    h->correction_factor = c.correction_factor;
    h->noise_scale_deg = c.noise_scale_deg;
    h->is_ntt_form = c.is_ntt_form;
    h->is_asymmetric = c.is_asymmetric;
    *words = v.size();
    if (host_data) {
      if (capacity_words < v.size()) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "output buffer too small");
      std::memcpy(host_data, v.data(), v.size() * sizeof(uint64_t));
    }
    return PHANTOM_OK;
  });
}

int phantom_rescale_to_next(const phantom_context* ctx, size_t chain_index, const uint64_t* in, uint64_t* out,
                            size_t polys, hipStream_t stream) {
  PHX_CAPI_GUARD({
    const auto& rt = tool(ctx, chain_index);
    if (rt.size_Ql() < 2) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "end of modulus switching chain reached");
    rt.rescale_ntt(in, out, polys, ctx->ctx->gpu_rns_tables(), stream);
    return from_hip(hipGetLastError());
  });
}

int phantom_apply_galois_ntt(const phantom_context* ctx, uint32_t galois_elt, const uint64_t* in, uint64_t* out,
                             size_t L, hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (!ctx) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null context");
    const size_t n = ctx->ctx->poly_degree();
    if (!(galois_elt & 1) || galois_elt >= 2 * n) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "invalid Galois element");
    const uint32_t* perm = ctx->ctx->galois_perm(galois_elt);
    return from_hip(phx::galois_ntt(in, out, perm, n, L, stream));
  });
}

int phantom_poly_op(const phantom_context* ctx, int op, const uint64_t* a, const uint64_t* b, uint64_t* out,
                    size_t off, size_t L, hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (!ctx) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null context");
    const auto& pc = *ctx->ctx;
    if (off + L > pc.size_QP()) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "limb range exceeds the chain");
    const phx::ModView m{pc.mod_QP().q + off, pc.mod_QP().barrett + 2 * off};
    const size_t n = pc.poly_degree();
    switch (op) {
      case PHANTOM_POLY_ADD: return from_hip(phx::poly_add(a, b, out, m, n, L, stream));
      case PHANTOM_POLY_SUB: return from_hip(phx::poly_sub(a, b, out, m, n, L, stream));
      case PHANTOM_POLY_MUL: return from_hip(phx::poly_mul(a, b, out, m, n, L, stream));
      case PHANTOM_POLY_NEGATE: return from_hip(phx::poly_negate(a, out, m, n, L, stream));
      default: return fail(PHANTOM_ERR_INVALID_ARGUMENT, "unknown op");
    }
  });
}

int phantom_switch_modulus_raise(const phantom_context* ctx, const uint64_t* in_q0, uint64_t* out, size_t L,
                                 hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (!ctx) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null context");
    const auto& pc = *ctx->ctx;
    if (L > pc.size_Q()) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "too many limbs");
    return from_hip(phx::switch_modulus_raise(in_q0, out, pc.mod_QP().q, pc.mod_QP().barrett, pc.poly_degree(), L,
                                              stream));
  });
}

}  // extern "C"
