// capi.cpp — extern "C" boundary of libphantom_amd.so (declared in include/phantom_amd.h).
// Converts C++ exceptions into status codes; every compute call is an async enqueue.
#include "phantom_amd.h"

#include <cstring>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../host/capi_internal.h"
#include "../host/hip_check.h"
#include "../host/modulus.h"
#include "../host/ntt_tables.h"
#include "ntt.h"

struct phantom_ntt_tables {
  std::unique_ptr<phantom::DeviceNttTables> dev;
};

namespace phantom::capi {

thread_local std::string g_last_error;

int fail(int code, const char* msg) {
  g_last_error = msg;
  return code;
}

int from_hip(hipError_t e) {
  if (e == hipSuccess) return PHANTOM_OK;
  g_last_error = hipGetErrorString(e);
  return e == hipErrorInvalidValue ? PHANTOM_ERR_INVALID_ARGUMENT : PHANTOM_ERR_HIP;
}

}  // namespace phantom::capi

using phantom::capi::fail;
using phantom::capi::from_hip;

extern "C" {

const char* phantom_status_string(int status) {
  switch (status) {
    case PHANTOM_OK: return "ok";
    case PHANTOM_ERR_INVALID_ARGUMENT: return "invalid argument";
    case PHANTOM_ERR_HIP: return "HIP runtime error";
    case PHANTOM_ERR_LOGIC: return "logic error";
    default: return "internal error";
  }
}

const char* phantom_last_error(void) { return phantom::capi::g_last_error.c_str(); }

const char* phantom_version(void) { return "phantom-amd 0.1 gfx950"; }

int phantom_coeff_modulus_create(size_t poly_modulus_degree, const int* bit_sizes, size_t count, uint64_t* out) {
  PHX_CAPI_GUARD({
    if (!bit_sizes || !out) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    std::vector<int> b(bit_sizes, bit_sizes + count);
    auto mods = phantom::arith::CoeffModulus::Create(poly_modulus_degree, b);
    for (size_t i = 0; i < count; ++i) out[i] = mods[i].value();
    return PHANTOM_OK;
  });
}

int phantom_ntt_tables_create(size_t n, const uint64_t* moduli, size_t num_moduli, phantom_ntt_tables** out) {
  PHX_CAPI_GUARD({
    if (!moduli || !out || num_moduli == 0) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "bad arguments");
    auto t = std::make_unique<phantom_ntt_tables>();
    std::vector<uint64_t> m(moduli, moduli + num_moduli);
    t->dev = std::make_unique<phantom::DeviceNttTables>(n, m, nullptr);
    PHX_CHECK(hipStreamSynchronize(nullptr));
    *out = t.release();
    return PHANTOM_OK;
  });
}

int phantom_ntt_tables_destroy(phantom_ntt_tables* tables) {
  delete tables;
  return PHANTOM_OK;
}

int phantom_ntt_tables_host(const phantom_ntt_tables* tables, size_t i, uint64_t* tw, uint64_t* tw_shoup,
                            uint64_t* itw, uint64_t* itw_shoup, uint64_t* n_inv) {
  PHX_CAPI_GUARD({
    if (!tables || i >= tables->dev->size()) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "bad table index");
    const auto& t = tables->dev->get();
    const size_t n = t.n;
    auto cp = [&](uint64_t* dst, const uint64_t* src) {
      if (dst) PHX_CHECK(hipMemcpy(dst, src + i * n, n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    };
    cp(tw, t.tw); cp(tw_shoup, t.tw_shoup); cp(itw, t.itw); cp(itw_shoup, t.itw_shoup);
    if (n_inv) PHX_CHECK(hipMemcpy(n_inv, t.n_inv + i, sizeof(uint64_t), hipMemcpyDeviceToHost));
    return PHANTOM_OK;
  });
}

static int check_range(const phantom_ntt_tables* t, size_t L, size_t start) {
  if (!t) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null tables");
  if (L == 0 || start + L > t->dev->size())
    return fail(PHANTOM_ERR_INVALID_ARGUMENT, "limb range exceeds the NTT tables");
  return PHANTOM_OK;
}

int phantom_nwt_forward_inplace(uint64_t* inout, const phantom_ntt_tables* tables, size_t L, size_t start,
                                hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (int s = check_range(tables, L, start)) return s;
    const size_t n = tables->dev->n();
    uint64_t* p = inout + start * n;
    return from_hip(phx::ntt_forward(tables->dev->get(), p, p, phx::LimbMap::contiguous((int)L, (int)start), stream));
  });
}

int phantom_nwt_backward_inplace(uint64_t* inout, const phantom_ntt_tables* tables, size_t L, size_t start,
                                 hipStream_t stream) {
  return phantom_nwt_backward(inout, inout, tables, L, start, stream);
}

int phantom_nwt_backward(uint64_t* out, const uint64_t* in, const phantom_ntt_tables* tables, size_t L,
                         size_t start, hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (int s = check_range(tables, L, start)) return s;
    const size_t n = tables->dev->n();
    return from_hip(phx::ntt_inverse(tables->dev->get(), in + start * n, out + start * n,
                                     phx::LimbMap::contiguous((int)L, (int)start), nullptr, nullptr, stream));
  });
}

int phantom_nwt_backward_scale(uint64_t* out, const uint64_t* in, const phantom_ntt_tables* tables, size_t L,
                               size_t start, const uint64_t* scale, const uint64_t* scale_shoup,
                               hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (int s = check_range(tables, L, start)) return s;
    if (!scale || !scale_shoup) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null scale");
    const size_t n = tables->dev->n();
    return from_hip(phx::ntt_inverse(tables->dev->get(), in + start * n, out + start * n,
                                     phx::LimbMap::contiguous((int)L, (int)start), scale, scale_shoup, stream));
  });
}

static phx::LimbMap special_map(size_t L, size_t start, size_t size_QP, size_t size_P) {
  phx::LimbMap m;
  m.num_limbs = (int)L;
  m.split = (int)(L >= size_P ? L - size_P : 0);
  m.first_a = (int)start;
  m.first_b = (int)(size_QP - size_P);
  return m;
}

int phantom_nwt_forward_include_special_mod_exclude_range(uint64_t* inout, const phantom_ntt_tables* tables,
                                                          size_t L, size_t start, size_t size_QP, size_t size_P,
                                                          size_t ex_begin, size_t ex_end, hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (!tables || L == 0 || size_P > L || size_QP > tables->dev->size() || start + L - size_P > size_QP - size_P)
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "bad special-mod limb range");
    if (ex_begin < start || ex_end > start + L || ex_end < ex_begin)
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "Excluded range in NTT is invalid.");
    const size_t n = tables->dev->n();
    phx::LimbMap m = special_map(L, start, size_QP, size_P);
    m.skip_begin = (int)(ex_begin - start);
    m.skip_end = (int)(ex_end - start);
    uint64_t* p = inout + start * n;
    return from_hip(phx::ntt_forward(tables->dev->get(), p, p, m, stream));
  });
}

int phantom_nwt_backward_inplace_include_special_mod(uint64_t* inout, const phantom_ntt_tables* tables, size_t L,
                                                     size_t start, size_t size_QP, size_t size_P,
                                                     hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (!tables || L == 0 || size_QP > tables->dev->size() || size_P > size_QP)
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "bad special-mod limb range");
    const size_t n = tables->dev->n();
    phx::LimbMap m = special_map(L, start, size_QP, size_P);
    uint64_t* p = inout + start * n;
    return from_hip(phx::ntt_inverse(tables->dev->get(), p, p, m, nullptr, nullptr, stream));
  });
}

int phantom_nwt_backward_inplace_scale(uint64_t* inout, const phantom_ntt_tables* tables, size_t L, size_t start,
                                       const uint64_t* scale, const uint64_t* scale_shoup, hipStream_t stream) {
  return phantom_nwt_backward_scale(inout, inout, tables, L, start, scale, scale_shoup, stream);
}

int phantom_nwt_forward_include_special_mod(uint64_t* inout, const phantom_ntt_tables* tables, size_t L, size_t start,
                                            size_t size_QP, size_t size_P, hipStream_t stream) {
  return phantom_nwt_forward_include_special_mod_exclude_range(inout, tables, L, start, size_QP, size_P, start, start,
                                                               stream);
}

int phantom_nwt_forward_fuse_moddown(uint64_t* ct, const uint64_t* cx, const uint64_t* bigPInv_mod_q,
                                     const uint64_t* bigPInv_mod_q_shoup, uint64_t* delta,
                                     const phantom_ntt_tables* tables, size_t L, size_t start, hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (int s = check_range(tables, L, start)) return s;
    if (!ct || !cx || !bigPInv_mod_q || !bigPInv_mod_q_shoup || !delta)
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    const size_t n = tables->dev->n();
    // NTT(delta) is not stored: the epilogue writes ct = (cx - NTT(delta)) P^-1 directly
    phx::NttEpilogue epi;
    epi.c = cx + start * n;
    epi.out = ct + start * n;
    epi.w = bigPInv_mod_q + start;
    epi.ws = bigPInv_mod_q_shoup + start;
    uint64_t* d = delta + start * n;
    return from_hip(phx::ntt_forward_fused(tables->dev->get(), d, d, phx::LimbMap::contiguous((int)L, (int)start),
                                           nullptr, 0, epi, stream));
  });
}

int phantom_fnwt_1d(uint64_t* inout, const phantom_ntt_tables* tables, size_t L, size_t start, hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (int s = check_range(tables, L, start)) return s;
    const size_t n = tables->dev->n();
    return from_hip(phx::ntt_1d_forward(tables->dev->get(), inout + start * n,
                                        phx::LimbMap::contiguous((int)L, (int)start), stream));
  });
}

int phantom_inwt_1d(uint64_t* inout, const phantom_ntt_tables* tables, size_t L, size_t start, const uint64_t* scalar,
                    const uint64_t* scalar_shoup, hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (int s = check_range(tables, L, start)) return s;
    if ((scalar == nullptr) != (scalar_shoup == nullptr)) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "scalar pair");
    const size_t n = tables->dev->n();
    return from_hip(phx::ntt_1d_inverse(tables->dev->get(), inout + start * n,
                                        phx::LimbMap::contiguous((int)L, (int)start), scalar, scalar_shoup, stream));
  });
}

}  // extern "C"
