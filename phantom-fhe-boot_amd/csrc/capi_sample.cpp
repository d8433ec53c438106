// capi_sample.cpp — C-ABI of the random samplers (declared in include/phantom_amd.h): the
// ChaCha20 block function on the host, and the device samplers behind key generation and
// encryption (the reference's sample_uniform_poly / sample_error_poly / sample_ternary_poly,
// src/prng.cu).  Tests pin them against an independent restatement (tests/chacha_np.py).
#include <cstring>

#include "../host/capi_internal.h"
#include "../host/context.h"
#include "chacha.h"
#include "ckks.h"
#include "phantom_amd.h"

using phantom::capi::fail;
using phantom::capi::from_hip;

// defined in capi_ckks.cpp
const phantom::PhantomContext& phantom_capi_context(const phantom_context* c);

namespace {
phx::ChaChaKey key_of(const uint32_t* k) {
  phx::ChaChaKey key;
  std::memcpy(key.k, k, sizeof(key.k));
  return key;
}
}  // namespace

extern "C" {

int phantom_chacha20_block(const uint32_t* key, uint64_t counter, uint64_t nonce, uint32_t* out) {
  if (!key || !out) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
  phx::chacha20_block(key_of(key), counter, nonce, out);
  return PHANTOM_OK;
}

int phantom_salsa20_block(const uint8_t* seed, uint64_t nonce, uint32_t* out) {
  if (!seed || !out) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
  phx::salsa20_block(phx::salsa_seed(seed), nonce, out);
  return PHANTOM_OK;
}

int phantom_sample_uniform_seeded(const phantom_context* ctx, const uint8_t* seed, uint64_t* out,
                                  size_t coeff_modulus_size, hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (!seed || !out) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    const phantom::PhantomContext& pc = phantom_capi_context(ctx);
    if (coeff_modulus_size < 1 || coeff_modulus_size > pc.size_QP())
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "limb count exceeds the chain");
    return from_hip(phx::sample_uniform_seeded(out, pc.mod_QP().q, pc.mod_QP().barrett, pc.poly_degree(),
                                               coeff_modulus_size, phx::salsa_seed(seed), stream));
  });
}

int phantom_sample_poly(const phantom_context* ctx, int kind, const uint32_t* key, uint64_t nonce, uint64_t* out,
                        size_t coeff_modulus_size, hipStream_t stream) {
  PHX_CAPI_GUARD({
    if (!key || !out) return fail(PHANTOM_ERR_INVALID_ARGUMENT, "null pointer");
    const phantom::PhantomContext& pc = phantom_capi_context(ctx);
    if (coeff_modulus_size < 1 || coeff_modulus_size > pc.size_QP())
      return fail(PHANTOM_ERR_INVALID_ARGUMENT, "limb count exceeds the chain");
    const size_t n = pc.poly_degree();
    const phx::ChaChaKey k = key_of(key);
    switch (kind) {
      case PHANTOM_SAMPLE_UNIFORM:
        return from_hip(phx::sample_uniform(out, pc.mod_QP().q, pc.mod_QP().barrett, n, coeff_modulus_size, k, nonce,
                                            stream));
      case PHANTOM_SAMPLE_CBD: return from_hip(phx::sample_cbd(out, pc.mod_QP().q, n, coeff_modulus_size, k, nonce, stream));
      case PHANTOM_SAMPLE_TERNARY:
        return from_hip(phx::sample_ternary(out, pc.mod_QP().q, n, coeff_modulus_size, k, nonce, stream));
      default: return fail(PHANTOM_ERR_INVALID_ARGUMENT, "unknown sampler");
    }
  });
}

}  // extern "C"
