// ckks.h — CKKS kernels beside the hot path: device-side sampling for key generation and
// encryption (the reference samples on the GPU too, src/prng.cu + sample_* in src/secretkey.cu),
// and the small bootstrap helpers of src/evaluate.cu (monomial multiply, extended-basis glue).
#pragma once

#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace phx {

// out[l][k] uniform in [0, q[l]) for l < L, k < n, from a counter-based generator keyed by
// (seed, stream_id).  Residues of a 128-bit random word reduced by Barrett (bias < 2^-64).
hipError_t sample_uniform(uint64_t* out, const uint64_t* q, const uint64_t* barrett, size_t n, size_t L, uint64_t seed,
                          uint64_t stream_id, hipStream_t s);

// out[l][k] = e_k mod q[l] with e_k a centered binomial sample (21 + 21 bits, sigma ~3.24),
// the same e_k for every limb (coefficient form; the caller NTTs it).
hipError_t sample_cbd(uint64_t* out, const uint64_t* q, size_t n, size_t L, uint64_t seed, uint64_t stream_id,
                      hipStream_t s);

// out[l][k] = in[l][k] * c[l] mod q[l] + (acc ? acc[l][k] : 0), Shoup constants c/c_shoup per limb
hipError_t mul_scalar_add(const uint64_t* in, const uint64_t* c, const uint64_t* c_shoup, const uint64_t* acc,
                          uint64_t* out, const uint64_t* q, size_t n, size_t L, hipStream_t s);

}  // namespace phx
