/*
 * phantom_amd.h — C-ABI of the MI355X-native CKKS hot path (libphantom_amd.so).
 *
 * Plain pointers and sizes only.  Device buffers are caller-owned HIP allocations laid out
 * like the reference's: a polynomial is limb-major uint64_t data[limb * n + k], a ciphertext
 * is poly-major data[(poly * L + limb) * n + k], every value in [0, q_limb).  All compute
 * entry points enqueue asynchronously on the given stream (the reference hard-codes
 * cudaStreamPerThread, e.g. src/evaluate.cu:1200) and return a status code instead of
 * throwing.
 *
 * Each entry point names the reference interface it replaces (file:line, relative to the
 * PhantomFHE repository root).
 */
#ifndef PHANTOM_AMD_H
#define PHANTOM_AMD_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------------------ */
#define PHANTOM_OK 0
#define PHANTOM_ERR_INVALID_ARGUMENT 1 /* std::invalid_argument in the reference (e.g. include/ntt.cuh:149) */
#define PHANTOM_ERR_HIP 2              /* std::runtime_error from PHANTOM_CHECK_CUDA (cuda_wrapper.cuh:19-47) */
#define PHANTOM_ERR_LOGIC 3            /* std::logic_error (e.g. CoeffModulus::Create out of primes) */
#define PHANTOM_ERR_INTERNAL 4

const char *phantom_status_string(int status);
/* message of the last error raised on the calling host thread ("" if none) */
const char *phantom_last_error(void);
/* library build identification, e.g. "phantom-amd 0.1 gfx950" */
const char *phantom_version(void);

/* ---- parameters (src/host/modulus.cu:80-111, src/host/numth.cu:207-332) ----------- */
/* CoeffModulus::Create(poly_modulus_degree, bit_sizes) -> out[count] */
int phantom_coeff_modulus_create(size_t poly_modulus_degree, const int *bit_sizes, size_t count, uint64_t *out);

/* ---- NTT tables (DNTTTable, include/ntt.cuh:36-129; built at src/context.cu:170-183) --- */
typedef struct phantom_ntt_tables phantom_ntt_tables;
int phantom_ntt_tables_create(size_t poly_modulus_degree, const uint64_t *moduli, size_t num_moduli,
                              phantom_ntt_tables **out);
int phantom_ntt_tables_destroy(phantom_ntt_tables *tables);
/* host copies of the tables for modulus index i (each array of length n) */
int phantom_ntt_tables_host(const phantom_ntt_tables *tables, size_t i, uint64_t *tw, uint64_t *tw_shoup,
                            uint64_t *itw, uint64_t *itw_shoup, uint64_t *n_inv);

/* ---- NTT launchers (include/ntt.cuh:157-226) ---------------------------------------- */
/* nwt_2d_radix8_forward_inplace(inout, tables, coeff_modulus_size, start_modulus_idx, stream)
 * (include/ntt.cuh:173-174, src/ntt/fntt_2d.cu:620-653) */
int phantom_nwt_forward_inplace(uint64_t *inout, const phantom_ntt_tables *tables, size_t coeff_modulus_size,
                                size_t start_modulus_idx, hipStream_t stream);
/* nwt_2d_radix8_backward_inplace (include/ntt.cuh:203-204, src/ntt/intt_2d.cu:724-757) */
int phantom_nwt_backward_inplace(uint64_t *inout, const phantom_ntt_tables *tables, size_t coeff_modulus_size,
                                 size_t start_modulus_idx, hipStream_t stream);
/* nwt_2d_radix8_backward(out, in, ...) (include/ntt.cuh:206-207, src/ntt/ntt_modup.cu:9-200) */
int phantom_nwt_backward(uint64_t *out, const uint64_t *in, const phantom_ntt_tables *tables,
                         size_t coeff_modulus_size, size_t start_modulus_idx, hipStream_t stream);
/* nwt_2d_radix8_backward_scale (include/ntt.cuh:209-211, src/ntt/ntt_modup.cu:356-393):
 * out = INTT(in) * scale[limb]; scale/scale_shoup are device arrays of coeff_modulus_size */
int phantom_nwt_backward_scale(uint64_t *out, const uint64_t *in, const phantom_ntt_tables *tables,
                               size_t coeff_modulus_size, size_t start_modulus_idx, const uint64_t *scale,
                               const uint64_t *scale_shoup, hipStream_t stream);
/* nwt_2d_radix8_forward_inplace_include_special_mod_exclude_range (include/ntt.cuh:188-193,
 * src/ntt/ntt_modup.cu:610-657): buffer limbs >= coeff_modulus_size - size_P use the last
 * size_P table rows (the special primes); limbs in [excluded_range_start, excluded_range_end)
 * are skipped. */
int phantom_nwt_forward_include_special_mod_exclude_range(uint64_t *inout, const phantom_ntt_tables *tables,
                                                          size_t coeff_modulus_size, size_t start_modulus_idx,
                                                          size_t size_QP, size_t size_P,
                                                          size_t excluded_range_start, size_t excluded_range_end,
                                                          hipStream_t stream);
/* nwt_2d_radix8_backward_inplace_include_special_mod (include/ntt.cuh:213-216,
 * src/ntt/intt_2d.cu:796-834) */
int phantom_nwt_backward_inplace_include_special_mod(uint64_t *inout, const phantom_ntt_tables *tables,
                                                     size_t coeff_modulus_size, size_t start_modulus_idx,
                                                     size_t size_QP, size_t size_P, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* PHANTOM_AMD_H */
