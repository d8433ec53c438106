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

/* nwt_2d_radix8_backward_inplace_scale (include/ntt.cuh:213-215): in place, output times scale[limb] */
int phantom_nwt_backward_inplace_scale(uint64_t *inout, const phantom_ntt_tables *tables, size_t coeff_modulus_size,
                                       size_t start_modulus_idx, const uint64_t *scale, const uint64_t *scale_shoup,
                                       hipStream_t stream);
/* nwt_2d_radix8_forward_inplace_include_special_mod (include/ntt.cuh:187-190) */
int phantom_nwt_forward_include_special_mod(uint64_t *inout, const phantom_ntt_tables *tables,
                                            size_t coeff_modulus_size, size_t start_modulus_idx, size_t size_QP,
                                            size_t size_P, hipStream_t stream);
/* nwt_2d_radix8_forward_inplace_fuse_moddown (include/ntt.cuh:176-180, src/ntt/ntt_moddown.cu:106-261):
 * ct = (cx - NTT(delta)) * bigPInv_mod_q per limb; delta (coefficient form) is the NTT input and
 * is not written back (this engine's epilogue form) */
int phantom_nwt_forward_fuse_moddown(uint64_t *ct, const uint64_t *cx, const uint64_t *bigPInv_mod_q,
                                     const uint64_t *bigPInv_mod_q_shoup, uint64_t *delta,
                                     const phantom_ntt_tables *tables, size_t coeff_modulus_size,
                                     size_t start_modulus_idx, hipStream_t stream);
/* fnwt_1d / inwt_1d (include/ntt.cuh:157-169, src/ntt/ntt_1d.cu): the radix-2 single-workgroup path,
 * n = 2^3 .. 2^11 (the 2-D launchers above use it for n < 2^10).  inwt_1d multiplies by
 * scalar[limb] when scalar / scalar_shoup are given (device arrays, may be NULL). */
int phantom_fnwt_1d(uint64_t *inout, const phantom_ntt_tables *tables, size_t coeff_modulus_size,
                    size_t start_modulus_idx, hipStream_t stream);
int phantom_inwt_1d(uint64_t *inout, const phantom_ntt_tables *tables, size_t coeff_modulus_size,
                    size_t start_modulus_idx, const uint64_t *scalar, const uint64_t *scalar_shoup,
                    hipStream_t stream);

/* ---- context (PhantomContext, include/context.cuh:133-272; src/context.cu:121-232) ------ */
typedef struct phantom_context phantom_context;
/* moduli: the full key-level chain (data primes then special_modulus_size special primes),
 * as produced by CoeffModulus::Create; scheme is CKKS. */
int phantom_context_create(size_t poly_modulus_degree, const uint64_t *moduli, size_t count,
                           size_t special_modulus_size, phantom_context **out);
int phantom_context_destroy(phantom_context *ctx);
/* Opt-in extension, no reference counterpart: on != 0 makes every moddown (and moddown +
 * rescale) mean-unbiased by adding floor(ibase / 2) to each output coefficient (DESIGN.md §3,
 * "Where the precision goes"); 0 (the default) restores the reference's arithmetic bit for bit.
 * Also set by PHX_UNBIASED_MODDOWN=1 at phantom_context_create. */
int phantom_context_set_unbiased_moddown(phantom_context *ctx, int on);
/* number of data primes at chain_index (chain 0 = key level Q u P, 1 = Q, ...) */
size_t phantom_context_coeff_modulus_size(const phantom_context *ctx, size_t chain_index);

/* ---- CKKS evaluation on raw device ciphertexts --------------------------------------- */
/* tensor_prod_2x2_rns_poly (src/polymath.cu:501-536) via bgv_ckks_multiply (src/evaluate.cu:415-473):
 * ct1, ct2 are [2][L][n] at chain_index, out [3][L][n] (out may alias ct1's storage if sized for 3) */
int phantom_multiply(const phantom_context *ctx, size_t chain_index, const uint64_t *ct1, const uint64_t *ct2,
                     uint64_t *out, hipStream_t stream);
/* tensor_square_2x2_rns_poly (src/polymath.cu:538-582), the branch bgv_ckks_multiply takes when both
 * operands are the same ciphertext (src/evaluate.cu:443-450): ct [2][L][n] -> out [3][L][n] =
 * (c0^2, 2 c0 c1, c1^2); out may alias ct's storage if sized for 3 */
int phantom_square(const phantom_context *ctx, size_t chain_index, const uint64_t *ct, uint64_t *out,
                   hipStream_t stream);
/* relinearize_inplace (src/evaluate.cu:1552-1589) -> keyswitch_inplace (src/eval_key_switch.cu:112-212):
 * ct is [3][L][n]; on return its first two polys hold the relinearized ciphertext.
 * key_digits: host array of dnum device pointers, each a [2][size_QP][n] key digit. */
int phantom_relinearize(const phantom_context *ctx, size_t chain_index, uint64_t *ct,
                        const uint64_t *const *key_digits, size_t dnum, hipStream_t stream);
/* relinearize_inplace followed by rescale_to_next_inplace (src/evaluate.cu:1552-1589, 1591-1647) as
 * ONE division by P q_last (the bootstrap's EvalMult + ModReduce path): ct3 [3][L][n] at
 * chain_index -> out [2][L-1][n]; the inner product's first L-1 limbs are formed inside the
 * finish (NTT epilogue).  Equals moddown_from_NTT with {q_last} u P as the special basis applied
 * to the P-scaled extended (c0, c1) + KeySwitch(c2). */
int phantom_relinearize_rescale(const phantom_context *ctx, size_t chain_index, const uint64_t *ct3, uint64_t *out,
                                const uint64_t *const *key_digits, size_t dnum, hipStream_t stream);
/* `count` relinearize + rescale products (1 <= count <= 16) in shared launches: every stage of the key
 * switch (modup INTT, digit conversions, digit NTTs, moddown-rescale INTT, conversion, NTT + finish)
 * runs once over all of them.  Product k: ct3 + k ct3_stride ([3][L][n]) -> out + k out_stride
 * ([2][L-1][n]); bit-identical to phantom_relinearize_rescale on each.  The reference issues one
 * relinearize_inplace + rescale_to_next_inplace per product (src/evaluate.cu:1552-1647); EvalMod's
 * Chebyshev ladder and double angle (src/bootstrap.cu:1657-1668, src/evaluate.cu:3264-3535) run
 * their independent products this way.  Not in place: the output range
 * [out, out + (count - 1) out_stride + 2 (L-1) n) must not meet the ct3 range (rejected). */
int phantom_relinearize_rescale_batch(const phantom_context *ctx, size_t chain_index, const uint64_t *ct3,
                                      size_t ct3_stride, size_t count, uint64_t *out, size_t out_stride,
                                      const uint64_t *const *key_digits, size_t dnum, hipStream_t stream);
/* keyswitch_inplace core: ct [2][L][n] += KeySwitch(c2 [L][n]) */
int phantom_keyswitch(const phantom_context *ctx, size_t chain_index, uint64_t *ct, const uint64_t *c2,
                      const uint64_t *const *key_digits, size_t dnum, hipStream_t stream);
/* DRNSTool::modup (src/rns_bconv.cu:530-628): c2 [L][n] NTT form -> t_mod_up [beta][L+P][n] */
int phantom_modup(const phantom_context *ctx, size_t chain_index, const uint64_t *c2, uint64_t *t_mod_up,
                  hipStream_t stream);
/* key_switch_inner_prod (include/evaluate.cuh:27-29, src/eval_key_switch.cu:88-109) */
int phantom_keyswitch_inner_prod(const phantom_context *ctx, size_t chain_index, const uint64_t *t_mod_up,
                                 const uint64_t *const *key_digits, size_t dnum, uint64_t *cx, hipStream_t stream);
/* DBaseConverter::bConv_BEHZ (src/rns_bconv.cu:212-229; bconv_mult_unroll2_kernel :40-69 and
 * bconv_matmul_unroll2_kernel :143-179): dst[j] = sum_i [src_i * qHat_i^-1]_{q_i} * (qHat_i mod p_j)
 * mod p_j for coefficient-form src [ibase_size][n] -> dst [obase_size][n] (device arrays); ibase /
 * obase are host arrays of moduli.  prescale = 0 skips the [x * qHat^-1] step (src already scaled,
 * as the key-switch drivers pass it).  Builds the converter's tables and synchronizes `stream`
 * before returning (a test / one-off entry; the drivers keep converters per level). */
int phantom_fast_bconv(const uint64_t *ibase, size_t ibase_size, const uint64_t *obase, size_t obase_size,
                       const uint64_t *src, uint64_t *dst, size_t n, int prescale, hipStream_t stream);
/* A converter kept across calls, as the reference's DBaseConverter object (include/rns_bconv.cuh
 * DBaseConverter; init at src/rns_bconv.cu:10-38): phantom_bconv_create builds the tables once
 * (the matrix-core fragments included) from host moduli and synchronizes `stream`;
 * phantom_bconv_run is bConv_BEHZ (src/rns_bconv.cu:212-229) with the same meaning as
 * phantom_fast_bconv, asynchronous on `stream`, no allocation; phantom_bconv_destroy frees the
 * tables (the caller makes sure no run on them is still in flight). */
typedef struct phantom_bconv phantom_bconv;
int phantom_bconv_create(const uint64_t *ibase, size_t ibase_size, const uint64_t *obase, size_t obase_size,
                         hipStream_t stream, phantom_bconv **out);
int phantom_bconv_run(const phantom_bconv *conv, const uint64_t *src, uint64_t *dst, size_t n, int prescale,
                      hipStream_t stream);
int phantom_bconv_destroy(phantom_bconv *conv);
/* DRNSTool::moddown_from_NTT (src/rns_bconv.cu:791-843): cx_i [L+P][n] NTT form (P limbs clobbered)
 * -> out [L][n] = (cx_i - NTT(bconv(INTT(cx_i|P)))) * P^-1 */
int phantom_moddown_from_ntt(const phantom_context *ctx, size_t chain_index, uint64_t *cx_i, uint64_t *out,
                             hipStream_t stream);
/* Fused forms used by the bootstrap (no single reference function; each replaces a pair):
 * phantom_moddown_modup: moddown_from_NTT of one extended-basis polynomial followed by the modup of
 * its result (KeySwitchDown + EvalFastRotationPrecompute in EvalLinearTransform's giant steps,
 * src/bootstrap.cu:1335-1348) = modup(moddown(cx_i)) bit for bit.  cx_i [QlP][n] is clobbered;
 * t_mod_up [beta][QlP][n].
 * phantom_moddown_rescale: moddown_from_NTT followed by rescale_to_next as one division by
 * P q_last (the same algorithm with {q_last} u P as the dropped basis): cx [polys][QlP][n] at
 * chain_index (clobbered) -> out [polys][Ql-1][n]. */
int phantom_moddown_modup(const phantom_context *ctx, size_t chain_index, uint64_t *cx_i, uint64_t *t_mod_up,
                          hipStream_t stream);
/* phantom_moddown_modup over `count` independent polynomials in one launch per stage (the giant
 * steps of one linear-transform level, src/bootstrap.cu:1335-1348): polynomial i at
 * cx + i * cx_stride (elements, >= QlP n; clobbered), its digits at t_mod_up + i * beta * QlP * n. */
int phantom_moddown_modup_batch(const phantom_context *ctx, size_t chain_index, uint64_t *cx, size_t count,
                                size_t cx_stride, uint64_t *t_mod_up, hipStream_t stream);
int phantom_moddown_rescale(const phantom_context *ctx, size_t chain_index, uint64_t *cx, uint64_t *out,
                            size_t polys, hipStream_t stream);
/* ---- the bootstrap's own kernels (src/bootstrap.cu:1157-1405, src/evaluate.cu:2299-3940) ------
 * Extended-basis ("Ext") polynomials are [Ql + P][n] at chain_index: the chain's data limbs, then
 * the special primes; Ext ciphertexts are [2][Ql + P][n].  Host arrays carry device pointers or
 * per-limb residues (copied into the launch here). */
/* EvalLinearTransform's hoisted inner sums (src/bootstrap.cu:1322-1332: EvalMultExt +
 * EvalAddExtInPlace, src/evaluate.cu:3786-3874), all giant steps in one launch:
 * outs[i] = sum_{j<g} babies[j] * pts[i g + j] for i < b (babies / outs Ext ciphertexts, pts Ext
 * plaintexts, host arrays of device pointers; g a power of two <= 32, b <= 64) */
int phantom_lt_bsgs(const phantom_context *ctx, size_t chain_index, const uint64_t *const *babies, size_t g,
                    const uint64_t *const *pts, size_t b, uint64_t *const *outs, hipStream_t stream);
/* KeySwitchExt (src/evaluate.cu:3876-3940): ct [2][Ql][n] -> out = P ct in the Ext basis */
int phantom_keyswitch_ext(const phantom_context *ctx, size_t chain_index, const uint64_t *ct, uint64_t *out,
                          hipStream_t stream);
/* EvalFastRotationExt (src/evaluate.cu:3660-3755) with a fused key: inner product of the shared
 * modup digits [beta][Ql+P][n] with the key, + P c0 when add_first (ct's c0 [Ql][n]), then the
 * NTT-domain automorphism of both polynomials: out [2][Ql+P][n] */
int phantom_fast_rotation_ext(const phantom_context *ctx, size_t chain_index, const uint64_t *ct,
                              const uint64_t *digits, const uint64_t *const *key_digits, size_t dnum,
                              uint32_t galois_elt, int add_first, uint64_t *out, hipStream_t stream);
/* the baby steps of a hoisted linear transform in ONE launch (src/bootstrap.cu:1266-1276: the loop
 * of EvalFastRotationExt(.., digits, true) with KeySwitchExt for rotation 0): for k < count,
 * outs[k] [2][Ql+P][n] = phantom_fast_rotation_ext(ct's c0, digits, key_digits[k], galois_elts[k],
 * add_first = 1), or phantom_keyswitch_ext(ct) where key_digits[k] is NULL; ct [2][Ql][n], the
 * shared digits read once.  key_digits: host array of `count` host arrays of dnum device pointers */
int phantom_fast_rotation_ext_batch(const phantom_context *ctx, size_t chain_index, const uint64_t *ct,
                                    const uint64_t *digits, const uint64_t *const *const *key_digits, size_t dnum,
                                    const uint32_t *galois_elts, size_t count, uint64_t *const *outs,
                                    hipStream_t stream);
/* a giant step of the linear transforms (src/bootstrap.cu:1335-1348: KeySwitchDown + Precompute +
 * EvalFastRotationExt + EvalAddExtInPlace) with c0 kept in the Ext basis:
 * acc (+)= automorphism(KS(modup(moddown(ext c1))) + (ext c0, 0)); ext's c1 P limbs are clobbered */
int phantom_rotate_ext_accumulate(const phantom_context *ctx, size_t chain_index, uint64_t *ext,
                                  const uint64_t *const *key_digits, size_t dnum, uint32_t galois_elt, uint64_t *acc,
                                  int accumulate, hipStream_t stream);
/* ---- lockstep groups: `group` (2..8) ciphertexts of one level through the same keys / plaintexts in
 * ONE launch (a bootstrap batch, src/bootstrap.cu:1157-1405 run per ciphertext by the reference).
 * The ciphertexts' workgroups for the same elements run on one XCD, so the shared operand is read
 * from HBM about once per group; every result equals the single-ciphertext entry above on that
 * ciphertext, bit for bit.
 * phantom_lt_bsgs_group: phantom_lt_bsgs for ciphertext c with babies[c] + j baby_stride (words) as
 * baby j; inner sum 0 goes to acc[c], inner sum i >= 1 to giants[c] + (i - 1) giant_stride.
 * g must be 32 and b <= 8 (the bootstrap's CoeffToSlot / SlotToCoeff levels). */
int phantom_lt_bsgs_group(const phantom_context *ctx, size_t chain_index, size_t group,
                          const uint64_t *const *babies, size_t baby_stride, size_t g, const uint64_t *const *pts,
                          size_t b, uint64_t *const *acc, uint64_t *const *giants, size_t giant_stride,
                          hipStream_t stream);
/* phantom_fast_rotation_ext_batch for ciphertext c = (cts[c], digits[c]) with outputs
 * outs[c * count + k]; the entries (key_digits, galois_elts) are shared, and every ciphertext's outputs
 * must sit at the same offsets from its first output (outs[c * count + k] - outs[c * count]). */
int phantom_fast_rotation_ext_batch_group(const phantom_context *ctx, size_t chain_index, size_t group,
                                          const uint64_t *const *cts, const uint64_t *const *digits,
                                          const uint64_t *const *const *key_digits, size_t dnum,
                                          const uint32_t *galois_elts, size_t count, uint64_t *const *outs,
                                          hipStream_t stream);
/* phantom_rotate_ext_accumulate of ext[c] into acc[c] for c < group by the same rotation key */
int phantom_rotate_ext_accumulate_group(const phantom_context *ctx, size_t chain_index, size_t group,
                                        uint64_t *const *ext, const uint64_t *const *key_digits, size_t dnum,
                                        uint32_t galois_elt, uint64_t *const *acc, int accumulate,
                                        hipStream_t stream);
/* the EvalMod products' tensors in ONE launch (count <= 8 jobs at one level, L = Ql limbs each):
 * out[k] [3][L][n] = factors[k] (ct1[k] x ct2[k]), then out[k][p] += c[k] t[k][p] for p < 2 when t[k]
 * (t[k][p] at t[k] + p t_stride; c[k] host residues per limb), then out[k][0] += consts[k] when
 * consts[k] (host residues per limb); factors[k] >= 1 */
int phantom_tensor_lin_batch(const phantom_context *ctx, size_t chain_index, size_t count, const uint64_t *const *ct1,
                             const uint64_t *const *ct2, uint64_t *const *out, const uint64_t *factors,
                             const uint64_t *const *t, size_t t_stride, const uint64_t *const *c,
                             const uint64_t *const *consts, hipStream_t stream);
/* tensor_prod_2x2 with MulAddRescale's linear epilogue: out [3][Ql][n] = f (ct1 x ct2), then
 * out[p] += c t[p] for p < 2 (t[p] at t + p t_stride; f, c: host residues per limb or NULL) */
int phantom_tensor_lin(const phantom_context *ctx, size_t chain_index, const uint64_t *ct1, const uint64_t *ct2,
                       uint64_t *out, const uint64_t *f, const uint64_t *t, size_t t_stride, const uint64_t *c,
                       hipStream_t stream);
/* d[p] = d[p] ca (ca NULL: unscaled) + (p < t_polys ? t[p] cb : 0), d [d_polys][Ql][n] */
int phantom_lin_comb(const phantom_context *ctx, size_t chain_index, uint64_t *d, size_t d_polys, const uint64_t *ca,
                     const uint64_t *t, size_t t_polys, size_t t_stride, const uint64_t *cb, hipStream_t stream);
/* EvalMultConstInplaceCore / MultByIntegerInPlace in residue form (src/evaluate.cu:2299-2412,
 * :3942-3970): out[p] = in[p] c (+ acc[p]) for `polys` polynomials, in[p] at in + p in_stride
 * (0: contiguous) — a larger stride reads the leading Ql limbs of longer polynomials */
int phantom_mul_scalar(const phantom_context *ctx, size_t chain_index, const uint64_t *in, size_t in_stride,
                       const uint64_t *c, const uint64_t *acc, uint64_t *out, size_t polys, hipStream_t stream);
/* Chebyshev leaves of EvalChebyshevSeriesPS (src/evaluate.cu:3264-3535; EvalLinearWSumMutable
 * :3537-3600 + the free term): out[m] = sum_k in[k] coef[m][k] + (cadd[m], 0) for m < M, k < K
 * (in[k] [2][>= Ql][n] with polynomial stride in_stride[k]; coef host [M][K][Ql], cadd [M][Ql]) */
int phantom_leaf_combine(const phantom_context *ctx, size_t chain_index, const uint64_t *const *in,
                         const size_t *in_stride, size_t K, const uint64_t *coef, const uint64_t *cadd,
                         uint64_t *const *out, size_t M, hipStream_t stream);

/* ---- serialization (host memory; no GPU involved) ------------------------------------
 * The byte format of PhantomCiphertext::save / load (include/ciphertext.h:184-225): the header
 * fields one by one (4 x size_t, double, uint64_t, size_t, bool, bool = 58 bytes) followed by
 * size * coeff_modulus_size * poly_modulus_degree uint64_t words. */
typedef struct phantom_ct_header {
  uint64_t chain_index, size, poly_modulus_degree, coeff_modulus_size;
  double scale;
  uint64_t correction_factor, noise_scale_deg;
  int is_ntt_form, is_asymmetric;
} phantom_ct_header;
/* writes the header and data (host) to out[capacity]; *written = bytes (needed size when too small) */
int phantom_ciphertext_serialize(const phantom_ct_header *h, const uint64_t *host_data, uint8_t *out,
                                 size_t capacity, size_t *written);
/* PhantomGaloisKey::save (include/secretkey.h:195-205) of host words (host only, no GPU):
 * host_keys = [count][dnum][2][size_QP][n]; writes count, then per key dnum and dnum key-level
 * ciphertexts (chain 0, size 2, n, size_QP, scale 1, correction 1, degree 1, NTT form, symmetric) */
int phantom_galois_key_serialize(size_t n, size_t size_QP, size_t dnum, size_t count, const uint64_t *host_keys,
                                 uint8_t *out, size_t capacity, size_t *written);
/* parses in[len]; copies the words to host_data[capacity_words] (may be null: header only);
 * *words = the ciphertext's word count */
int phantom_ciphertext_deserialize(const uint8_t *in, size_t len, phantom_ct_header *h, uint64_t *host_data,
                                   size_t capacity_words, size_t *words);

/* rescale_to_next (src/evaluate.cu:1779-1801) -> divide_and_round_q_last_ntt (src/rns.cu:1160-1184):
 * in [polys][L][n] at chain_index -> out [polys][L-1][n] */
int phantom_rescale_to_next(const phantom_context *ctx, size_t chain_index, const uint64_t *in, uint64_t *out,
                            size_t polys, hipStream_t stream);
/* apply_galois_ntt (src/galois.cu:104-119) with the PrecomputeAutoMapKernel table (src/util.cu:941-958);
 * out must not alias in (PHANTOM_ERR_INVALID_ARGUMENT) */
int phantom_apply_galois_ntt(const phantom_context *ctx, uint32_t galois_elt, const uint64_t *in, uint64_t *out,
                             size_t coeff_modulus_size, hipStream_t stream);
/* elementwise ops over limbs [limb_offset, limb_offset + L) of the key-level chain
 * (add_rns_poly / sub_rns_poly / multiply_rns_poly / negate, src/polymath.cu) */
#define PHANTOM_POLY_ADD 0
#define PHANTOM_POLY_SUB 1
#define PHANTOM_POLY_MUL 2
#define PHANTOM_POLY_NEGATE 3
int phantom_poly_op(const phantom_context *ctx, int op, const uint64_t *a, const uint64_t *b, uint64_t *out,
                    size_t limb_offset, size_t coeff_modulus_size, hipStream_t stream);
/* switchModulusKernel as used by RaiseMod (src/evaluate.cu:2414-2503): coefficient-form limb 0
 * lifted to L limbs (centered representative of the q0 residue) */
int phantom_switch_modulus_raise(const phantom_context *ctx, const uint64_t *in_q0, uint64_t *out,
                                 size_t coeff_modulus_size, hipStream_t stream);

/* ---- bootstrapping sessions (bootstrapping/bootstrapping_example.cu:69-160; src/bootstrap.cu) ----
 * A session is the SimpleBootstrapExample set-up as one object: N = 2^log_n, Q = {60, depth x 59},
 * P = special x 60 (CoeffModulus::Create), scale 2^59, levelBudget {enc, dec}, num_slots slots
 * (0 = N/2; a smaller power of two = sparse packing, SparseBootStrapping :200-309), numIterations
 * and precision of EvalBootstrap (src/bootstrap.cu:843-900).  Keys are derived from the 32-byte
 * secret `seed`: every rank of a multi-GPU job that passes the same seed regenerates the same keys,
 * so no key crosses the interconnect.
 * Ciphertexts cross this boundary serialized in PhantomCiphertext::save's byte format
 * (include/ciphertext.h:184-225) and held in DEVICE memory, `stride` bytes apart: the form in which
 * a batch is scattered to ranks and gathered back. */
/* algorithmic HBM bytes of the homomorphic operations issued since the last reset (process-wide,
 * host/traffic.h): out[0] key-switching key bytes, out[1] linear-transform plaintext bytes,
 * out[2] ciphertext operand / result bytes — the numerator of the bootstrap's roofline */
int phantom_traffic_read(uint64_t *out);
int phantom_traffic_reset(void);
/* The engine's device allocator (host/buffer.h DevicePool, the reference's cudaMallocAsync pool with
 * an unbounded release threshold, src/context.cu:127-131): out[0] bytes held from the driver,
 * out[1] bytes live (handed out), out[2] peak live and out[3] peak held since the last reset. */
int phantom_pool_stats(uint64_t *out);
int phantom_pool_reset_peak(void);
/* EvalMod's Chebyshev interpolant (host only): out[degree + 1] = coefficients c of
 * (2 pi)^(-2^-r) cos(2 pi (K y - 1/4) / 2^r) on [-1, 1], r = double_angle_iterations, with
 * p(y) = sum_k c_k T_k(y) (c_0 NOT halved; the reference's tables g_coefficientsUniform/Sparse,
 * include/bootstrap.cuh:217-255, hold 2 c_0 first) */
int phantom_eval_mod_coefficients(uint32_t K, uint32_t double_angle_iterations, int degree, double *out);
typedef struct phantom_boot_session phantom_boot_session;
int phantom_boot_session_create(int log_n, int depth, int special, const uint32_t *level_budget, uint32_t num_slots,
                                uint32_t num_iterations, uint32_t precision, const uint8_t *seed,
                                phantom_boot_session **out);
int phantom_boot_session_destroy(phantom_boot_session *s);
/* encrypt `count` vectors of num_slots reals (values[count][num_slots]) at chain_index with that
 * level's FLEXIBLEAUTO scale; *ct_bytes = the size of one serialized ciphertext */
int phantom_boot_encrypt(phantom_boot_session *s, const double *values, size_t count, size_t chain_index,
                         uint8_t *dev_out, size_t stride, size_t *ct_bytes);
/* size of one serialized bootstrap output */
int phantom_boot_output_bytes(phantom_boot_session *s, size_t *bytes);
/* the same sizes from the session parameters alone (host only, no GPU): one serialized input at
 * chain_index, one serialized output, and the output's chain index */
int phantom_boot_layout(int log_n, int depth, int special, const uint32_t *level_budget, uint32_t num_slots,
                        uint32_t num_iterations, size_t chain_index, size_t *in_bytes, size_t *out_bytes,
                        size_t *out_chain);
/* EvalBootstrap of `count` serialized ciphertexts, `lanes` side by side (EvalBootstrapBatch) */
int phantom_boot_run(phantom_boot_session *s, const uint8_t *dev_in, size_t in_stride, size_t count, uint8_t *dev_out,
                     size_t out_stride, int lanes);
/* phantom_boot_run with each lane bootstrapping `group` ciphertexts (1..8) at a time in lockstep
 * (phantom_boot_run uses 4; 8 is ~1.5% faster at C5 for ~80 GiB more device memory) */
int phantom_boot_run_grouped(phantom_boot_session *s, const uint8_t *dev_in, size_t in_stride, size_t count,
                             uint8_t *dev_out, size_t out_stride, int lanes, int group);
/* decrypt + decode one serialized ciphertext: the real parts of its num_slots slots */
int phantom_boot_decrypt(phantom_boot_session *s, const uint8_t *dev_in, size_t capacity, double *values_out);

/* ---- random sampling (src/prng.cu; seeds: include/prng.cuh:13-24) ---------------------
 * Every draw of key generation and encryption is ChaCha20 keystream (RFC 8439 block function,
 * 64-bit block counter in state words 12-13, 64-bit nonce in words 14-15): draw `nonce` of the
 * stream keyed by key[8].  The reference samples from Salsa20 seeded by std::random_device. */
/* out[16] = ChaCha20 block (host only, no GPU) */
int phantom_chacha20_block(const uint32_t *key, uint64_t counter, uint64_t nonce, uint32_t *out);
/* device polynomial [coeff_modulus_size][n] over the first limbs of the key-level chain:
 *   PHANTOM_SAMPLE_UNIFORM: element e = 128-bit keystream word pair e mod q (sample_uniform_poly)
 *   PHANTOM_SAMPLE_CBD:     centered binomial 21+21 bits of 64-bit word k (sample_error_poly)
 *   PHANTOM_SAMPLE_TERNARY: 64-bit word k mod 3 minus 1 (sample_ternary_poly)
 * the last two write the same signed value to every limb (coefficient form). */
/* the reference's Salsa20 block (src/prng.cu:17-140; host only): seed[64], nonce -> out[16] */
int phantom_salsa20_block(const uint8_t *seed, uint64_t nonce, uint32_t *out);
/* the reference's uniform expansion of a public 64-byte seed (sample_uniform_poly,
 * src/prng.cu:164-197): `a` of a seed-compressed symmetric ciphertext, [coeff_modulus_size][n]
 * over the first limbs of the key-level chain, bit for bit as the reference */
int phantom_sample_uniform_seeded(const phantom_context *ctx, const uint8_t *seed, uint64_t *out,
                                  size_t coeff_modulus_size, hipStream_t stream);
#define PHANTOM_SAMPLE_UNIFORM 0
#define PHANTOM_SAMPLE_CBD 1
#define PHANTOM_SAMPLE_TERNARY 2
int phantom_sample_poly(const phantom_context *ctx, int kind, const uint32_t *key, uint64_t nonce, uint64_t *out,
                        size_t coeff_modulus_size, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* PHANTOM_AMD_H */
