/*
 * oracle.h — CPU restatement of PhantomFHE's CKKS hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity checker for the MI355X engine.  Only tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() may load it; the product library
 * (phantom-fhe-boot_amd/) never links or calls it.
 *
 * Every function restates the reference algorithm in plain C with exact 128-bit
 * integer arithmetic and cites the reference file:line it follows
 * (paths relative to the reference repository root).
 *
 * Parity pinning: the reference ships no bit-level golden vectors for this path
 * (test/ntt_test.cu:63-68,116-121 only check INTT(NTT(x)) == x).  The oracle is
 * pinned by (1) the reference's own round-trip test, re-run here at the same sizes
 * and moduli; (2) the modulus values the reference's host code produced for the C3
 * chain, recorded in SURVEY.md §8 and committed as tests/golden/moduli_c3.json;
 * (3) mathematical known-answer tests (naive negacyclic DFT, CRT reconstruction).
 * See DESIGN.md §Oracle.
 *
 * Layout conventions follow the reference: a polynomial is limb-major
 * data[limb * n + k]; a ciphertext is poly-major data[(poly * L + limb) * n + k].
 */
#ifndef PHANTOM_ORACLE_H
#define PHANTOM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- scalar number theory (src/host/numth.cu, src/host/modulus.cu) ---- */
uint64_t or_mulmod(uint64_t a, uint64_t b, uint64_t q);
uint64_t or_powmod(uint64_t a, uint64_t e, uint64_t q);
uint64_t or_invmod(uint64_t a, uint64_t q);
int or_is_prime(uint64_t v);
uint64_t or_shoup(uint64_t w, uint64_t q);
void or_barrett_ratio(uint64_t q, uint64_t out[2]);
int or_get_primes(size_t n, int bit_size, size_t count, uint64_t *out);
int or_coeff_modulus_create(size_t n, const int *bit_sizes, size_t count, uint64_t *out);
uint64_t or_minimal_primitive_root(uint64_t degree, uint64_t q);

/* ---- NTT tables (src/host/ntt.cu:11-56) ---- */
int or_ntt_tables(size_t n, uint64_t q, uint64_t *tw, uint64_t *tw_shoup, uint64_t *itw,
                  uint64_t *itw_shoup, uint64_t *n_inv, uint64_t *n_inv_shoup);

/* ---- NTT (include/butterfly.cuh:10-109, src/ntt/ntt_1d.cu, src/ntt/fntt_2d.cu, intt_2d.cu) ---- */
void or_ntt_fwd(uint64_t *data, size_t n, size_t L, const uint64_t *moduli);
void or_ntt_inv(uint64_t *data, size_t n, size_t L, const uint64_t *moduli);
void or_ntt_fwd_naive(const uint64_t *in, uint64_t *out, size_t n, uint64_t q);
/* precomputed-table form used for CPU baseline timing (tables built once, not per call) */
typedef struct or_ntt_plan or_ntt_plan;
or_ntt_plan *or_ntt_plan_create(size_t n, size_t L, const uint64_t *moduli);
void or_ntt_plan_destroy(or_ntt_plan *plan);
void or_ntt_plan_fwd(const or_ntt_plan *plan, uint64_t *data, size_t L, int threads);
void or_ntt_plan_inv(const or_ntt_plan *plan, uint64_t *data, size_t L, int threads);

/* ---- elementwise RNS polynomial arithmetic (src/polymath.cu) ---- */
void or_poly_add(const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n, size_t L, const uint64_t *moduli);
void or_poly_sub(const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n, size_t L, const uint64_t *moduli);
void or_poly_negate(const uint64_t *a, uint64_t *out, size_t n, size_t L, const uint64_t *moduli);
void or_poly_mul(const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n, size_t L, const uint64_t *moduli);
void or_poly_mul_scalar(const uint64_t *a, const uint64_t *scalars, uint64_t *out, size_t n, size_t L,
                        const uint64_t *moduli);
void or_tensor_prod_2x2(const uint64_t *ct1, const uint64_t *ct2, uint64_t *out, size_t n, size_t L,
                        const uint64_t *moduli);
/* the reference's Salsa20 generator (src/prng.cu:17-140) and uniform sampler (:164-197) */
void or_salsa20_core(const uint32_t in[16], uint32_t out[16]);
void or_salsa20_block(const uint8_t seed[64], uint64_t nonce, uint32_t out[16]);
void or_sample_uniform_seeded(const uint8_t seed[64], const uint64_t *moduli, size_t n, size_t L, uint64_t *out);
void or_tensor_square_2x2(const uint64_t *ct, uint64_t *out, size_t n, size_t L, const uint64_t *moduli);

/* ---- base conversion (src/rns_bconv.cu:22-229, include/host/rns.h:135-199) ---- */
void or_bconv(const uint64_t *in, uint64_t *out, size_t n, const uint64_t *ibase, size_t ibase_size,
              const uint64_t *obase, size_t obase_size);

/* ---- hybrid key switching (src/rns.cu:11-190, src/rns_bconv.cu:530-843, src/eval_key_switch.cu) ---- */
/* qlp = the Ql moduli followed by the size_P special moduli; keys are indexed over the full QP chain. */
void or_modup(const uint64_t *c2_ntt, uint64_t *t_mod_up, size_t n, const uint64_t *ql, size_t size_ql,
              const uint64_t *p, size_t size_p);
void or_keyswitch_inner_prod(const uint64_t *t_mod_up, const uint64_t *const *evk, uint64_t *cx, size_t n,
                             size_t size_ql, size_t size_q, size_t size_p, size_t beta, const uint64_t *qp_full);
void or_moddown_from_ntt(uint64_t *cx_i, uint64_t *ct_out, size_t n, const uint64_t *ql, size_t size_ql,
                         const uint64_t *p, size_t size_p);
void or_keyswitch_add(uint64_t *ct, const uint64_t *c2, const uint64_t *const *evk, size_t n, size_t size_ql,
                      size_t size_q, size_t size_p, const uint64_t *qp_full);
void or_relinearize(uint64_t *ct3, size_t n, size_t size_ql, size_t size_q, size_t size_p,
                    const uint64_t *const *evk, const uint64_t *qp_full);

/* ---- rescale (src/rns.cu:1128-1184, src/evaluate.cu:1591-1647) ---- */
void or_rescale_ntt(const uint64_t *ct, uint64_t *out, size_t n, size_t size_ql, size_t polys,
                    const uint64_t *ql);
void or_mod_switch_drop_ntt(const uint64_t *ct, uint64_t *out, size_t n, size_t size_ql, size_t polys);

/* ---- automorphism (src/util.cu:908-958, src/galois.cu:104-119) ---- */
void or_galois_perm_ntt(uint32_t galois_elt, size_t n, uint32_t *perm);
void or_apply_galois_ntt(const uint64_t *in, uint64_t *out, size_t n, size_t L, uint32_t galois_elt);

/* ---- bootstrap helpers (src/evaluate.cu:2414-2554) ---- */
void or_switch_modulus_raise(const uint64_t *in_q0, uint64_t *out, size_t n, uint64_t q0, const uint64_t *ql,
                             size_t size_ql);
void or_monomial_ntt(uint64_t *out, size_t n, size_t L, const uint64_t *moduli, uint32_t power);

/* ---- bootstrap kernels (src/bootstrap.cu:1157-1405 linear transforms, src/evaluate.cu:2299-3940) ---- */
void or_lt_bsgs(const uint64_t *const *baby, size_t g, const uint64_t *const *pts, size_t b, uint64_t *const *out,
                size_t n, size_t size_ql, size_t size_q, size_t size_p, const uint64_t *qp_full);
void or_keyswitch_ext(const uint64_t *ct, uint64_t *out, size_t n, size_t size_ql, size_t size_q, size_t size_p,
                      const uint64_t *qp_full);
void or_fast_rotation_ext(const uint64_t *c0, const uint64_t *digits, const uint64_t *const *evk, uint32_t galois_elt,
                          int add_first, uint64_t *out, size_t n, size_t size_ql, size_t size_q, size_t size_p,
                          const uint64_t *qp_full);
void or_rotate_ext_accumulate(uint64_t *ext, const uint64_t *const *evk, uint32_t galois_elt, uint64_t *acc,
                              int accumulate, size_t n, size_t size_ql, size_t size_q, size_t size_p,
                              const uint64_t *qp_full);
void or_mul_scalar_acc(const uint64_t *in, size_t in_stride, const uint64_t *c, const uint64_t *acc, uint64_t *out,
                       size_t polys, size_t n, size_t L, const uint64_t *moduli);
void or_tensor_lin(const uint64_t *ct1, const uint64_t *ct2, uint64_t *out, size_t n, size_t L,
                   const uint64_t *moduli, const uint64_t *f, const uint64_t *t, size_t t_stride, const uint64_t *c);
void or_lin_comb(uint64_t *d, size_t d_polys, const uint64_t *ca, const uint64_t *t, size_t t_polys,
                 size_t t_stride, const uint64_t *cb, size_t n, size_t L, const uint64_t *moduli);
void or_leaf_combine(const uint64_t *const *in, const size_t *in_stride, size_t K, const uint64_t *coef,
                     const uint64_t *cadd, uint64_t *const *out, size_t M, size_t n, size_t L, const uint64_t *moduli);

#ifdef __cplusplus
}
#endif
#endif
