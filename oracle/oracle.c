/*
 * oracle.c — CPU restatement of PhantomFHE's CKKS hot path.  TEST INFRASTRUCTURE ONLY:
 * loaded by tests/, bench.py's cpu_baseline leg and __graft_entry__.smoke() as the
 * checker; never linked into or called by the product library.
 *
 * All arithmetic is exact (unsigned __int128).  Where the reference uses lazy
 * reductions (Shoup butterflies with values in [0, 4q)) the restatement keeps the same
 * lazy form and the same final reduction, so intermediate bounds are checked too.
 * Reference paths are relative to the PhantomFHE repository root.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------ */
/* scalar number theory                                                 */
/* ------------------------------------------------------------------ */

uint64_t or_mulmod(uint64_t a, uint64_t b, uint64_t q) { return (uint64_t)(((u128)a * b) % q); }

uint64_t or_powmod(uint64_t a, uint64_t e, uint64_t q) {
    uint64_t r = 1 % q;
    a %= q;
    while (e) {
        if (e & 1) r = or_mulmod(r, a, q);
        a = or_mulmod(a, a, q);
        e >>= 1;
    }
    return r;
}

/* try_invert_uint_mod (include/host/uintarithsmallmod.h): extended Euclid; 0 if not invertible */
uint64_t or_invmod(uint64_t a, uint64_t q) {
    __int128 t = 0, nt = 1, r = q, nr = a % q;
    while (nr) {
        __int128 quo = r / nr, tmp;
        tmp = t - quo * nt; t = nt; nt = tmp;
        tmp = r - quo * nr; r = nr; nr = tmp;
    }
    if (r != 1) return 0;
    if (t < 0) t += q;
    return (uint64_t)t;
}

/* is_prime (src/host/numth.cu:160-204): Miller-Rabin.  The reference draws random bases
 * (std::random_device); a deterministic base set that is exact for all 64-bit inputs
 * gives the same verdict on every prime the reference accepts. */
int or_is_prime(uint64_t v) {
    static const uint64_t small[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    if (v < 2) return 0;
    for (size_t i = 0; i < sizeof(small) / sizeof(small[0]); i++) {
        if (v == small[i]) return 1;
        if (v % small[i] == 0) return 0;
    }
    uint64_t d = v - 1;
    int r = 0;
    while ((d & 1) == 0) { d >>= 1; r++; }
    static const uint64_t bases[] = {2, 325, 9375, 28178, 450775, 9780504, 1795265022};
    for (size_t i = 0; i < 7; i++) {
        uint64_t a = bases[i] % v;
        if (a == 0) continue;
        uint64_t x = or_powmod(a, d, v);
        if (x == 1 || x == v - 1) continue;
        int ok = 0;
        for (int k = 1; k < r; k++) {
            x = or_mulmod(x, x, v);
            if (x == v - 1) { ok = 1; break; }
        }
        if (!ok) return 0;
    }
    return 1;
}

/* compute_shoup (include/host/uintarithsmallmod.h:119-124): floor(w * 2^64 / q) */
uint64_t or_shoup(uint64_t w, uint64_t q) { return (uint64_t)(((u128)w << 64) / q); }

/* Modulus::set_value (src/host/modulus.cu:15-48): const_ratio = floor(2^128 / q) as {lo, hi} */
void or_barrett_ratio(uint64_t q, uint64_t out[2]) {
    /* 2^128 / q computed as ((2^128 - 1) / q) corrected; q is never a power of two here */
    u128 all = ~(u128)0;
    u128 quo = all / q;
    u128 rem = all - quo * q;
    if (rem + 1 == q) quo += 1;
    out[0] = (uint64_t)quo;
    out[1] = (uint64_t)(quo >> 64);
}

/* get_primes (src/host/numth.cu:207-233): descend from 2^bits - 2n + 1 in steps of 2n */
int or_get_primes(size_t n, int bit_size, size_t count, uint64_t *out) {
    uint64_t factor = 2 * (uint64_t)n;
    uint64_t value = ((uint64_t)1 << bit_size) - factor + 1;
    uint64_t lower = (uint64_t)1 << (bit_size - 1);
    size_t found = 0;
    while (found < count && value > lower) {
        if (or_is_prime(value)) out[found++] = value;
        value -= factor;
    }
    return found == count ? 0 : -1;
}

/* CoeffModulus::Create (src/host/modulus.cu:80-111): per bit size, primes are found
 * largest-first and handed out from the back, so the first request of a size receives
 * the smallest prime found for that size. */
int or_coeff_modulus_create(size_t n, const int *bit_sizes, size_t count, uint64_t *out) {
    for (size_t i = 0; i < count; i++) {
        int b = bit_sizes[i];
        int seen = 0;
        for (size_t j = 0; j < i; j++) if (bit_sizes[j] == b) { seen = 1; break; }
        if (seen) continue;
        size_t cnt = 0;
        for (size_t j = 0; j < count; j++) if (bit_sizes[j] == b) cnt++;
        uint64_t *primes = (uint64_t *)malloc(cnt * sizeof(uint64_t));
        if (or_get_primes(n, b, cnt, primes) != 0) { free(primes); return -1; }
        size_t back = cnt;
        for (size_t j = 0; j < count; j++)
            if (bit_sizes[j] == b) out[j] = primes[--back];
        free(primes);
    }
    return 0;
}

/* try_minimal_primitive_root (src/host/numth.cu:309-332): the smallest primitive
 * degree-th root of unity mod q (unique, independent of the random starting root). */
uint64_t or_minimal_primitive_root(uint64_t degree, uint64_t q) {
    if ((q - 1) % degree) return 0;
    uint64_t quot = (q - 1) / degree;
    uint64_t root = 0;
    for (uint64_t g = 2; g < q; g++) {
        uint64_t c = or_powmod(g, quot, q);
        if (or_powmod(c, degree >> 1, q) == q - 1) { root = c; break; }
    }
    if (!root) return 0;
    uint64_t gen_sq = or_mulmod(root, root, q), cur = root, best = root;
    for (uint64_t i = 0; i < degree; i++) {
        if (cur < best) best = cur;
        cur = or_mulmod(cur, gen_sq, q);
    }
    return best;
}

static size_t rev_bits(size_t x, int bits) {
    size_t r = 0;
    for (int i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}

static int log2_exact(size_t n) {
    int l = 0;
    while (((size_t)1 << l) < n) l++;
    return ((size_t)1 << l) == n ? l : -1;
}

/* NTT::NTT (src/host/ntt.cu:11-56): tw[brv(i)] = psi^i, itw[brv(i)] = psi^-i,
 * itw[1] pre-multiplied by n^-1. */
int or_ntt_tables(size_t n, uint64_t q, uint64_t *tw, uint64_t *tw_shoup, uint64_t *itw,
                  uint64_t *itw_shoup, uint64_t *n_inv, uint64_t *n_inv_shoup) {
    int logn = log2_exact(n);
    if (logn < 0) return -1;
    uint64_t psi = or_minimal_primitive_root(2 * (uint64_t)n, q);
    if (!psi) return -1;
    uint64_t ipsi = or_invmod(psi, q);
    uint64_t p = 1, ip = 1;
    for (size_t i = 0; i < n; i++) {
        size_t r = rev_bits(i, logn);
        tw[r] = p;
        itw[r] = ip;
        p = or_mulmod(p, psi, q);
        ip = or_mulmod(ip, ipsi, q);
    }
    uint64_t ninv = or_invmod((uint64_t)n % q, q);
    if (n > 1) itw[1] = or_mulmod(itw[1], ninv, q);
    for (size_t i = 0; i < n; i++) {
        tw_shoup[i] = or_shoup(tw[i], q);
        itw_shoup[i] = or_shoup(itw[i], q);
    }
    *n_inv = ninv;
    *n_inv_shoup = or_shoup(ninv, q);
    return 0;
}

/* ------------------------------------------------------------------ */
/* NTT                                                                  */
/* ------------------------------------------------------------------ */

static inline uint64_t mulhi64(uint64_t a, uint64_t b) { return (uint64_t)(((u128)a * b) >> 64); }
static inline uint64_t csub(uint64_t x, uint64_t m) { return x >= m ? x - m : x; }

typedef struct {
    size_t n;
    uint64_t q;
    uint64_t *tw, *tws, *itw, *itws, ninv, ninvs;
} tables_t;

static int tables_make(tables_t *t, size_t n, uint64_t q) {
    t->n = n; t->q = q;
    t->tw = malloc(n * 8); t->tws = malloc(n * 8); t->itw = malloc(n * 8); t->itws = malloc(n * 8);
    return or_ntt_tables(n, q, t->tw, t->tws, t->itw, t->itws, &t->ninv, &t->ninvs);
}

static void tables_free(tables_t *t) { free(t->tw); free(t->tws); free(t->itw); free(t->itws); }

/* Forward negacyclic NTT, radix-2 Cooley-Tukey with the lazy Shoup butterfly of
 * include/butterfly.cuh:10-22 (values kept in [0, 4q)), final reduction to [0, q)
 * as src/ntt/ntt_1d.cu:57-61 / src/ntt/fntt_2d.cu:187-193.  Output is bit-reversed:
 * A[i] = a(psi^(2*brv(i)+1)). */
static void ntt_fwd_one(uint64_t *a, const tables_t *t) {
    const size_t n = t->n;
    const uint64_t q = t->q, q2 = 2 * q;
    for (size_t m = 1, len = n / 2; m < n; m <<= 1, len >>= 1) {
        for (size_t i = 0; i < m; i++) {
            const uint64_t w = t->tw[m + i], ws = t->tws[m + i];
            uint64_t *x = a + 2 * i * len;
            for (size_t j = 0; j < len; j++) {
                uint64_t u = csub(x[j], q2);                      /* [0, 2q) */
                uint64_t v = x[j + len] * w - mulhi64(x[j + len], ws) * q; /* [0, 2q) */
                x[j] = u + v;                                     /* [0, 4q) */
                x[j + len] = u + q2 - v;                          /* [0, 4q) */
            }
        }
    }
    for (size_t j = 0; j < n; j++) a[j] = csub(csub(a[j], q2), q);
}

/* Inverse: Gentleman-Sande with the lazy butterfly of include/butterfly.cuh:28-37,
 * stages in reverse order, n^-1 applied as in src/ntt/intt_2d.cu:195-205 (the
 * x output of the last stage times n^-1, the y output through the folded itw[1]). */
static void ntt_inv_one(uint64_t *a, const tables_t *t) {
    const size_t n = t->n;
    const uint64_t q = t->q, q2 = 2 * q;
    for (size_t m = n / 2, len = 1; m >= 1; m >>= 1, len <<= 1) {
        for (size_t i = 0; i < m; i++) {
            const uint64_t w = t->itw[m + i], ws = t->itws[m + i];
            uint64_t *x = a + 2 * i * len;
            for (size_t j = 0; j < len; j++) {
                uint64_t u = x[j], v = x[j + len];
                uint64_t s = csub(u + v, q2);                     /* [0, 2q) */
                uint64_t d = u + q2 - v;                          /* [0, 4q) */
                if (m == 1) {
                    /* final stage: x * n^-1, y * (psi^-1 * n^-1) */
                    s = s * t->ninv - mulhi64(s, t->ninvs) * q;
                }
                x[j] = s;
                x[j + len] = d * w - mulhi64(d, ws) * q;        /* [0, 2q) */
            }
        }
        if (m == 1) break;
    }
    for (size_t j = 0; j < n; j++) a[j] = csub(csub(a[j], q2), q);
}

void or_ntt_fwd(uint64_t *data, size_t n, size_t L, const uint64_t *moduli) {
#pragma omp parallel for schedule(dynamic)
    for (size_t l = 0; l < L; l++) {
        tables_t t;
        tables_make(&t, n, moduli[l]);
        ntt_fwd_one(data + l * n, &t);
        tables_free(&t);
    }
}

void or_ntt_inv(uint64_t *data, size_t n, size_t L, const uint64_t *moduli) {
#pragma omp parallel for schedule(dynamic)
    for (size_t l = 0; l < L; l++) {
        tables_t t;
        tables_make(&t, n, moduli[l]);
        ntt_inv_one(data + l * n, &t);
        tables_free(&t);
    }
}

struct or_ntt_plan {
    size_t n, L;
    tables_t *t;
};

or_ntt_plan *or_ntt_plan_create(size_t n, size_t L, const uint64_t *moduli) {
    or_ntt_plan *p = malloc(sizeof(or_ntt_plan));
    p->n = n; p->L = L;
    p->t = malloc(L * sizeof(tables_t));
    for (size_t l = 0; l < L; l++) tables_make(&p->t[l], n, moduli[l]);
    return p;
}

void or_ntt_plan_destroy(or_ntt_plan *p) {
    for (size_t l = 0; l < p->L; l++) tables_free(&p->t[l]);
    free(p->t);
    free(p);
}

void or_ntt_plan_fwd(const or_ntt_plan *p, uint64_t *data, size_t L, int threads) {
#pragma omp parallel for num_threads(threads) schedule(static)
    for (size_t l = 0; l < L; l++) ntt_fwd_one(data + l * p->n, &p->t[l]);
}

void or_ntt_plan_inv(const or_ntt_plan *p, uint64_t *data, size_t L, int threads) {
#pragma omp parallel for num_threads(threads) schedule(static)
    for (size_t l = 0; l < L; l++) ntt_inv_one(data + l * p->n, &p->t[l]);
}

/* Known-answer definition of the negacyclic NTT (O(n^2)): A[i] = sum_j a_j psi^((2 brv(i) + 1) j). */
void or_ntt_fwd_naive(const uint64_t *in, uint64_t *out, size_t n, uint64_t q) {
    int logn = log2_exact(n);
    uint64_t psi = or_minimal_primitive_root(2 * (uint64_t)n, q);
    for (size_t i = 0; i < n; i++) {
        uint64_t root = or_powmod(psi, 2 * rev_bits(i, logn) + 1, q);
        uint64_t acc = 0, p = 1;
        for (size_t j = 0; j < n; j++) {
            acc = (uint64_t)(((u128)acc + (u128)in[j] * p) % q);
            p = or_mulmod(p, root, q);
        }
        out[i] = acc;
    }
}

/* ------------------------------------------------------------------ */
/* elementwise (src/polymath.cu)                                        */
/* ------------------------------------------------------------------ */

/* add_rns_poly (src/polymath.cu:41) */
void or_poly_add(const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n, size_t L, const uint64_t *moduli) {
    for (size_t l = 0; l < L; l++)
        for (size_t k = 0; k < n; k++) out[l * n + k] = csub(a[l * n + k] + b[l * n + k], moduli[l]);
}

/* sub_rns_poly (src/polymath.cu:127) */
void or_poly_sub(const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n, size_t L, const uint64_t *moduli) {
    for (size_t l = 0; l < L; l++)
        for (size_t k = 0; k < n; k++) out[l * n + k] = csub(a[l * n + k] + moduli[l] - b[l * n + k], moduli[l]);
}

/* negate_rns_poly (src/polymath.cu), negate_uint64_mod (include/uintmodmath.cuh:134-138) */
void or_poly_negate(const uint64_t *a, uint64_t *out, size_t n, size_t L, const uint64_t *moduli) {
    for (size_t l = 0; l < L; l++)
        for (size_t k = 0; k < n; k++) out[l * n + k] = a[l * n + k] ? moduli[l] - a[l * n + k] : 0;
}

/* multiply_rns_poly (src/polymath.cu:192-209): Barrett product, fully reduced */
void or_poly_mul(const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n, size_t L, const uint64_t *moduli) {
    for (size_t l = 0; l < L; l++)
        for (size_t k = 0; k < n; k++) out[l * n + k] = or_mulmod(a[l * n + k], b[l * n + k], moduli[l]);
}

/* multiply_scalar_rns_poly (src/polymath.cu:220-261): one scalar per limb */
void or_poly_mul_scalar(const uint64_t *a, const uint64_t *scalars, uint64_t *out, size_t n, size_t L,
                        const uint64_t *moduli) {
    for (size_t l = 0; l < L; l++)
        for (size_t k = 0; k < n; k++) out[l * n + k] = or_mulmod(a[l * n + k], scalars[l], moduli[l]);
}

/* tensor_prod_2x2_rns_poly (src/polymath.cu:501-536): d0 = c0 c0', d1 = c0 c1' + c1 c0',
 * d2 = c1 c1' (the reference computes d1 by Karatsuba; the value is the same). */
void or_tensor_prod_2x2(const uint64_t *ct1, const uint64_t *ct2, uint64_t *out, size_t n, size_t L,
                        const uint64_t *moduli) {
    const size_t s = n * L;
    for (size_t l = 0; l < L; l++) {
        uint64_t q = moduli[l];
        for (size_t k = 0; k < n; k++) {
            size_t i = l * n + k;
            uint64_t a0 = ct1[i], a1 = ct1[s + i], b0 = ct2[i], b1 = ct2[s + i];
            out[i] = or_mulmod(a0, b0, q);
            out[s + i] = (uint64_t)(((u128)a0 * b1 + (u128)a1 * b0) % q);
            out[2 * s + i] = or_mulmod(a1, b1, q);
        }
    }
}

/* tensor_square_2x2_rns_poly (src/polymath.cu:538-582): d0 = c0^2, d1 = (c0 c1 << 1) reduced as
 * one 128-bit value (:559-562; 2 c0 c1 < 2^123 for q < 2^61), d2 = c1^2.  out may alias ct. */
void or_tensor_square_2x2(const uint64_t *ct, uint64_t *out, size_t n, size_t L, const uint64_t *moduli) {
    const size_t s = n * L;
    for (size_t l = 0; l < L; l++) {
        uint64_t q = moduli[l];
        for (size_t k = 0; k < n; k++) {
            size_t i = l * n + k;
            uint64_t c0 = ct[i], c1 = ct[s + i];
            out[i] = or_mulmod(c0, c0, q);
            out[s + i] = (uint64_t)((((u128)c0 * c1) << 1) % q);
            out[2 * s + i] = or_mulmod(c1, c1, q);
        }
    }
}

/* ------------------------------------------------------------------ */
/* seed expansion of symmetric ciphertexts (src/prng.cu)                 */
/* ------------------------------------------------------------------ */

static uint32_t or_rotl32(uint32_t u, int c) { return (u << c) | (u >> (32 - c)); }

/* the Salsa20 core (20 rounds + feed-forward), as the loop of salsa20_gpu (src/prng.cu:48-99) */
void or_salsa20_core(const uint32_t in[16], uint32_t out[16]) {
    uint32_t x[16];
    for (int i = 0; i < 16; i++) x[i] = in[i];
    for (int r = 0; r < 10; r++) {
        /* columns */
        x[4] ^= or_rotl32(x[0] + x[12], 7);  x[8] ^= or_rotl32(x[4] + x[0], 9);
        x[12] ^= or_rotl32(x[8] + x[4], 13); x[0] ^= or_rotl32(x[12] + x[8], 18);
        x[9] ^= or_rotl32(x[5] + x[1], 7);   x[13] ^= or_rotl32(x[9] + x[5], 9);
        x[1] ^= or_rotl32(x[13] + x[9], 13); x[5] ^= or_rotl32(x[1] + x[13], 18);
        x[14] ^= or_rotl32(x[10] + x[6], 7); x[2] ^= or_rotl32(x[14] + x[10], 9);
        x[6] ^= or_rotl32(x[2] + x[14], 13); x[10] ^= or_rotl32(x[6] + x[2], 18);
        x[3] ^= or_rotl32(x[15] + x[11], 7); x[7] ^= or_rotl32(x[3] + x[15], 9);
        x[11] ^= or_rotl32(x[7] + x[3], 13); x[15] ^= or_rotl32(x[11] + x[7], 18);
        /* rows */
        x[1] ^= or_rotl32(x[0] + x[3], 7);   x[2] ^= or_rotl32(x[1] + x[0], 9);
        x[3] ^= or_rotl32(x[2] + x[1], 13);  x[0] ^= or_rotl32(x[3] + x[2], 18);
        x[6] ^= or_rotl32(x[5] + x[4], 7);   x[7] ^= or_rotl32(x[6] + x[5], 9);
        x[4] ^= or_rotl32(x[7] + x[6], 13);  x[5] ^= or_rotl32(x[4] + x[7], 18);
        x[11] ^= or_rotl32(x[10] + x[9], 7); x[8] ^= or_rotl32(x[11] + x[10], 9);
        x[9] ^= or_rotl32(x[8] + x[11], 13); x[10] ^= or_rotl32(x[9] + x[8], 18);
        x[12] ^= or_rotl32(x[15] + x[14], 7); x[13] ^= or_rotl32(x[12] + x[15], 9);
        x[14] ^= or_rotl32(x[13] + x[12], 13); x[15] ^= or_rotl32(x[14] + x[13], 18);
    }
    for (int i = 0; i < 16; i++) out[i] = x[i] + in[i];
}

static uint32_t or_le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* one 64-byte block of salsa20_gpu(out, 64, nonce, seed, 64) (src/prng.cu:17-47): the state holds
 * seed bytes 0..31 in words 0..7, the nonce in words 8..9 and seed bytes 32..55 in words 10..15
 * (bytes 56..63 of the 64-byte seed are unused; no constants, no block counter) */
void or_salsa20_block(const uint8_t seed[64], uint64_t nonce, uint32_t out[16]) {
    uint32_t in[16];
    for (int i = 0; i < 8; i++) in[i] = or_le32(seed + 4 * i);
    in[8] = (uint32_t)nonce;
    in[9] = (uint32_t)(nonce >> 32);
    for (int i = 0; i < 6; i++) in[10 + i] = or_le32(seed + 32 + 4 * i);
    or_salsa20_core(in, out);
}

/* sample_uniform_poly (src/prng.cu:164-197): thread tid < (n / 8) L fills out[8 tid .. 8 tid + 8)
 * of limb tid / (n / 8) with the block of nonce tid read as 8 little-endian 64-bit words, each
 * reduced mod q; a word above max_multiple = 2^64 - 1 - ((2^64 - 1) mod q) - 1 is rejected by
 * replacing the WHOLE block with the one of nonce tid + tries n L (tries = 1, 2, ..) and
 * continuing at the same word index */
void or_sample_uniform_seeded(const uint8_t seed[64], const uint64_t *moduli, size_t n, size_t L, uint64_t *out) {
    const size_t per = n >> 3;
    for (size_t tid = 0; tid < per * L; tid++) {
        const uint64_t q = moduli[tid / per];
        const uint64_t maxr = ~(uint64_t)0;
        const uint64_t max_multiple = maxr - maxr % q - 1;
        uint32_t blk[16];
        uint64_t tries = 0;
        or_salsa20_block(seed, tid, blk);
        tries++;
        for (int index = 0; index < 8; index++) {
            uint64_t r = (uint64_t)blk[2 * index] | ((uint64_t)blk[2 * index + 1] << 32);
            while (r > max_multiple) {
                or_salsa20_block(seed, tid + tries * n * L, blk);
                tries++;
                r = (uint64_t)blk[2 * index] | ((uint64_t)blk[2 * index + 1] << 32);
            }
            out[tid * 8 + index] = r % q;
        }
    }
}

/* ------------------------------------------------------------------ */
/* base conversion                                                      */
/* ------------------------------------------------------------------ */

/* DBaseConverter::bConv_BEHZ (src/rns_bconv.cu:212-229) with constants from the host
 * BaseConverter (include/host/rns.h:135-199): y_j = sum_i [x_i * qHat_i^-1]_{q_i} * (qHat_i mod p_j) mod p_j. */
void or_bconv(const uint64_t *in, uint64_t *out, size_t n, const uint64_t *ibase, size_t ibase_size,
              const uint64_t *obase, size_t obase_size) {
    uint64_t *qhat_inv = malloc(ibase_size * 8);
    uint64_t *qhat_mod_p = malloc(ibase_size * obase_size * 8);
    for (size_t i = 0; i < ibase_size; i++) {
        uint64_t prod = 1 % ibase[i];
        for (size_t k = 0; k < ibase_size; k++)
            if (k != i) prod = or_mulmod(prod, ibase[k] % ibase[i], ibase[i]);
        qhat_inv[i] = or_invmod(prod, ibase[i]);
        for (size_t j = 0; j < obase_size; j++) {
            uint64_t pr = 1 % obase[j];
            for (size_t k = 0; k < ibase_size; k++)
                if (k != i) pr = or_mulmod(pr, ibase[k] % obase[j], obase[j]);
            qhat_mod_p[i * obase_size + j] = pr;
        }
    }
#pragma omp parallel for schedule(static)
    for (size_t k = 0; k < n; k++) {
        for (size_t j = 0; j < obase_size; j++) {
            u128 acc = 0;
            for (size_t i = 0; i < ibase_size; i++) {
                uint64_t t = or_mulmod(in[i * n + k], qhat_inv[i], ibase[i]);
                acc += (u128)t * qhat_mod_p[i * obase_size + j];
            }
            out[j * n + k] = (uint64_t)(acc % obase[j]);
        }
    }
    free(qhat_inv);
    free(qhat_mod_p);
}

/* ------------------------------------------------------------------ */
/* hybrid key switching                                                 */
/* ------------------------------------------------------------------ */

static void concat_qlp(const uint64_t *ql, size_t size_ql, const uint64_t *p, size_t size_p, uint64_t *qlp) {
    memcpy(qlp, ql, size_ql * 8);
    memcpy(qlp + size_ql, p, size_p * 8);
}

/* DRNSTool::modup (src/rns_bconv.cu:530-628) for CKKS with alpha = size_P > 1:
 * per digit beta (alpha limbs of Ql, the last digit possibly shorter):
 *   own limbs     <- the NTT-form input (modup_copy_partQl_kernel, :522-528)
 *   other limbs   <- NTT( bconv_{digit -> QlP \ digit}( INTT(c2)|digit ) )
 * output layout [beta][size_QlP][n]. */
void or_modup(const uint64_t *c2_ntt, uint64_t *t_mod_up, size_t n, const uint64_t *ql, size_t size_ql,
              const uint64_t *p, size_t size_p) {
    const size_t alpha = size_p;
    const size_t beta = (size_ql + alpha - 1) / alpha;
    const size_t size_qlp = size_ql + size_p;
    uint64_t *qlp = malloc(size_qlp * 8);
    concat_qlp(ql, size_ql, p, size_p, qlp);
    uint64_t *coeff = malloc(size_ql * n * 8);
    memcpy(coeff, c2_ntt, size_ql * n * 8);
    or_ntt_inv(coeff, n, size_ql, ql);
    for (size_t b = 0; b < beta; b++) {
        size_t start = alpha * b;
        size_t part = (b == beta - 1) ? size_ql - alpha * (beta - 1) : alpha;
        uint64_t *dst = t_mod_up + b * size_qlp * n;
        size_t ocount = size_qlp - part;
        uint64_t *obase = malloc(ocount * 8);
        size_t o = 0;
        for (size_t j = 0; j < size_qlp; j++)
            if (j < start || j >= start + part) obase[o++] = qlp[j];
        uint64_t *conv = malloc(ocount * n * 8);
        or_bconv(coeff + start * n, conv, n, ql + start, part, obase, ocount);
        o = 0;
        for (size_t j = 0; j < size_qlp; j++) {
            if (j >= start && j < start + part) {
                memcpy(dst + j * n, c2_ntt + j * n, n * 8);
            } else {
                memcpy(dst + j * n, conv + o * n, n * 8);
                or_ntt_fwd(dst + j * n, n, 1, &qlp[j]);
                o++;
            }
        }
        free(conv);
        free(obase);
    }
    free(coeff);
    free(qlp);
}

/* key_switch_inner_prod_c2_and_evk (src/eval_key_switch.cu:26-85):
 * cx[t][nid] = sum_{i<beta} t_mod_up[i][nid] * evk[i][t][twr(nid)] mod q_twr(nid), where
 * twr(nid) = nid for nid < size_Ql and size_Q + (nid - size_Ql) for the special limbs.
 * evk[i] points at a [2][size_QP][n] key digit. */
void or_keyswitch_inner_prod(const uint64_t *t_mod_up, const uint64_t *const *evk, uint64_t *cx, size_t n,
                             size_t size_ql, size_t size_q, size_t size_p, size_t beta, const uint64_t *qp_full) {
    const size_t size_qlp = size_ql + size_p;
    const size_t size_qp = size_q + size_p;
#pragma omp parallel for schedule(static)
    for (size_t nid = 0; nid < size_qlp; nid++) {
        size_t twr = nid >= size_ql ? size_q + (nid - size_ql) : nid;
        uint64_t q = qp_full[twr];
        for (size_t k = 0; k < n; k++) {
            u128 acc0 = 0, acc1 = 0;
            for (size_t i = 0; i < beta; i++) {
                uint64_t c = t_mod_up[(i * size_qlp + nid) * n + k];
                acc0 += (u128)c * evk[i][twr * n + k];
                acc1 += (u128)c * evk[i][(size_qp + twr) * n + k];
            }
            cx[nid * n + k] = (uint64_t)(acc0 % q);
            cx[(size_qlp + nid) * n + k] = (uint64_t)(acc1 % q);
        }
    }
}

/* DRNSTool::moddown_from_NTT (src/rns_bconv.cu:791-843), CKKS branch:
 * INTT of the P limbs, delta = bconv_{P -> Ql}, then (fused NTT, src/ntt/ntt_moddown.cu:199-214)
 * out_j = (cx_j - NTT(delta)_j) * P^-1 mod q_j.  cx_i is [size_QlP][n] in NTT form and is
 * clobbered (its P limbs end in coefficient form, as in the reference). */
void or_moddown_from_ntt(uint64_t *cx_i, uint64_t *ct_out, size_t n, const uint64_t *ql, size_t size_ql,
                         const uint64_t *p, size_t size_p) {
    uint64_t *pl = cx_i + size_ql * n;
    or_ntt_inv(pl, n, size_p, p);
    uint64_t *delta = malloc(size_ql * n * 8);
    or_bconv(pl, delta, n, p, size_p, ql, size_ql);
    or_ntt_fwd(delta, n, size_ql, ql);
    for (size_t j = 0; j < size_ql; j++) {
        uint64_t q = ql[j];
        uint64_t pmod = 1;
        for (size_t i = 0; i < size_p; i++) pmod = or_mulmod(pmod, p[i] % q, q);
        uint64_t pinv = or_invmod(pmod, q);
        for (size_t k = 0; k < n; k++) {
            uint64_t d = csub(cx_i[j * n + k] + q - delta[j * n + k], q);
            ct_out[j * n + k] = or_mulmod(d, pinv, q);
        }
    }
    free(delta);
}

/* keyswitch_inplace (src/eval_key_switch.cu:112-212), CKKS: modup -> inner product ->
 * moddown x2 -> add_to_ct_kernel (src/rns_bconv.cu:763-789).  ct is [2][size_Ql][n];
 * qp_full is the full key-level chain (size_Q data primes then size_P special primes). */
void or_keyswitch_add(uint64_t *ct, const uint64_t *c2, const uint64_t *const *evk, size_t n, size_t size_ql,
                      size_t size_q, size_t size_p, const uint64_t *qp_full) {
    const size_t size_qlp = size_ql + size_p;
    const size_t beta = (size_ql + size_p - 1) / size_p;
    const uint64_t *p = qp_full + size_q;
    uint64_t *tmu = malloc(beta * size_qlp * n * 8);
    or_modup(c2, tmu, n, qp_full, size_ql, p, size_p);
    uint64_t *cx = malloc(2 * size_qlp * n * 8);
    or_keyswitch_inner_prod(tmu, evk, cx, n, size_ql, size_q, size_p, beta, qp_full);
    uint64_t *down = malloc(size_ql * n * 8);
    for (size_t t = 0; t < 2; t++) {
        or_moddown_from_ntt(cx + t * size_qlp * n, down, n, qp_full, size_ql, p, size_p);
        or_poly_add(ct + t * size_ql * n, down, ct + t * size_ql * n, n, size_ql, qp_full);
    }
    free(down);
    free(cx);
    free(tmu);
}

/* relinearize_inplace (src/evaluate.cu:1552-1589): key-switch c2 into (c0, c1).
 * ct3 is [3][size_Ql][n]; on return its first two polys hold the result. */
void or_relinearize(uint64_t *ct3, size_t n, size_t size_ql, size_t size_q, size_t size_p,
                    const uint64_t *const *evk, const uint64_t *qp_full) {
    or_keyswitch_add(ct3, ct3 + 2 * size_ql * n, evk, n, size_ql, size_q, size_p, qp_full);
}

/* ------------------------------------------------------------------ */
/* rescale                                                              */
/* ------------------------------------------------------------------ */

/* DRNSTool::divide_and_round_q_last_ntt (src/rns.cu:1160-1184) with kernels :1128-1158:
 * c_L <- INTT(last limb); t_j = NTT_j(c_L mod q_j); out_j = (c_j - t_j) * q_L^-1 mod q_j.
 * ct is [polys][size_Ql][n]; out is [polys][size_Ql - 1][n]. */
void or_rescale_ntt(const uint64_t *ct, uint64_t *out, size_t n, size_t size_ql, size_t polys,
                    const uint64_t *ql) {
    const size_t nl = size_ql - 1;
    const uint64_t qlast = ql[nl];
    uint64_t *last = malloc(n * 8);
    uint64_t *t = malloc(nl * n * 8);
    for (size_t c = 0; c < polys; c++) {
        const uint64_t *ci = ct + c * size_ql * n;
        uint64_t *co = out + c * nl * n;
        memcpy(last, ci + nl * n, n * 8);
        or_ntt_inv(last, n, 1, &qlast);
        for (size_t j = 0; j < nl; j++)
            for (size_t k = 0; k < n; k++) t[j * n + k] = last[k] % ql[j];
        or_ntt_fwd(t, n, nl, ql);
        for (size_t j = 0; j < nl; j++) {
            uint64_t inv = or_invmod(qlast % ql[j], ql[j]);
            for (size_t k = 0; k < n; k++) {
                uint64_t d = csub(ci[j * n + k] + ql[j] - t[j * n + k], ql[j]);
                co[j * n + k] = or_mulmod(d, inv, ql[j]);
            }
        }
    }
    free(t);
    free(last);
}

/* mod_switch_drop_to_next (src/evaluate.cu:1650-1690), CKKS in NTT form: drop the last limb. */
void or_mod_switch_drop_ntt(const uint64_t *ct, uint64_t *out, size_t n, size_t size_ql, size_t polys) {
    for (size_t c = 0; c < polys; c++)
        memcpy(out + c * (size_ql - 1) * n, ct + c * size_ql * n, (size_ql - 1) * n * 8);
}

/* ------------------------------------------------------------------ */
/* automorphism                                                         */
/* ------------------------------------------------------------------ */

/* PrecomputeAutoMapKernel (src/util.cu:941-958): perm[brv(j)] = brv(((2j+1) k mod 2n - 1) / 2) */
void or_galois_perm_ntt(uint32_t galois_elt, size_t n, uint32_t *perm) {
    int logn = log2_exact(n);
    const uint64_t m = 2 * (uint64_t)n;
    for (size_t j = 0; j < n; j++) {
        uint64_t idx = ((2 * (uint64_t)j + 1) * galois_elt) % m;
        perm[rev_bits(j, logn)] = (uint32_t)rev_bits((size_t)((idx - 1) >> 1), logn);
    }
}

/* apply_galois_ntt_permutation_direct (src/galois.cu:104-119): dst[j] = src[perm[j]] per limb */
void or_apply_galois_ntt(const uint64_t *in, uint64_t *out, size_t n, size_t L, uint32_t galois_elt) {
    uint32_t *perm = malloc(n * sizeof(uint32_t));
    or_galois_perm_ntt(galois_elt, n, perm);
    for (size_t l = 0; l < L; l++)
        for (size_t j = 0; j < n; j++) out[l * n + j] = in[l * n + perm[j]];
    free(perm);
}

/* ------------------------------------------------------------------ */
/* bootstrap helpers                                                    */
/* ------------------------------------------------------------------ */

/* switchModulusKernel (src/evaluate.cu:2414-2457), used by RaiseMod: lift the q0
 * residue (coefficient form) to every limb with a centered representative. */
void or_switch_modulus_raise(const uint64_t *in_q0, uint64_t *out, size_t n, uint64_t q0, const uint64_t *ql,
                             size_t size_ql) {
    const uint64_t half = q0 >> 1;
    for (size_t j = 0; j < size_ql; j++) {
        uint64_t qj = ql[j];
        for (size_t k = 0; k < n; k++) {
            uint64_t v = in_q0[k];
            uint64_t r;
            if (v > half) {
                /* negative representative v - q0 */
                uint64_t neg = (q0 - v) % qj;
                r = neg ? qj - neg : 0;
            } else {
                r = v % qj;
            }
            out[j * n + k] = r;
        }
    }
}

/* MultByMonomialInPlace (src/evaluate.cu:2521-2554): NTT form of X^power (power < 2n,
 * X^n = -1), one limb per modulus. */
void or_monomial_ntt(uint64_t *out, size_t n, size_t L, const uint64_t *moduli, uint32_t power) {
    for (size_t l = 0; l < L; l++) {
        uint64_t *o = out + l * n;
        memset(o, 0, n * 8);
        uint32_t pw = power % (2 * (uint32_t)n);
        if (pw < n) o[pw] = 1;
        else o[pw - n] = moduli[l] - 1;
        or_ntt_fwd(o, n, 1, &moduli[l]);
    }
}

/* ------------------------------------------------------------------ */
/* bootstrap kernels (hoisted linear transforms, EvalMod)              */
/* ------------------------------------------------------------------ */

/* modulus of buffer limb l of an extended-basis (Ql u P) polynomial */
static uint64_t ext_mod(size_t l, size_t size_ql, size_t size_q, const uint64_t *qp_full) {
    return l < size_ql ? qp_full[l] : qp_full[size_q + (l - size_ql)];
}

/* The hoisted baby-step / giant-step inner sums of EvalLinearTransform (src/bootstrap.cu:1322-1332):
 * for every giant step i < b, out[i] = sum_{j<g} EvalMultExt(baby[j], pt[i g + j]) accumulated with
 * EvalAddExtInPlace (src/evaluate.cu:3786-3874): both polynomials of a [2][Ql+P][n] extended-basis
 * ciphertext times a [Ql+P][n] plaintext, limb by limb, mod the limb's prime. */
void or_lt_bsgs(const uint64_t *const *baby, size_t g, const uint64_t *const *pts, size_t b, uint64_t *const *out,
                size_t n, size_t size_ql, size_t size_q, size_t size_p, const uint64_t *qp_full) {
    const size_t qlp = size_ql + size_p;
#pragma omp parallel for schedule(static)
    for (size_t l = 0; l < qlp; l++) {
        const uint64_t q = ext_mod(l, size_ql, size_q, qp_full);
        for (size_t i = 0; i < b; i++)
            for (size_t t = 0; t < 2; t++)
                for (size_t k = 0; k < n; k++) {
                    uint64_t acc = 0;
                    for (size_t j = 0; j < g; j++) {
                        const uint64_t x = baby[j][(t * qlp + l) * n + k];
                        const uint64_t w = pts[i * g + j][l * n + k];
                        acc = csub(acc + or_mulmod(x, w, q), q);
                    }
                    out[i][(t * qlp + l) * n + k] = acc;
                }
    }
}

/* KeySwitchExt (src/evaluate.cu:3876-3940): (c0, c1) at Ql -> P (c0, c1) in the extended basis,
 * the P limbs zero.  ct [2][Ql][n] -> out [2][Ql+P][n]. */
void or_keyswitch_ext(const uint64_t *ct, uint64_t *out, size_t n, size_t size_ql, size_t size_q, size_t size_p,
                      const uint64_t *qp_full) {
    const size_t qlp = size_ql + size_p;
    memset(out, 0, 2 * qlp * n * 8);
    for (size_t t = 0; t < 2; t++)
        for (size_t l = 0; l < size_ql; l++) {
            const uint64_t q = qp_full[l];
            uint64_t pm = 1;
            for (size_t i = 0; i < size_p; i++) pm = or_mulmod(pm, qp_full[size_q + i] % q, q);
            for (size_t k = 0; k < n; k++) out[(t * qlp + l) * n + k] = or_mulmod(ct[(t * size_ql + l) * n + k], pm, q);
        }
}

/* EvalFastRotationExt (src/evaluate.cu:3660-3755) with a fused key: cx = the key-switch inner
 * product of the shared modup digits (or_keyswitch_inner_prod), then, if add_first, cx[0] += P c0
 * on the Ql limbs, then the NTT-domain automorphism of both polynomials
 * (apply_galois_ntt_permutation_direct, src/galois.cu:104-119).  c0: [Ql][n]; out [2][Ql+P][n]. */
void or_fast_rotation_ext(const uint64_t *c0, const uint64_t *digits, const uint64_t *const *evk, uint32_t galois_elt,
                          int add_first, uint64_t *out, size_t n, size_t size_ql, size_t size_q, size_t size_p,
                          const uint64_t *qp_full) {
    const size_t qlp = size_ql + size_p, beta = (size_ql + size_p - 1) / size_p;
    uint64_t *cx = malloc(2 * qlp * n * 8);
    or_keyswitch_inner_prod(digits, evk, cx, n, size_ql, size_q, size_p, beta, qp_full);
    if (add_first)
        for (size_t l = 0; l < size_ql; l++) {
            const uint64_t q = qp_full[l];
            uint64_t pm = 1;
            for (size_t i = 0; i < size_p; i++) pm = or_mulmod(pm, qp_full[size_q + i] % q, q);
            for (size_t k = 0; k < n; k++)
                cx[l * n + k] = csub(cx[l * n + k] + or_mulmod(c0[l * n + k], pm, q), q);
        }
    or_apply_galois_ntt(cx, out, n, 2 * qlp, galois_elt);
    free(cx);
}

/* A giant step of EvalLinearTransform in the extended basis (src/bootstrap.cu:1335-1348:
 * KeySwitchDown of the inner sum's c1, EvalFastRotationPrecompute of it, EvalFastRotationExt,
 * EvalAddExtInPlace into the accumulator), with c0 kept P-scaled in Ql u P:
 *   digits = modup(moddown(ext c1));  cx = inner product;  x = (cx0 + ext c0, cx1);
 *   acc (+)= automorphism(x).  ext [2][Ql+P][n] (c1's P limbs clobbered), acc [2][Ql+P][n]. */
void or_rotate_ext_accumulate(uint64_t *ext, const uint64_t *const *evk, uint32_t galois_elt, uint64_t *acc,
                              int accumulate, size_t n, size_t size_ql, size_t size_q, size_t size_p,
                              const uint64_t *qp_full) {
    const size_t qlp = size_ql + size_p, beta = (size_ql + size_p - 1) / size_p;
    const uint64_t *p = qp_full + size_q;
    uint64_t *c1 = malloc(size_ql * n * 8);
    or_moddown_from_ntt(ext + qlp * n, c1, n, qp_full, size_ql, p, size_p);
    uint64_t *digits = malloc(beta * qlp * n * 8);
    or_modup(c1, digits, n, qp_full, size_ql, p, size_p);
    uint64_t *cx = malloc(2 * qlp * n * 8);
    or_keyswitch_inner_prod(digits, evk, cx, n, size_ql, size_q, size_p, beta, qp_full);
    for (size_t l = 0; l < qlp; l++) {
        const uint64_t q = ext_mod(l, size_ql, size_q, qp_full);
        for (size_t k = 0; k < n; k++) cx[l * n + k] = csub(cx[l * n + k] + ext[l * n + k], q);
    }
    uint64_t *rot = malloc(2 * qlp * n * 8);
    or_apply_galois_ntt(cx, rot, n, 2 * qlp, galois_elt);
    for (size_t t = 0; t < 2; t++)
        for (size_t l = 0; l < qlp; l++) {
            const uint64_t q = ext_mod(l, size_ql, size_q, qp_full);
            for (size_t k = 0; k < n; k++) {
                const size_t e = (t * qlp + l) * n + k;
                acc[e] = accumulate ? csub(acc[e] + rot[e], q) : rot[e];
            }
        }
    free(rot);
    free(cx);
    free(digits);
    free(c1);
}

/* multiply every polynomial by per-limb integer constants, optionally accumulating:
 * out[p][l] = in[p][l] * c[l] (+ acc[p][l]) mod q_l — the residue form of EvalMultConstInplaceCore
 * / MultByIntegerInPlace (src/evaluate.cu:2299-2412, :3942-3970).  in[p] at in + p * in_stride. */
void or_mul_scalar_acc(const uint64_t *in, size_t in_stride, const uint64_t *c, const uint64_t *acc, uint64_t *out,
                       size_t polys, size_t n, size_t L, const uint64_t *moduli) {
    for (size_t p = 0; p < polys; p++)
        for (size_t l = 0; l < L; l++)
            for (size_t k = 0; k < n; k++) {
                const size_t e = l * n + k;
                uint64_t v = or_mulmod(in[p * in_stride + e], c[l], moduli[l]);
                if (acc) v = csub(v + acc[p * L * n + e], moduli[l]);
                out[p * L * n + e] = v;
            }
}

/* tensor product with a linear epilogue — EvalMult (tensor_prod_2x2_rns_poly, src/polymath.cu:501-536)
 * times the integer f (EvalMultConst), plus c * t added to the first two polynomials (EvalAdd of a
 * constant multiple): d = f (ct1 x ct2); d[p] += c t[p] for p < 2.  f / c: per-limb residues or NULL. */
void or_tensor_lin(const uint64_t *ct1, const uint64_t *ct2, uint64_t *out, size_t n, size_t L,
                   const uint64_t *moduli, const uint64_t *f, const uint64_t *t, size_t t_stride, const uint64_t *c) {
    or_tensor_prod_2x2(ct1, ct2, out, n, L, moduli);
    for (size_t p = 0; p < 3; p++)
        for (size_t l = 0; l < L; l++) {
            const uint64_t q = moduli[l];
            for (size_t k = 0; k < n; k++) {
                uint64_t *d = &out[(p * L + l) * n + k];
                if (f) *d = or_mulmod(*d, f[l], q);
                if (t && c && p < 2) *d = csub(*d + or_mulmod(t[p * t_stride + l * n + k], c[l], q), q);
            }
        }
}

/* d[p] = d[p] * ca (if ca) + (p < t_polys ? t[p] * cb : 0), t[p] at t + p * t_stride */
void or_lin_comb(uint64_t *d, size_t d_polys, const uint64_t *ca, const uint64_t *t, size_t t_polys,
                 size_t t_stride, const uint64_t *cb, size_t n, size_t L, const uint64_t *moduli) {
    for (size_t p = 0; p < d_polys; p++)
        for (size_t l = 0; l < L; l++) {
            const uint64_t q = moduli[l];
            for (size_t k = 0; k < n; k++) {
                uint64_t *x = &d[(p * L + l) * n + k];
                if (ca) *x = or_mulmod(*x, ca[l], q);
                if (t && p < t_polys) *x = csub(*x + or_mulmod(t[p * t_stride + l * n + k], cb[l], q), q);
            }
        }
}

/* The Chebyshev leaves of EvalChebyshevSeriesPS (src/evaluate.cu:3264-3535): each leaf is a
 * weighted sum of the power ciphertexts T_1..T_K plus a constant, EvalLinearWSumMutable
 * (:3537-3600) + EvalAddConst: out[m][t][l] = sum_k in[k][t][l] coef[m][k][l] + (t == 0 ? cadd[m][l] : 0).
 * in[k] is [2][>= L][n] with polynomial stride in_stride[k]; out[m] is [2][L][n];
 * coef [M][K][L], cadd [M][L] are residues. */
void or_leaf_combine(const uint64_t *const *in, const size_t *in_stride, size_t K, const uint64_t *coef,
                     const uint64_t *cadd, uint64_t *const *out, size_t M, size_t n, size_t L, const uint64_t *moduli) {
    for (size_t m = 0; m < M; m++)
        for (size_t t = 0; t < 2; t++)
            for (size_t l = 0; l < L; l++) {
                const uint64_t q = moduli[l];
                for (size_t k = 0; k < n; k++) {
                    u128 acc = 0;
                    for (size_t i = 0; i < K; i++)
                        acc += (u128)in[i][t * in_stride[i] + l * n + k] * coef[(m * K + i) * L + l];
                    uint64_t v = (uint64_t)(acc % q);
                    if (t == 0) v = csub(v + cadd[m * L + l], q);
                    out[m][(t * L + l) * n + k] = v;
                }
            }
}

