"""CPU oracle pinned against the reference's own fixtures/tests and mathematical KATs.

The reference ships no bit-level golden vectors for the hot path:
test/ntt_test.cu only checks INTT(NTT(x)) == x.  These tests pin the oracle by
  * the modulus values the reference's host code produced (tests/golden/moduli_c3.json),
  * the reference's round-trip test at its own sizes/moduli (test/ntt_test.cu:71-151),
  * the defining formulas: naive negacyclic DFT, CRT reconstruction for base conversion,
    exact big-integer formulas for moddown / rescale, coefficient-domain automorphisms,
  * an end-to-end relinearization decrypt check with real (seeded) keys.
"""
import json
import os

import numpy as np
import pytest

import oracle_lib as O
from oracle_lib import P, arr

HERE = os.path.dirname(os.path.abspath(__file__))


def crt(residues, moduli):
    Q = 1
    for q in moduli:
        Q *= q
    x = 0
    for r, q in zip(residues, moduli):
        qh = Q // q
        x += int(r) * qh * pow(qh, -1, q)
    return x % Q, Q


def brv(x, bits):
    return int(format(x, f"0{bits}b")[::-1], 2) if bits else 0


# --------------------------------------------------------------------------------------
# parameters
# --------------------------------------------------------------------------------------

def test_c3_moduli_match_reference_host_output():
    g = json.load(open(os.path.join(HERE, "golden", "moduli_c3.json")))
    mods = O.coeff_modulus_create(65536, [60] + [50] * 44 + [60] * 15)
    assert len(mods) == 60
    for k, v in g["known"].items():
        assert mods[int(k)] == v, (k, mods[int(k)], v)
    for q in mods:
        assert O.lib().or_is_prime(q) and (q - 1) % (2 * 65536) == 0
    assert len(set(mods)) == 60


def test_coeff_modulus_pop_back_order():
    # the first request of a bit size gets the smallest prime found (modulus.cu:96-110)
    m = O.coeff_modulus_create(4096, [50, 50, 50])
    assert m[0] < m[1] < m[2]
    assert m[2] == max(m)


def test_minimal_primitive_root():
    for n, bits in [(16, 30), (1024, 50), (4096, 60)]:
        q = O.coeff_modulus_create(n, [bits])[0]
        psi = O.lib().or_minimal_primitive_root(2 * n, q)
        assert pow(psi, n, q) == q - 1
        # no smaller primitive 2n-th root: all primitive roots are psi^(odd)
        roots = sorted(pow(psi, k, q) for k in range(1, 2 * n, 2))
        assert roots[0] == psi


def test_ntt_tables_layout():
    n = 256
    q = O.coeff_modulus_create(n, [50])[0]
    (tw, tws, itw, itws), ninv = O.ntt_tables(n, q)
    psi = O.lib().or_minimal_primitive_root(2 * n, q)
    for i in range(n):
        assert int(tw[brv(i, 8)]) == pow(psi, i, q)
        assert int(tws[i]) == (int(tw[i]) << 64) // q
    assert ninv * n % q == 1
    # itw[1] is pre-multiplied by n^-1 (src/host/ntt.cu:53-55)
    assert int(itw[1]) == pow(psi, -brv(1, 8), q) * ninv % q
    assert int(itw[3]) == pow(psi, -brv(3, 8), q)


# --------------------------------------------------------------------------------------
# NTT
# --------------------------------------------------------------------------------------

@pytest.mark.parametrize("n,bits", [(8, 20), (64, 40), (256, 50), (1024, 50), (1024, 60)])
def test_ntt_matches_naive_negacyclic_dft(rng, n, bits):
    q = O.coeff_modulus_create(n, [bits])[0]
    a = O.random_limbs(rng, n, [q])
    got = O.ntt_fwd(a, n, [q])
    want = np.zeros(n, dtype=np.uint64)
    O.lib().or_ntt_fwd_naive(P(a), P(want), n, q)
    assert np.array_equal(got, want)


def test_ntt_roundtrip_reference_test_config1():
    # test/ntt_test.cu:78-122 with N = 4096, CoeffModulus::Create(4096, {50}), constant-2 input
    n = 4096
    q = O.coeff_modulus_create(n, [50])
    a = np.full(n, 2, dtype=np.uint64)
    f = O.ntt_fwd(a, n, q)
    assert not np.array_equal(f, a)
    assert np.array_equal(O.ntt_inv(f, n, q), a)


@pytest.mark.parametrize("log_n", list(range(11, 18)))
@pytest.mark.parametrize("batch", [1, 10])
def test_ntt_roundtrip_reference_sweep(rng, log_n, batch):
    # test/ntt_test.cu:124-151: N = 2^11..2^17, batch 1 and 10, 50-bit primes
    n = 1 << log_n
    q = O.coeff_modulus_create(n, [50] * batch)
    a = O.random_limbs(rng, n, q)
    assert np.array_equal(O.ntt_inv(O.ntt_fwd(a, n, q), n, q), a)


def test_ntt_is_a_ring_homomorphism(rng):
    # NTT(a * b mod X^n + 1) == NTT(a) . NTT(b)
    n = 64
    q = O.coeff_modulus_create(n, [50])[0]
    a = [int(x) for x in rng.integers(0, q, n)]
    b = [int(x) for x in rng.integers(0, q, n)]
    c = [0] * n
    for i in range(n):
        for j in range(n):
            k = i + j
            if k < n:
                c[k] = (c[k] + a[i] * b[j]) % q
            else:
                c[k - n] = (c[k - n] - a[i] * b[j]) % q
    fa, fb, fc = (O.ntt_fwd(arr(v), n, [q]) for v in (a, b, c))
    assert [int(x) * int(y) % q for x, y in zip(fa, fb)] == [int(x) for x in fc]


# --------------------------------------------------------------------------------------
# elementwise
# --------------------------------------------------------------------------------------

def test_tensor_product_formula(rng):
    n = 32
    mods = O.coeff_modulus_create(n, [60, 50, 50])
    L = len(mods)
    c1 = np.concatenate([O.random_limbs(rng, n, mods) for _ in range(2)])
    c2 = np.concatenate([O.random_limbs(rng, n, mods) for _ in range(2)])
    out = np.zeros(3 * L * n, dtype=np.uint64)
    O.lib().or_tensor_prod_2x2(P(c1), P(c2), P(out), n, L, P(arr(mods)))
    s = L * n
    for l, q in enumerate(mods):
        for k in range(n):
            i = l * n + k
            a0, a1, b0, b1 = int(c1[i]), int(c1[s + i]), int(c2[i]), int(c2[s + i])
            assert int(out[i]) == a0 * b0 % q
            assert int(out[s + i]) == (a0 * b1 + a1 * b0) % q
            assert int(out[2 * s + i]) == a1 * b1 % q


def test_tensor_square_formula(rng):
    """or_tensor_square_2x2 (polymath.cu:538-582) = the product with itself, exact, incl. q - 1"""
    n = 32
    mods = O.coeff_modulus_create(n, [60, 59, 50])
    L = len(mods)
    c = np.concatenate([O.random_limbs(rng, n, mods) for _ in range(2)])
    c[:4] = mods[0] - 1
    c[L * n: L * n + 4] = mods[0] - 1
    out = np.zeros(3 * L * n, dtype=np.uint64)
    O.lib().or_tensor_square_2x2(P(c), P(out), n, L, P(arr(mods)))
    prod = np.zeros_like(out)
    O.lib().or_tensor_prod_2x2(P(c), P(c), P(prod), n, L, P(arr(mods)))
    assert np.array_equal(out, prod)
    s = L * n
    for l, q in enumerate(mods):
        for k in range(n):
            i = l * n + k
            a0, a1 = int(c[i]), int(c[s + i])
            assert int(out[s + i]) == 2 * a0 * a1 % q


# --------------------------------------------------------------------------------------
# base conversion, moddown, rescale
# --------------------------------------------------------------------------------------

def test_bconv_is_fast_crt_with_bounded_overflow(rng):
    n = 16
    ib = O.coeff_modulus_create(n, [50, 50, 50])
    ob = O.coeff_modulus_create(n, [60, 60])
    x = O.random_limbs(rng, n, ib)
    y = np.zeros(len(ob) * n, dtype=np.uint64)
    O.lib().or_bconv(P(x), P(y), n, P(arr(ib)), len(ib), P(arr(ob)), len(ob))
    Q = ib[0] * ib[1] * ib[2]
    for k in range(n):
        X, _ = crt([x[i * n + k] for i in range(3)], ib)
        # the fast conversion returns X + alpha Q with 0 <= alpha < ibase_size
        exact = sum(int(x[i * n + k]) * pow(Q // ib[i], -1, ib[i]) % ib[i] * (Q // ib[i]) for i in range(3))
        assert (exact - X) % Q == 0 and 0 <= (exact - X) // Q < 3
        for j, p in enumerate(ob):
            assert int(y[j * n + k]) == exact % p


def test_moddown_exact_formula(rng):
    n = 32
    ql = O.coeff_modulus_create(n, [60, 50, 50])
    p = O.coeff_modulus_create(n, [60] * 3)[:2]  # two 60-bit primes distinct from q0 (the largest)
    assert ql[0] not in p
    qlp = ql + p
    cx_coeff = O.random_limbs(rng, n, qlp)
    cx = np.concatenate([O.ntt_fwd(cx_coeff[i * n:(i + 1) * n], n, [qlp[i]]) for i in range(len(qlp))])
    out = np.zeros(len(ql) * n, dtype=np.uint64)
    O.lib().or_moddown_from_ntt(P(cx), P(out), n, P(arr(ql)), len(ql), P(arr(p)), len(p))
    out_coeff = O.ntt_inv(out, n, ql)
    Pp = p[0] * p[1]
    for k in range(n):
        # Delta = sum_i [x_i Phat_i^-1]_{p_i} Phat_i (exact integer), out = (C - Delta) / P mod q_j
        xs = [int(cx_coeff[(len(ql) + i) * n + k]) for i in range(2)]
        delta = sum(xs[i] * pow(Pp // p[i], -1, p[i]) % p[i] * (Pp // p[i]) for i in range(2))
        for j, q in enumerate(ql):
            c = int(cx_coeff[j * n + k])
            assert int(out_coeff[j * n + k]) == (c - delta) * pow(Pp, -1, q) % q


def test_rescale_exact_formula(rng):
    n = 64
    ql = O.coeff_modulus_create(n, [60, 50, 50, 50])
    L = len(ql)
    coeff = np.concatenate([O.random_limbs(rng, n, ql) for _ in range(2)])
    ct = np.concatenate([O.ntt_fwd(coeff[c * L * n:(c + 1) * L * n], n, ql) for c in range(2)])
    out = np.zeros(2 * (L - 1) * n, dtype=np.uint64)
    O.lib().or_rescale_ntt(P(ct), P(out), n, L, 2, P(arr(ql)))
    for c in range(2):
        oc = O.ntt_inv(out[c * (L - 1) * n:(c + 1) * (L - 1) * n], n, ql[:-1])
        for k in range(n):
            last = int(coeff[(c * L + L - 1) * n + k])
            for j in range(L - 1):
                v = int(coeff[(c * L + j) * n + k])
                assert int(oc[j * n + k]) == (v - last) * pow(ql[-1], -1, ql[j]) % ql[j]


# --------------------------------------------------------------------------------------
# automorphisms and bootstrap helpers
# --------------------------------------------------------------------------------------

@pytest.mark.parametrize("k", [5, 25, 3 * 5 ** 7, 127])  # 127 = 2n - 1: conjugation at n = 64
def test_galois_ntt_permutation_matches_coefficient_automorphism(rng, k):
    n = 64
    q = O.coeff_modulus_create(n, [50])[0]
    a = [int(x) for x in rng.integers(0, q, n)]
    k %= 2 * n
    sa = [0] * n
    for i in range(n):
        e = i * k % (2 * n)
        if e < n:
            sa[e] = (sa[e] + a[i]) % q
        else:
            sa[e - n] = (sa[e - n] - a[i]) % q
    fa = O.ntt_fwd(arr(a), n, [q])
    got = np.zeros(n, dtype=np.uint64)
    O.lib().or_apply_galois_ntt(P(fa), P(got), n, 1, k)
    assert np.array_equal(got, O.ntt_fwd(arr(sa), n, [q]))


def test_switch_modulus_centered_lift(rng):
    n = 16
    mods = O.coeff_modulus_create(n, [60, 50, 60])
    q0 = mods[0]
    v = O.random_limbs(rng, n, [q0])
    out = np.zeros(3 * n, dtype=np.uint64)
    O.lib().or_switch_modulus_raise(P(v), P(out), n, q0, P(arr(mods)), 3)
    for k in range(n):
        x = int(v[k])
        c = x - q0 if x > q0 // 2 else x
        for j, q in enumerate(mods):
            assert int(out[j * n + k]) == c % q


def test_monomial_ntt():
    n = 32
    mods = O.coeff_modulus_create(n, [50, 50])
    for pw in [0, 5, n, n + 3, 2 * n - 1]:
        out = np.zeros(2 * n, dtype=np.uint64)
        O.lib().or_monomial_ntt(P(out), n, 2, P(arr(mods)), pw)
        for l, q in enumerate(mods):
            c = [0] * n
            c[pw % n] = 1 if pw < n else q - 1
            assert np.array_equal(out[l * n:(l + 1) * n], O.ntt_fwd(arr(c), n, [q]))


# --------------------------------------------------------------------------------------
# end-to-end key switching with real keys
# --------------------------------------------------------------------------------------

def _polymul_ntt(a, b, n, mods):
    out = np.zeros_like(a)
    O.lib().or_poly_mul(P(a), P(b), P(out), n, len(mods), P(arr(mods)))
    return out


def test_relinearize_decrypts_to_tensor(rng):
    """Relinearisation with a hybrid key for s^2 (secretkey.cu:362-406 construction):
    <(c0', c1'), (1, s)> == c0 + c1 s + c2 s^2 + small error (mod Q_l)."""
    n = 64
    size_q, size_p = 4, 2
    qp = O.coeff_modulus_create(n, [60, 50, 50, 50, 60, 60])
    q, p = qp[:size_q], qp[size_q:]
    dnum = size_q // size_p
    # ternary secret over QP, NTT form
    s_int = rng.integers(-1, 2, n)
    s = np.concatenate([O.ntt_fwd(arr([int(v) % m for v in s_int]), n, [m]) for m in qp])
    s2 = _polymul_ntt(s, s, n, qp)
    Pm = p[0] * p[1]
    keys = []
    for d in range(dnum):
        a = O.random_limbs(rng, n, qp)
        e_int = rng.integers(-3, 4, n)
        e = np.concatenate([O.ntt_fwd(arr([int(v) % m for v in e_int]), n, [m]) for m in qp])
        as_ = _polymul_ntt(a, s, n, qp)
        b = np.zeros_like(a)
        for i, m in enumerate(qp):
            sl = slice(i * n, (i + 1) * n)
            v = (-(as_[sl].astype(object)) - e[sl].astype(object)) % m
            if d * size_p <= i < (d + 1) * size_p:  # digit d gets + P * s^2 on its own primes
                v = (v + (Pm % m) * s2[sl].astype(object)) % m
            b[sl] = v.astype(np.uint64)
        keys.append(np.concatenate([b, a]))
    size_ql = size_q  # top level
    ct = np.concatenate([O.random_limbs(rng, n, q) for _ in range(3)])
    ref = ct.copy()
    key_ptrs = (O.u64p * dnum)(*[P(k) for k in keys])
    O.lib().or_relinearize(P(ct), n, size_ql, size_q, size_p, key_ptrs, P(arr(qp)))
    L = size_ql
    c0, c1 = ct[:L * n], ct[L * n:2 * L * n]
    r0, r1, r2 = ref[:L * n], ref[L * n:2 * L * n], ref[2 * L * n:3 * L * n]
    sq, s2q = s[:L * n], s2[:L * n]
    lhs = (c0.astype(object) + _polymul_ntt(c1, sq, n, q).astype(object))
    rhs = (r0.astype(object) + _polymul_ntt(r1, sq, n, q).astype(object) + _polymul_ntt(r2, s2q, n, q).astype(object))
    diff = np.zeros(L * n, dtype=np.uint64)
    for i, m in enumerate(q):
        sl = slice(i * n, (i + 1) * n)
        diff[sl] = ((lhs[sl] - rhs[sl]) % m).astype(np.uint64)
    diff_c = O.ntt_inv(diff, n, q)
    Q = 1
    for m in q:
        Q *= m
    for k in range(n):
        x, _ = crt([diff_c[i * n + k] for i in range(L)], q)
        if x > Q // 2:
            x -= Q
        # key-switch noise ~ sum over digits of |c2 digit| * |e| / P + rounding: tiny vs Q
        assert abs(x) < 2 ** 40, x


# ---- EvalMod coefficients pinned to the reference's own tables ------------------------------

@pytest.mark.parametrize("which", ["uniform", "sparse"])
def test_eval_mod_coefficients_match_reference_tables(which):
    """The engine interpolates EvalMod's scaled cosine itself (host/bootstrap.cpp
    chebyshev_coefficients); the reference ships the same series as fixed tables
    (include/bootstrap.cuh:217-255, tests/golden/eval_mod_coefficients.json).  Same function, same
    degree: the coefficients agree to 1e-13 (the tables' printed precision), with the reference's
    c[0]/2 free-term convention (src/evaluate.cu:3259)."""
    import ctypes
    import json
    import os
    import phantom_amd as PA
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "eval_mod_coefficients.json")))[which]
    ref = np.array(g["coefficients"])
    out = (ctypes.c_double * ref.size)()
    PA.check(PA.load().phantom_eval_mod_coefficients(g["K"], g["double_angle_iterations"], ref.size - 1, out))
    ours = np.array(out[:])
    want = ref.copy()
    want[0] /= 2
    assert np.max(np.abs(ours - want)) < 1e-13, np.max(np.abs(ours - want))
