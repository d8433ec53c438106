"""GPU parity of the CKKS hot path (multiply, modup, key-switch inner product, moddown,
relinearize, rescale, automorphism, ModRaise lift) against the CPU oracle, bit-exact.

Config 3: N = 2^16, Q = {60, 44 x 50}, P = 15 x 60 (examples/3_ckks.cu:796-803).
A small chain (N = 2^12, 7 data primes, alpha = 3) exercises partial digits and lower levels.
Key-switching keys are uniform random digits here (parity is a property of the arithmetic, not
of key structure); tests/test_oracle.py checks the oracle's key switch decrypts correctly.
"""
import ctypes

import numpy as np
import pytest

import ks_oracle as KO
import oracle_lib as O
import phantom_amd as PA
from gpu_util import ptr, stream, to_dev, to_host

pytestmark = pytest.mark.gpu

C3_BITS = [60] + [50] * 44 + [60] * 15
SMALL_BITS = [60, 50, 50, 50, 50, 50, 50, 60, 60, 60]


def _make(n, bits, special):
    mods = O.coeff_modulus_create(n, bits)
    return PA.Context(n, mods, special)


@pytest.fixture(scope="module")
def c3():
    return _make(1 << 16, C3_BITS, 15)


@pytest.fixture(scope="module")
def small():
    return _make(1 << 12, SMALL_BITS, 3)


def _lib():
    return PA.load()


def _rand_ct(rng, ctx, chain, polys):
    ql = ctx.ql(chain)
    return np.concatenate([O.random_limbs(rng, ctx.n, ql) for _ in range(polys)])


def _keys(rng, ctx):
    dnum = -(-ctx.size_Q // ctx.size_P)
    keys = [np.concatenate([O.random_limbs(rng, ctx.n, ctx.moduli) for _ in range(2)]) for _ in range(dnum)]
    return keys, [to_dev(k) for k in keys]


def _oracle_keys(keys):
    return (O.u64p * len(keys))(*[O.P(k) for k in keys])


@pytest.mark.parametrize("fixture,chain", [("c3", 1), ("small", 1), ("small", 4)])
def test_multiply(request, rng, fixture, chain):
    ctx = request.getfixturevalue(fixture)
    ql = ctx.ql(chain)
    a, b = _rand_ct(rng, ctx, chain, 2), _rand_ct(rng, ctx, chain, 2)
    da, db = to_dev(a), to_dev(b)
    dout = to_dev(np.zeros(3 * len(ql) * ctx.n, dtype=np.uint64))
    PA.check(_lib().phantom_multiply(ctx.handle, chain, ptr(da), ptr(db), ptr(dout), stream()))
    want = np.zeros(3 * len(ql) * ctx.n, dtype=np.uint64)
    O.lib().or_tensor_prod_2x2(O.P(a), O.P(b), O.P(want), ctx.n, len(ql), O.P(O.arr(ql)))
    assert np.array_equal(to_host(dout), want)


@pytest.mark.parametrize("fixture,chain", [("c3", 1), ("small", 1), ("small", 5)])
def test_square(request, rng, fixture, chain):
    """tensor_square_2x2_rns_poly (src/polymath.cu:538-582), out of place and in place"""
    ctx = request.getfixturevalue(fixture)
    ql = ctx.ql(chain)
    a = _rand_ct(rng, ctx, chain, 2)
    # extreme residues: q - 1 and 0 in the first limb
    a[: ctx.n // 2] = ql[0] - 1
    a[ctx.n // 2: ctx.n] = 0
    want = np.zeros(3 * len(ql) * ctx.n, dtype=np.uint64)
    O.lib().or_tensor_square_2x2(O.P(a), O.P(want), ctx.n, len(ql), O.P(O.arr(ql)))
    da = to_dev(a)
    dout = to_dev(np.zeros(3 * len(ql) * ctx.n, dtype=np.uint64))
    PA.check(_lib().phantom_square(ctx.handle, chain, ptr(da), ptr(dout), stream()))
    assert np.array_equal(to_host(dout), want)
    dio = to_dev(np.concatenate([a, np.zeros(len(ql) * ctx.n, dtype=np.uint64)]))
    PA.check(_lib().phantom_square(ctx.handle, chain, ptr(dio), ptr(dio), stream()))
    assert np.array_equal(to_host(dio), want)
    # the square is the product with itself
    prod = np.zeros_like(want)
    O.lib().or_tensor_prod_2x2(O.P(a), O.P(a), O.P(prod), ctx.n, len(ql), O.P(O.arr(ql)))
    assert np.array_equal(prod, want)


@pytest.mark.parametrize("fixture,chain", [("c3", 1), ("small", 1), ("small", 2), ("small", 6)])
def test_modup(request, rng, fixture, chain):
    ctx = request.getfixturevalue(fixture)
    ql, p = ctx.ql(chain), ctx.moduli[ctx.size_Q:]
    beta = -(-len(ql) // ctx.size_P)
    c2 = O.random_limbs(rng, ctx.n, ql)
    d = to_dev(c2)
    dout = to_dev(np.zeros(beta * (len(ql) + len(p)) * ctx.n, dtype=np.uint64))
    PA.check(_lib().phantom_modup(ctx.handle, chain, ptr(d), ptr(dout), stream()))
    want = np.zeros(beta * (len(ql) + len(p)) * ctx.n, dtype=np.uint64)
    O.lib().or_modup(O.P(c2), O.P(want), ctx.n, O.P(O.arr(ql)), len(ql), O.P(O.arr(p)), len(p))
    assert np.array_equal(to_host(dout), want)


@pytest.mark.parametrize("fixture,chain", [("c3", 1), ("small", 3)])
def test_inner_product(request, rng, fixture, chain):
    ctx = request.getfixturevalue(fixture)
    ql, p = ctx.ql(chain), ctx.moduli[ctx.size_Q:]
    qlp = ql + p
    beta = -(-len(ql) // ctx.size_P)
    tmu = np.concatenate([O.random_limbs(rng, ctx.n, qlp) for _ in range(beta)])
    keys, dkeys = _keys(rng, ctx)
    dt = to_dev(tmu)
    dcx = to_dev(np.zeros(2 * len(qlp) * ctx.n, dtype=np.uint64))
    kp = PA.ptr_array([ptr(k) for k in dkeys])
    PA.check(_lib().phantom_keyswitch_inner_prod(ctx.handle, chain, ptr(dt), kp, len(dkeys), ptr(dcx), stream()))
    want = np.zeros(2 * len(qlp) * ctx.n, dtype=np.uint64)
    O.lib().or_keyswitch_inner_prod(O.P(tmu), _oracle_keys(keys), O.P(want), ctx.n, len(ql), ctx.size_Q, ctx.size_P,
                                    beta, O.P(O.arr(ctx.moduli)))
    assert np.array_equal(to_host(dcx), want)


@pytest.mark.parametrize("fixture,chain", [("c3", 1), ("c3", 30), ("small", 1), ("small", 5)])
def test_moddown(request, rng, fixture, chain):
    ctx = request.getfixturevalue(fixture)
    ql, p = ctx.ql(chain), ctx.moduli[ctx.size_Q:]
    cx = O.random_limbs(rng, ctx.n, ql + p)
    d = to_dev(cx)
    dout = to_dev(np.zeros(len(ql) * ctx.n, dtype=np.uint64))
    PA.check(_lib().phantom_moddown_from_ntt(ctx.handle, chain, ptr(d), ptr(dout), stream()))
    want = np.zeros(len(ql) * ctx.n, dtype=np.uint64)
    cxo = cx.copy()
    O.lib().or_moddown_from_ntt(O.P(cxo), O.P(want), ctx.n, O.P(O.arr(ql)), len(ql), O.P(O.arr(p)), len(p))
    assert np.array_equal(to_host(dout), want)


@pytest.mark.parametrize("fixture,chain", [("c3", 1), ("c3", 30), ("small", 1), ("small", 2), ("small", 5)])
def test_moddown_modup_fused(request, rng, fixture, chain):
    """The giant-step fusion equals modup(moddown(cx)) bit for bit."""
    ctx = request.getfixturevalue(fixture)
    ql, p = ctx.ql(chain), ctx.moduli[ctx.size_Q:]
    beta = -(-len(ql) // ctx.size_P)
    cx = O.random_limbs(rng, ctx.n, ql + p)
    d = to_dev(cx)
    dout = to_dev(np.zeros(beta * (len(ql) + len(p)) * ctx.n, dtype=np.uint64))
    PA.check(_lib().phantom_moddown_modup(ctx.handle, chain, ptr(d), ptr(dout), stream()))
    down = np.zeros(len(ql) * ctx.n, dtype=np.uint64)
    O.lib().or_moddown_from_ntt(O.P(cx.copy()), O.P(down), ctx.n, O.P(O.arr(ql)), len(ql), O.P(O.arr(p)), len(p))
    want = np.zeros(beta * (len(ql) + len(p)) * ctx.n, dtype=np.uint64)
    O.lib().or_modup(O.P(down), O.P(want), ctx.n, O.P(O.arr(ql)), len(ql), O.P(O.arr(p)), len(p))
    assert np.array_equal(to_host(dout), want)


@pytest.mark.parametrize("fixture,chain", [("c3", 1), ("c3", 30), ("small", 2), ("small", 5)])
def test_moddown_modup_batch(request, rng, fixture, chain):
    """The giant steps' batched moddown∘modup (3 polynomials at a padded stride, full and short
    digits) equals modup(moddown(cx_i)) of each polynomial bit for bit."""
    ctx = request.getfixturevalue(fixture)
    ql, p = ctx.ql(chain), ctx.moduli[ctx.size_Q:]
    qlp = len(ql) + len(p)
    beta, count, stride = -(-len(ql) // ctx.size_P), 3, 2 * (len(ql) + len(p)) * ctx.n
    cxs = [O.random_limbs(rng, ctx.n, ql + p) for _ in range(count)]
    buf = np.zeros(count * stride, dtype=np.uint64)
    for i, cx in enumerate(cxs):
        buf[i * stride:i * stride + cx.size] = cx
    d = to_dev(buf)
    dout = to_dev(np.zeros(count * beta * qlp * ctx.n, dtype=np.uint64))
    PA.check(_lib().phantom_moddown_modup_batch(ctx.handle, chain, ptr(d), count, stride, ptr(dout), stream()))
    got = to_host(dout).reshape(count, -1)
    for i, cx in enumerate(cxs):
        down = np.zeros(len(ql) * ctx.n, dtype=np.uint64)
        O.lib().or_moddown_from_ntt(O.P(cx.copy()), O.P(down), ctx.n, O.P(O.arr(ql)), len(ql), O.P(O.arr(p)), len(p))
        want = np.zeros(beta * qlp * ctx.n, dtype=np.uint64)
        O.lib().or_modup(O.P(down), O.P(want), ctx.n, O.P(O.arr(ql)), len(ql), O.P(O.arr(p)), len(p))
        assert np.array_equal(got[i], want), i


@pytest.mark.parametrize("fixture,chain", [("c3", 1), ("c3", 30), ("small", 1), ("small", 5)])
def test_moddown_rescale_fused(request, rng, fixture, chain):
    """moddown + rescale as one division by P q_last = moddown_from_NTT with {q_last} u P as the
    special basis (the buffer layout [Ql-1][q_last][P] is exactly that split)."""
    ctx = request.getfixturevalue(fixture)
    ql, p = ctx.ql(chain), ctx.moduli[ctx.size_Q:]
    polys = 2
    cxs = [O.random_limbs(rng, ctx.n, ql + p) for _ in range(polys)]
    d = to_dev(np.concatenate(cxs))
    dout = to_dev(np.zeros(polys * (len(ql) - 1) * ctx.n, dtype=np.uint64))
    PA.check(_lib().phantom_moddown_rescale(ctx.handle, chain, ptr(d), ptr(dout), polys, stream()))
    want = []
    for cx in cxs:
        w = np.zeros((len(ql) - 1) * ctx.n, dtype=np.uint64)
        O.lib().or_moddown_from_ntt(O.P(cx.copy()), O.P(w), ctx.n, O.P(O.arr(ql[:-1])), len(ql) - 1,
                                    O.P(O.arr([ql[-1]] + list(p))), len(p) + 1)
        want.append(w)
    assert np.array_equal(to_host(dout), np.concatenate(want))


@pytest.mark.parametrize("fixture,chain", [("c3", 1), ("small", 1), ("small", 4), ("small", 7)])
def test_relinearize(request, rng, fixture, chain):
    ctx = request.getfixturevalue(fixture)
    ql = ctx.ql(chain)
    ct = _rand_ct(rng, ctx, chain, 3)
    keys, dkeys = _keys(rng, ctx)
    d = to_dev(ct)
    kp = PA.ptr_array([ptr(k) for k in dkeys])
    PA.check(_lib().phantom_relinearize(ctx.handle, chain, ptr(d), kp, len(dkeys), stream()))
    want = ct.copy()
    O.lib().or_relinearize(O.P(want), ctx.n, len(ql), ctx.size_Q, ctx.size_P, _oracle_keys(keys),
                           O.P(O.arr(ctx.moduli)))
    got = to_host(d)
    L = len(ql)
    assert np.array_equal(got[:2 * L * ctx.n], want[:2 * L * ctx.n])


@pytest.mark.parametrize("fixture,chain", [("c3", 1), ("c3", 30), ("small", 1), ("small", 5)])
def test_relinearize_rescale(request, rng, fixture, chain):
    """The bootstrap's EvalMult + ModReduce key switch (include/phantom_amd.h
    phantom_relinearize_rescale): the P-scaled (c0, c1) + KeySwitch(c2), divided by P q_last at
    once, with the inner product's first L-1 limbs formed in the finish's epilogue; bit-exact vs
    the oracle's inner product + addend + moddown_from_NTT over the special basis {q_last} u P."""
    ctx = request.getfixturevalue(fixture)
    ql, p = ctx.ql(chain), ctx.moduli[ctx.size_Q:]
    L, n = len(ql), ctx.n
    ct = _rand_ct(rng, ctx, chain, 3)
    keys, dkeys = _keys(rng, ctx)
    d = to_dev(ct)
    dout = to_dev(np.zeros(2 * (L - 1) * n, dtype=np.uint64))
    kp = PA.ptr_array([ptr(k) for k in dkeys])
    PA.check(_lib().phantom_relinearize_rescale(ctx.handle, chain, ptr(d), ptr(dout), kp, len(dkeys), stream()))
    assert np.array_equal(to_host(dout), KO.relinearize_rescale(ctx, chain, ct, keys))


@pytest.mark.parametrize("fixture,chain,count", [("c3", 1, 2), ("c3", 30, 3), ("small", 1, 5), ("small", 5, 1)])
def test_relinearize_rescale_batch(request, rng, fixture, chain, count):
    """`count` relinearize + rescale products in shared launches (include/phantom_amd.h
    phantom_relinearize_rescale_batch: batched modup with grouped digit NTTs, one moddown-rescale
    over 2 count polynomials with per-product outputs and addends): every product bit-exact vs the
    oracle composition, with padded strides between the products."""
    ctx = request.getfixturevalue(fixture)
    L, n = len(ctx.ql(chain)), ctx.n
    cts = [_rand_ct(rng, ctx, chain, 3) for _ in range(count)]
    keys, dkeys = _keys(rng, ctx)
    s_in, s_out = 3 * L * n + 5 * n, 2 * (L - 1) * n + 3 * n
    buf = np.zeros(count * s_in, dtype=np.uint64)
    for k, ct in enumerate(cts):
        buf[k * s_in:k * s_in + 3 * L * n] = ct
    d = to_dev(buf)
    dout = to_dev(np.full(count * s_out, 9, dtype=np.uint64))
    kp = PA.ptr_array([ptr(k) for k in dkeys])
    PA.check(_lib().phantom_relinearize_rescale_batch(ctx.handle, chain, ptr(d), s_in, count, ptr(dout), s_out, kp,
                                                      len(dkeys), stream()))
    got = to_host(dout)
    for k, ct in enumerate(cts):
        assert np.array_equal(got[k * s_out:k * s_out + 2 * (L - 1) * n], KO.relinearize_rescale(ctx, chain, ct, keys)), k
        assert np.all(got[k * s_out + 2 * (L - 1) * n:(k + 1) * s_out] == 9), k  # padding untouched


@pytest.mark.parametrize("fixture,chain", [("c3", 1), ("c3", 44), ("small", 1), ("small", 6)])
def test_rescale(request, rng, fixture, chain):
    ctx = request.getfixturevalue(fixture)
    ql = ctx.ql(chain)
    L = len(ql)
    ct = _rand_ct(rng, ctx, chain, 2)
    d = to_dev(ct)
    dout = to_dev(np.zeros(2 * (L - 1) * ctx.n, dtype=np.uint64))
    PA.check(_lib().phantom_rescale_to_next(ctx.handle, chain, ptr(d), ptr(dout), 2, stream()))
    want = np.zeros(2 * (L - 1) * ctx.n, dtype=np.uint64)
    O.lib().or_rescale_ntt(O.P(ct), O.P(want), ctx.n, L, 2, O.P(O.arr(ql)))
    assert np.array_equal(to_host(dout), want)
    assert np.array_equal(to_host(d), ct)  # input untouched


def test_rescale_at_last_level_is_rejected(small):
    d = to_dev(np.zeros(2 * small.n, dtype=np.uint64))
    rc = _lib().phantom_rescale_to_next(small.handle, 7, ptr(d), ptr(d), 2, stream())
    assert rc == 1 and b"end of modulus switching chain" in _lib().phantom_last_error()


@pytest.mark.parametrize("elt", [5, 25, 3125, 2 * (1 << 12) - 1])
def test_galois(small, rng, elt):
    L = 4
    a = O.random_limbs(rng, small.n, small.moduli[:L])
    d, dout = to_dev(a), to_dev(np.zeros_like(a))
    PA.check(_lib().phantom_apply_galois_ntt(small.handle, elt, ptr(d), ptr(dout), L, stream()))
    want = np.zeros_like(a)
    O.lib().or_apply_galois_ntt(O.P(a), O.P(want), small.n, L, elt)
    assert np.array_equal(to_host(dout), want)


def test_switch_modulus_raise(small, rng):
    L = small.size_Q
    q0 = small.moduli[0]
    v = O.random_limbs(rng, small.n, [q0])
    d, dout = to_dev(v), to_dev(np.zeros(L * small.n, dtype=np.uint64))
    PA.check(_lib().phantom_switch_modulus_raise(small.handle, ptr(d), ptr(dout), L, stream()))
    want = np.zeros(L * small.n, dtype=np.uint64)
    O.lib().or_switch_modulus_raise(O.P(v), O.P(want), small.n, q0, O.P(O.arr(small.moduli)), L)
    assert np.array_equal(to_host(dout), want)


@pytest.mark.parametrize("op", [0, 1, 2, 3])
def test_poly_ops(small, rng, op):
    off, L = 2, 5
    mods = small.moduli[off:off + L]
    a, b = O.random_limbs(rng, small.n, mods), O.random_limbs(rng, small.n, mods)
    da, db, do = to_dev(a), to_dev(b), to_dev(np.zeros_like(a))
    PA.check(_lib().phantom_poly_op(small.handle, op, ptr(da), ptr(db), ptr(do), off, L, stream()))
    want = np.zeros_like(a)
    m = O.arr(mods)
    fn = [O.lib().or_poly_add, O.lib().or_poly_sub, O.lib().or_poly_mul][op] if op < 3 else None
    if fn:
        fn(O.P(a), O.P(b), O.P(want), small.n, L, O.P(m))
    else:
        O.lib().or_poly_negate(O.P(a), O.P(want), small.n, L, O.P(m))
    assert np.array_equal(to_host(do), want)


# ---- samplers (src/prng.cu sample_*_poly) against the numpy ChaCha20 restatement -----------

@pytest.mark.parametrize("kind", [0, 1, 2])
def test_device_samplers_match_chacha20(kind):
    import chacha_np as C
    n = 4096
    mods = PA.coeff_modulus_create(n, [60, 50, 40, 60])
    ctx = PA.Context(n, mods, 1)
    key = [0x01234567, 0x89ABCDEF, 7, 11, 13, 17, 19, 0xFFFFFFF1]
    nonce = (5 << 40) | 3
    L = 3
    out = to_dev(np.zeros(L * n, dtype=np.uint64))
    k = (ctypes.c_uint32 * 8)(*key)
    PA.check(PA.load().phantom_sample_poly(ctx.handle, kind, k, nonce, ptr(out), L, stream()))
    got = to_host(out)
    want = [C.sample_uniform, C.sample_cbd, C.sample_ternary][kind](key, nonce, mods[:L], n)
    assert np.array_equal(got, want)
    if kind == 0:  # residues, and not a constant: every limb covers most of its range
        for l, q in enumerate(mods[:L]):
            assert got[l * n:(l + 1) * n].max() < q and got[l * n:(l + 1) * n].max() > q // 2
    else:
        small = np.where(got[:n] > mods[0] // 2, got[:n].astype(np.float64) - mods[0], got[:n].astype(np.float64))
        assert np.abs(small).max() <= (21 if kind == 1 else 1)
    ctx.close()


@pytest.mark.parametrize("log_n,which", [(12, "reject"), (16, "c4")])
def test_sample_uniform_seeded_matches_reference_expansion(log_n, which):
    """`a` of a seed-compressed symmetric ciphertext: the device expansion of a 64-byte seed
    (phantom_sample_uniform_seeded, csrc/salsa.h) equals the oracle's restatement of the
    reference's sample_uniform_poly (src/prng.cu:164-197) bit for bit — at primes where the
    rejection path is frequent (3 * 2^58 + k 2^17 + 1) and on the C4 chain (40 limbs)."""
    from test_capi import SALSA_REJECT_PRIMES
    n = 1 << log_n
    if which == "reject":
        mods = SALSA_REJECT_PRIMES + O.coeff_modulus_create(n, [60])
        ctx = PA.Context(n, mods, 1)
    else:
        mods = O.coeff_modulus_create(n, [60] + [59] * 29 + [60] * 10)
        ctx = PA.Context(n, mods, 10)
    L = len(mods) - (1 if which == "reject" else 0)
    for seed in (bytes(range(64)), bytes((31 * i + 5) & 0xFF for i in range(64))):
        dout = to_dev(np.zeros(L * n, dtype=np.uint64))
        PA.check(_lib().phantom_sample_uniform_seeded(ctx.handle, seed, ptr(dout), L, stream()))
        want = np.zeros(L * n, dtype=np.uint64)
        O.lib().or_sample_uniform_seeded(seed, O.P(O.arr(mods[:L])), n, L, O.P(want))
        assert np.array_equal(to_host(dout), want)
