"""Bit-exact GPU parity of the lockstep-group kernels on the C5 product path, at config C4's size,
through the C-ABI, against the CPU oracle applied to each ciphertext on its own:

  phantom_lt_bsgs_group                 lt_bsgs_group_kernel          vs or_lt_bsgs
  phantom_fast_rotation_ext_batch_group keyswitch_rotate_batch_group  vs or_fast_rotation_ext / or_keyswitch_ext
  phantom_rotate_ext_accumulate_group   keyswitch_rotate_group        vs or_rotate_ext_accumulate

The reference bootstraps one ciphertext at a time (src/bootstrap.cu:843-1129); the oracle functions
restate its per-ciphertext EvalMultExt + EvalAddExtInPlace inner sums (bootstrap.cu:1322-1332) and
EvalFastRotationExt / KeySwitchExt (src/evaluate.cu:3660-3755, 3786-3837, 3876-3940).  Shapes: the
CoeffToSlot levels (chains 2 and 3: g 32, b 8, beta 3) and the SlotToCoeff levels (chains 17 and
18: beta 2), groups of 2, 4 and 8 with distinct inputs per ciphertext."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
import phantom_amd as PA
from gpu_util import ptr, stream, to_dev, to_host, torch

pytestmark = pytest.mark.gpu

N = 1 << 16
C4_BITS = [60] + [59] * 29 + [60] * 10
SIZE_P = 10


@pytest.fixture(scope="module")
def c4():
    mods = O.coeff_modulus_create(N, C4_BITS)
    return PA.Context(N, mods, SIZE_P)


def _lib():
    return PA.load()


def _ext_mods(ctx, chain):
    return ctx.ql(chain) + ctx.moduli[ctx.size_Q:]


def _rand(rng, mods, polys=1):
    return np.concatenate([O.random_limbs(rng, N, mods) for _ in range(polys)])


def _vp(addrs):
    return PA.ptr_array(list(addrs))


def _keys(rng, ctx):
    dnum = -(-ctx.size_Q // ctx.size_P)
    keys = [_rand(rng, ctx.moduli, 2) for _ in range(dnum)]
    return keys, [to_dev(k) for k in keys]


@pytest.mark.parametrize("chain,b,group", [(2, 8, 2), (3, 8, 4), (17, 8, 8), (18, 3, 8), (2, 8, 5), (18, 3, 7)])
def test_lt_bsgs_group(c4, rng, chain, b, group):
    """inner sums of `group` ciphertexts in one launch == or_lt_bsgs per ciphertext (odd group sizes:
    the balanced lockstep groups of EvalBootstrapBatch)"""
    g = 32
    em = _ext_mods(c4, chain)
    W = 2 * len(em) * N
    pool = [_rand(rng, em, 2) for _ in range(g + 8)]  # ciphertext c takes babies pool[(3 j + 7 c) % 40]
    dpool = [to_dev(x) for x in pool]
    sel = [[(3 * j + 7 * c) % len(pool) for j in range(g)] for c in range(group)]
    pts = [_rand(rng, em) for _ in range(g * b)]
    pts[5] = np.zeros_like(pts[5])  # an absent diagonal reads the zero plaintext
    dpts = [to_dev(x) for x in pts]
    t = torch()
    dbabies = [t.cat([dpool[i] for i in sel[c]]) for c in range(group)]  # contiguous, stride W
    dacc = [to_dev(np.full(W, 3, dtype=np.uint64)) for _ in range(group)]
    dgiant = [to_dev(np.full(max(b - 1, 1) * W, 9, dtype=np.uint64)) for _ in range(group)]
    PA.check(_lib().phantom_lt_bsgs_group(c4.handle, chain, group, _vp(ptr(x) for x in dbabies), W, g,
                                          _vp(ptr(x) for x in dpts), b, _vp(ptr(x) for x in dacc),
                                          _vp(ptr(x) for x in dgiant), W, stream()))
    mods = O.P(O.arr(c4.moduli))
    for c in range(group):
        want = [np.zeros(W, dtype=np.uint64) for _ in range(b)]
        O.lib().or_lt_bsgs(O.ptrs([pool[i] for i in sel[c]]), g, O.ptrs(pts), b, O.ptrs(want), N, len(c4.ql(chain)),
                           c4.size_Q, c4.size_P, mods)
        assert np.array_equal(to_host(dacc[c]), want[0]), (c, 0)
        giants = to_host(dgiant[c])
        for i in range(1, b):
            assert np.array_equal(giants[(i - 1) * W:i * W], want[i]), (c, i)


@pytest.mark.parametrize("bits,b,group", [(61, 8, 2), (61, 3, 3), (59, 8, 4)])
def test_lt_bsgs_group_moduli(rng, bits, b, group):
    """grouped inner sums at the split partial sums' bounds: N = 4096, 8 + 2 moduli of `bits` bits
    (61-bit: folded every 4 products, LtGroupArgs::q60 = 0) == or_lt_bsgs per ciphertext"""
    n, size_p, chain, g = 1 << 12, 2, 1, 32
    ctx = PA.Context(n, O.coeff_modulus_create(n, [bits] * 10), size_p)
    em = ctx.ql(chain) + ctx.moduli[ctx.size_Q:]
    W = 2 * len(em) * n
    rand = lambda polys: np.concatenate([O.random_limbs(rng, n, em) for _ in range(polys)])
    babies = [[rand(2) for _ in range(g)] for _ in range(group)]
    pts = [rand(1) for _ in range(g * b)]
    dbabies = [to_dev(np.concatenate(bs)) for bs in babies]
    dpts = [to_dev(x) for x in pts]
    dacc = [to_dev(np.full(W, 3, dtype=np.uint64)) for _ in range(group)]
    dgiant = [to_dev(np.full(max(b - 1, 1) * W, 9, dtype=np.uint64)) for _ in range(group)]
    PA.check(_lib().phantom_lt_bsgs_group(ctx.handle, chain, group, _vp(ptr(x) for x in dbabies), W, g,
                                          _vp(ptr(x) for x in dpts), b, _vp(ptr(x) for x in dacc),
                                          _vp(ptr(x) for x in dgiant), W, stream()))
    mods = O.P(O.arr(ctx.moduli))
    for c in range(group):
        want = [np.zeros(W, dtype=np.uint64) for _ in range(b)]
        O.lib().or_lt_bsgs(O.ptrs(babies[c]), g, O.ptrs(pts), b, O.ptrs(want), n, len(ctx.ql(chain)), ctx.size_Q,
                           ctx.size_P, mods)
        assert np.array_equal(to_host(dacc[c]), want[0]), (bits, c, 0)
        giants = to_host(dgiant[c])
        for i in range(1, b):
            assert np.array_equal(giants[(i - 1) * W:i * W], want[i]), (bits, c, i)


@pytest.mark.parametrize("chain,count,group", [(2, 32, 2), (3, 12, 4), (17, 32, 2), (18, 12, 8)])
def test_fast_rotation_ext_batch_group(c4, rng, chain, count, group):
    """the baby steps of `group` ciphertexts in one launch == per ciphertext and rotation
    or_fast_rotation_ext (add_first) / or_keyswitch_ext for the identity entry"""
    ql = c4.ql(chain)
    em = _ext_mods(c4, chain)
    W = 2 * len(em) * N
    beta = -(-len(ql) // SIZE_P)
    cts = [_rand(rng, ql, 2) for _ in range(group)]
    digits = [_rand(rng, em, beta) for _ in range(group)]
    elts = [pow(5, 3 * k + 1, 2 * N) for k in range(count)]
    elts[-1] = 2 * N - 1  # a conjugation among the rotations
    identity_at = 0
    dnum = -(-c4.size_Q // SIZE_P)
    keysets = [_keys(rng, c4) for _ in range(3)]  # three key sets shared round robin
    kset = [keysets[k % 3] for k in range(count)]
    dcts, ddig = [to_dev(x) for x in cts], [to_dev(x) for x in digits]
    douts = [to_dev(np.full(count * W, 5, dtype=np.uint64)) for _ in range(group)]
    key_arrays = [None if k == identity_at else _vp(ptr(x) for x in kset[k][1]) for k in range(count)]
    kk = (ctypes.POINTER(ctypes.c_void_p) * count)(*[ctypes.cast(a, ctypes.POINTER(ctypes.c_void_p)) if a is not None
                                                     else None for a in key_arrays])
    el = (ctypes.c_uint32 * count)(*elts)
    outs = [ptr(douts[c]) + 8 * k * W for c in range(group) for k in range(count)]
    PA.check(_lib().phantom_fast_rotation_ext_batch_group(c4.handle, chain, group, _vp(ptr(x) for x in dcts),
                                                          _vp(ptr(x) for x in ddig), kk, dnum, el, count, _vp(outs),
                                                          stream()))
    mods = O.P(O.arr(c4.moduli))
    for c in range(group):
        got = to_host(douts[c])
        for k in range(count):
            want = np.zeros(W, dtype=np.uint64)
            if k == identity_at:
                O.lib().or_keyswitch_ext(O.P(cts[c]), O.P(want), N, len(ql), c4.size_Q, c4.size_P, mods)
            else:
                O.lib().or_fast_rotation_ext(O.P(cts[c]), O.P(digits[c]), O.ptrs(kset[k][0]), elts[k], 1, O.P(want), N,
                                             len(ql), c4.size_Q, c4.size_P, mods)
            assert np.array_equal(got[k * W:(k + 1) * W], want), (c, k)


@pytest.mark.parametrize("bits,chain,group", [(61, 1, 2), (61, 3, 4), (59, 1, 4), (59, 4, 2)])
def test_fast_rotation_ext_batch_group_moduli_and_beta(rng, bits, chain, group):
    """the grouped baby steps' two reductions at their partial-sum bounds: N = 4096, 8 + 2 moduli
    of `bits` bits, so beta = 4 at chain 1 (all of Q).  61-bit moduli take the exact form (a lazy sum below
    6q), moduli below 2^60 the approximate-quotient form (below 12q); both == or_fast_rotation_ext
    / or_keyswitch_ext per ciphertext and rotation"""
    n, size_p = 1 << 12, 2
    mods = O.coeff_modulus_create(n, [bits] * 10)
    ctx = PA.Context(n, mods, size_p)
    ql = ctx.ql(chain)
    em = ql + ctx.moduli[ctx.size_Q:]
    W = 2 * len(em) * n
    beta = -(-len(ql) // size_p)
    dnum = -(-ctx.size_Q // size_p)
    count = 5
    cts = [np.concatenate([O.random_limbs(rng, n, ql) for _ in range(2)]) for _ in range(group)]
    digits = [np.concatenate([O.random_limbs(rng, n, em) for _ in range(beta)]) for _ in range(group)]
    elts = [pow(5, 3 * k + 1, 2 * n) for k in range(count)]
    elts[-1] = 2 * n - 1
    keys = [[np.concatenate([O.random_limbs(rng, n, ctx.moduli) for _ in range(2)]) for _ in range(dnum)]
            for _ in range(2)]
    dkeys = [[to_dev(x) for x in ks] for ks in keys]
    dcts, ddig = [to_dev(x) for x in cts], [to_dev(x) for x in digits]
    douts = [to_dev(np.full(count * W, 5, dtype=np.uint64)) for _ in range(group)]
    key_arrays = [None if k == 0 else _vp(ptr(x) for x in dkeys[k % 2]) for k in range(count)]
    kk = (ctypes.POINTER(ctypes.c_void_p) * count)(*[ctypes.cast(a, ctypes.POINTER(ctypes.c_void_p)) if a is not None
                                                     else None for a in key_arrays])
    el = (ctypes.c_uint32 * count)(*elts)
    outs = [ptr(douts[c]) + 8 * k * W for c in range(group) for k in range(count)]
    PA.check(_lib().phantom_fast_rotation_ext_batch_group(ctx.handle, chain, group, _vp(ptr(x) for x in dcts),
                                                          _vp(ptr(x) for x in ddig), kk, dnum, el, count, _vp(outs),
                                                          stream()))
    pm = O.P(O.arr(ctx.moduli))
    for c in range(group):
        got = to_host(douts[c])
        for k in range(count):
            want = np.zeros(W, dtype=np.uint64)
            if k == 0:
                O.lib().or_keyswitch_ext(O.P(cts[c]), O.P(want), n, len(ql), ctx.size_Q, ctx.size_P, pm)
            else:
                O.lib().or_fast_rotation_ext(O.P(cts[c]), O.P(digits[c]), O.ptrs(keys[k % 2]), elts[k], 1, O.P(want),
                                             n, len(ql), ctx.size_Q, ctx.size_P, pm)
            assert np.array_equal(got[k * W:(k + 1) * W], want), (bits, c, k)


def test_fast_rotation_ext_batch_group_rejects_ragged_offsets(c4, rng):
    """every ciphertext's outputs must sit at the entry offsets of ciphertext 0"""
    chain, count, group = 17, 2, 2
    ql, em = c4.ql(chain), _ext_mods(c4, chain)
    W = 2 * len(em) * N
    dcts = [to_dev(np.zeros(2 * len(ql) * N, dtype=np.uint64)) for _ in range(group)]
    ddig = [to_dev(np.zeros(2 * len(em) * N, dtype=np.uint64)) for _ in range(group)]
    douts = [to_dev(np.zeros(3 * W, dtype=np.uint64)) for _ in range(group)]
    kk = (ctypes.POINTER(ctypes.c_void_p) * count)(None, None)
    el = (ctypes.c_uint32 * count)(1, 1)
    outs = [ptr(douts[0]), ptr(douts[0]) + 8 * W, ptr(douts[1]), ptr(douts[1]) + 16 * W]
    rc = _lib().phantom_fast_rotation_ext_batch_group(c4.handle, chain, group, _vp(ptr(x) for x in dcts),
                                                      _vp(ptr(x) for x in ddig), kk, 2, el, count, _vp(outs), stream())
    assert rc != 0


@pytest.mark.parametrize("chain,group,accumulate", [(2, 2, 1), (3, 4, 1), (17, 8, 1), (18, 8, 0)])
def test_rotate_ext_accumulate_group(c4, rng, chain, group, accumulate):
    """one giant-step rotation of `group` ciphertexts in one launch == or_rotate_ext_accumulate each"""
    em = _ext_mods(c4, chain)
    W = 2 * len(em) * N
    exts = [_rand(rng, em, 2) for _ in range(group)]
    accs = [_rand(rng, em, 2) for _ in range(group)]
    keys, dkeys = _keys(rng, c4)
    elt = pow(5, 1024 * (chain % 5 + 1), 2 * N)
    dext, dacc = [to_dev(x) for x in exts], [to_dev(x) for x in accs]
    PA.check(_lib().phantom_rotate_ext_accumulate_group(c4.handle, chain, group, _vp(ptr(x) for x in dext),
                                                        _vp(ptr(x) for x in dkeys), len(dkeys), elt,
                                                        _vp(ptr(x) for x in dacc), accumulate, stream()))
    mods = O.P(O.arr(c4.moduli))
    for c in range(group):
        want = accs[c].copy()
        O.lib().or_rotate_ext_accumulate(O.P(exts[c].copy()), O.ptrs(keys), elt, O.P(want), accumulate, N,
                                         len(c4.ql(chain)), c4.size_Q, c4.size_P, mods)
        assert np.array_equal(to_host(dacc[c]), want), c
