"""The opt-in unbiased moddown (include/phantom_amd.h phantom_context_set_unbiased_moddown,
host/rns_tool.h RnsTool::set_unbias; no reference counterpart).  With it on, every moddown adds
floor(size_P / 2) and every moddown + rescale floor((size_P + 1) / 2) to each output coefficient,
and nothing else changes: each case below is the bit-exact oracle result of the reference's
arithmetic (the same composition tests/test_gpu_ckks.py checks with the option off) plus that
constant, checked by taking the difference back to the coefficient domain with the oracle's
INTT.  Turning the option off again restores the reference's results bit for bit.  Both parities
of size_P: 3 (k = 1 / 2) and 4 (k = 2 / 2), at N = 2^12 (2-D NTT path, partial digits) and one
case at the C3 shape."""
import numpy as np
import pytest

import ks_oracle as KO
import oracle_lib as O
import phantom_amd as PA
from gpu_util import ptr, stream, to_dev, to_host

pytestmark = pytest.mark.gpu

SHAPES = {
    "p3": (1 << 12, [60, 50, 50, 50, 50, 50, 50, 60, 60, 60], 3),
    "p4": (1 << 12, [60, 50, 50, 50, 50, 50, 50, 60, 60, 60, 60], 4),
    "c3": (1 << 16, [60] + [50] * 44 + [60] * 15, 15),
}


@pytest.fixture(scope="module")
def contexts():
    made = {}

    def get(name):
        if name not in made:
            n, bits, special = SHAPES[name]
            made[name] = PA.Context(n, O.coeff_modulus_create(n, bits), special)
        return made[name]
    yield get
    for c in made.values():
        c.set_unbiased_moddown(False)


def _lib():
    return PA.load()


def _keys(rng, ctx):
    dnum = -(-ctx.size_Q // ctx.size_P)
    keys = [np.concatenate([O.random_limbs(rng, ctx.n, ctx.moduli) for _ in range(2)]) for _ in range(dnum)]
    return keys, [to_dev(k) for k in keys]


def _sub(a, b, moduli, n):
    q = np.repeat(np.array(moduli, dtype=np.uint64), n)
    q = np.tile(q, a.size // q.size)
    return np.where(a >= b, a - b, a + q - b)


def _assert_constant(got, want, moduli, n, k):
    """got - want (NTT form, [polys][L][n]) is the constant polynomial k in every limb"""
    L = len(moduli)
    diff = _sub(got, want, moduli, n)
    for p in range(got.size // (L * n)):
        coeffs = O.ntt_inv(diff[p * L * n:(p + 1) * L * n], n, moduli)
        assert np.all(coeffs == k), (p, np.unique(coeffs)[:8])


def _moddown(ctx, chain, cx):
    ql, p = ctx.ql(chain), ctx.moduli[ctx.size_Q:]
    d = to_dev(cx)
    dout = to_dev(np.zeros(len(ql) * ctx.n, dtype=np.uint64))
    PA.check(_lib().phantom_moddown_from_ntt(ctx.handle, chain, ptr(d), ptr(dout), stream()))
    return to_host(dout)


@pytest.mark.parametrize("shape,chain", [("p3", 1), ("p3", 5), ("p4", 1), ("p4", 6), ("c3", 30)])
def test_unbiased_moddown(contexts, rng, shape, chain):
    ctx = contexts(shape)
    ql, p = ctx.ql(chain), ctx.moduli[ctx.size_Q:]
    cx = O.random_limbs(rng, ctx.n, ql + p)
    want = np.zeros(len(ql) * ctx.n, dtype=np.uint64)
    O.lib().or_moddown_from_ntt(O.P(cx.copy()), O.P(want), ctx.n, O.P(O.arr(ql)), len(ql), O.P(O.arr(p)), len(p))
    ctx.set_unbiased_moddown(True)
    try:
        got = _moddown(ctx, chain, cx)
    finally:
        ctx.set_unbiased_moddown(False)
    _assert_constant(got, want, ql, ctx.n, ctx.size_P // 2)
    assert np.array_equal(_moddown(ctx, chain, cx), want)  # off again: the reference's bits


@pytest.mark.parametrize("shape,chain", [("p3", 1), ("p4", 2), ("c3", 1)])
def test_unbiased_moddown_rescale(contexts, rng, shape, chain):
    ctx = contexts(shape)
    ql, p = ctx.ql(chain), ctx.moduli[ctx.size_Q:]
    cxs = [O.random_limbs(rng, ctx.n, ql + p) for _ in range(2)]
    want = []
    for cx in cxs:
        w = np.zeros((len(ql) - 1) * ctx.n, dtype=np.uint64)
        O.lib().or_moddown_from_ntt(O.P(cx.copy()), O.P(w), ctx.n, O.P(O.arr(ql[:-1])), len(ql) - 1,
                                    O.P(O.arr([ql[-1]] + list(p))), len(p) + 1)
        want.append(w)
    d = to_dev(np.concatenate(cxs))
    dout = to_dev(np.zeros(2 * (len(ql) - 1) * ctx.n, dtype=np.uint64))
    ctx.set_unbiased_moddown(True)
    try:
        PA.check(_lib().phantom_moddown_rescale(ctx.handle, chain, ptr(d), ptr(dout), 2, stream()))
    finally:
        ctx.set_unbiased_moddown(False)
    _assert_constant(to_host(dout), np.concatenate(want), ql[:-1], ctx.n, (ctx.size_P + 1) // 2)


@pytest.mark.parametrize("shape,chain", [("p3", 2), ("p4", 1)])
def test_unbiased_moddown_modup(contexts, rng, shape, chain):
    """the giant steps' coefficient-domain form: modup(moddown(cx) + k)"""
    ctx = contexts(shape)
    ql, p = ctx.ql(chain), ctx.moduli[ctx.size_Q:]
    n, beta = ctx.n, -(-len(ql) // ctx.size_P)
    cx = O.random_limbs(rng, n, ql + p)
    down = np.zeros(len(ql) * n, dtype=np.uint64)
    O.lib().or_moddown_from_ntt(O.P(cx.copy()), O.P(down), n, O.P(O.arr(ql)), len(ql), O.P(O.arr(p)), len(p))
    const = O.ntt_fwd(np.full(len(ql) * n, ctx.size_P // 2, dtype=np.uint64), n, ql)
    down = np.where(down + const >= np.repeat(np.array(ql, dtype=np.uint64), n),
                    down + const - np.repeat(np.array(ql, dtype=np.uint64), n), down + const)
    want = np.zeros(beta * (len(ql) + len(p)) * n, dtype=np.uint64)
    O.lib().or_modup(O.P(down), O.P(want), n, O.P(O.arr(ql)), len(ql), O.P(O.arr(p)), len(p))
    d = to_dev(cx)
    dout = to_dev(np.zeros(beta * (len(ql) + len(p)) * n, dtype=np.uint64))
    ctx.set_unbiased_moddown(True)
    try:
        PA.check(_lib().phantom_moddown_modup(ctx.handle, chain, ptr(d), ptr(dout), stream()))
    finally:
        ctx.set_unbiased_moddown(False)
    assert np.array_equal(to_host(dout), want)


@pytest.mark.parametrize("shape,chain", [("p3", 1), ("p4", 3)])
def test_unbiased_key_switch_forms(contexts, rng, shape, chain):
    """the fused key-switch forms (inner product in the INTT prologue and the finish epilogue):
    relinearize (moddown, k = floor(size_P / 2)), relinearize + rescale and its batched form with
    per-product outputs (k = floor((size_P + 1) / 2))"""
    ctx = contexts(shape)
    ql = ctx.ql(chain)
    L, n = len(ql), ctx.n
    keys, dkeys = _keys(rng, ctx)
    kp = PA.ptr_array([ptr(k) for k in dkeys])
    cts = [np.concatenate([O.random_limbs(rng, n, ql) for _ in range(3)]) for _ in range(3)]
    want_relin = cts[0].copy()
    O.lib().or_relinearize(O.P(want_relin), n, L, ctx.size_Q, ctx.size_P, (O.u64p * len(keys))(*[O.P(k) for k in keys]),
                           O.P(O.arr(ctx.moduli)))
    want_rr = [KO.relinearize_rescale(ctx, chain, ct, keys) for ct in cts]
    d_relin = to_dev(cts[0])
    d_rr = to_dev(cts[1])
    dout = to_dev(np.zeros(2 * (L - 1) * n, dtype=np.uint64))
    s_in, s_out = 3 * L * n, 2 * (L - 1) * n
    d_batch = to_dev(np.concatenate(cts))
    dout_b = to_dev(np.zeros(3 * s_out, dtype=np.uint64))
    ctx.set_unbiased_moddown(True)
    try:
        PA.check(_lib().phantom_relinearize(ctx.handle, chain, ptr(d_relin), kp, len(dkeys), stream()))
        PA.check(_lib().phantom_relinearize_rescale(ctx.handle, chain, ptr(d_rr), ptr(dout), kp, len(dkeys), stream()))
        PA.check(_lib().phantom_relinearize_rescale_batch(ctx.handle, chain, ptr(d_batch), s_in, 3, ptr(dout_b), s_out,
                                                          kp, len(dkeys), stream()))
    finally:
        ctx.set_unbiased_moddown(False)
    _assert_constant(to_host(d_relin)[:2 * L * n], want_relin[:2 * L * n], ql, n, ctx.size_P // 2)
    k_r = (ctx.size_P + 1) // 2
    _assert_constant(to_host(dout), want_rr[1], ql[:-1], n, k_r)
    got_b = to_host(dout_b)
    for k in range(3):
        _assert_constant(got_b[k * s_out:(k + 1) * s_out], want_rr[k], ql[:-1], n, k_r)
