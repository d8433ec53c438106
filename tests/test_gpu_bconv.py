"""GPU parity of the fast base conversion (DBaseConverter::bConv_BEHZ, src/rns_bconv.cu:212-229)
through phantom_fast_bconv, bit-exact against the oracle's or_bconv, over the shapes that pick
the matrix-core kernel's variants (ksteps KT = ceil(ibase / 8), row blocks NJB = ceil(obase / 16)),
prime sizes from 30 to 61 bits, and the shapes that fall back to the 30-bit-split kernel
(ibase > 16, obase > 64, n not a multiple of 16).  The output buffer carries a sentinel row past
obase: a write outside [obase][n] fails the test."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
import phantom_amd as PA
from gpu_util import ptr, stream, to_dev, to_host

pytestmark = pytest.mark.gpu

SENTINEL = np.uint64(0xDEADBEEFCAFEF00D)

# (n, ibase prime bits, obase prime bits)
SHAPES = [
    (4096, [50] * 15, [50] * 45),          # C3 digit: KT 2, NJB 3
    (1 << 16, [59] * 10, [60] * 30),       # C4 digit / moddown: KT 2, NJB 2
    (4096, [60] * 16, [60] * 64),          # largest matrix-core shape: KT 2, NJB 4
    (4096, [30, 31, 32], [59] * 10),       # small input primes: KT 1, NJB 1
    (2048, [61] * 9, [30] * 17),           # 61-bit inputs, small outputs: KT 2, NJB 2
    (16, [40] * 8, [45] * 16),             # one tile, exact block sizes
    (4096, [50], [50] * 44),               # one input limb (a short last digit)
    (4096, [50] * 20, [50] * 30),          # ibase > 16: 30-bit-split fallback
    (1024, [50] * 5, [55] * 70),           # obase > 64: fallback
    (8, [50] * 4, [50] * 6),               # n not a multiple of 16: fallback
]


def _moduli(n, ib_bits, ob_bits):
    # distinct primes = 1 mod 2n for both bases (the chain generator never repeats a prime)
    mods = O.coeff_modulus_create(max(n, 1024), ib_bits + ob_bits)
    return mods[: len(ib_bits)], mods[len(ib_bits):]


@pytest.mark.parametrize("prescale", [1, 0])
@pytest.mark.parametrize("n,ib_bits,ob_bits", SHAPES)
def test_fast_bconv_matches_oracle(rng, n, ib_bits, ob_bits, prescale):
    ibase, obase = _moduli(n, ib_bits, ob_bits)
    x = O.random_limbs(rng, n, ibase)
    # oracle: or_bconv prescales; for prescale = 0 feed it inputs whose [x qHat^-1] is x itself
    ib_arr = np.array(ibase, dtype=np.uint64)
    ob_arr = np.array(obase, dtype=np.uint64)
    if prescale:
        x_oracle = x
    else:
        # or_bconv prescales by qHat_i^-1: hand it x_i qHat_i so the prescale gives back x_i
        qhat = []
        for i, q in enumerate(ibase):
            prod = 1
            for k, qk in enumerate(ibase):
                if k != i:
                    prod = prod * qk % q
            qhat.append(prod)
        sc = np.array(qhat, dtype=np.uint64)
        x_oracle = np.zeros_like(x)
        O.lib().or_poly_mul_scalar(O.P(x), O.P(sc), O.P(x_oracle), n, len(ibase), O.P(ib_arr))
    want = np.zeros(len(obase) * n, dtype=np.uint64)
    O.lib().or_bconv(O.P(x_oracle), O.P(want), n, O.P(ib_arr), len(ibase), O.P(ob_arr), len(obase))
    d_in = to_dev(x)
    d_out = to_dev(np.full((len(obase) + 1) * n, SENTINEL, dtype=np.uint64))
    lib = PA.load()
    PA.check(lib.phantom_fast_bconv(ib_arr.ctypes.data_as(PA.u64p), len(ibase), ob_arr.ctypes.data_as(PA.u64p),
                                    len(obase), ptr(d_in), ptr(d_out), n, prescale, stream()))
    got = to_host(d_out)
    assert np.all(got[len(obase) * n:] == SENTINEL), "write past obase"
    assert np.array_equal(got[: len(obase) * n], want)

    # the same conversion through a kept converter (phantom_bconv_create / _run), run twice on
    # one handle: the tables are built once and reused
    h = PA.vp()
    PA.check(lib.phantom_bconv_create(ib_arr.ctypes.data_as(PA.u64p), len(ibase), ob_arr.ctypes.data_as(PA.u64p),
                                      len(obase), stream(), ctypes.byref(h)))
    try:
        for _ in range(2):
            d_out2 = to_dev(np.full((len(obase) + 1) * n, SENTINEL, dtype=np.uint64))
            PA.check(lib.phantom_bconv_run(h, ptr(d_in), ptr(d_out2), n, prescale, stream()))
            got2 = to_host(d_out2)
            assert np.all(got2[len(obase) * n:] == SENTINEL), "write past obase"
            assert np.array_equal(got2[: len(obase) * n], want)
    finally:
        PA.check(lib.phantom_bconv_destroy(h))


def test_fast_bconv_rejects_empty():
    lib = PA.load()
    one = np.array([65537], dtype=np.uint64)
    rc = lib.phantom_fast_bconv(one.ctypes.data_as(PA.u64p), 0, one.ctypes.data_as(PA.u64p), 1, None, None, 16, 1,
                                stream())
    assert rc != 0
    assert lib.phantom_bconv_run(None, None, None, 16, 1, stream()) != 0
    h = PA.vp()
    assert lib.phantom_bconv_create(one.ctypes.data_as(PA.u64p), 0, one.ctypes.data_as(PA.u64p), 1, stream(),
                                    ctypes.byref(h)) != 0
