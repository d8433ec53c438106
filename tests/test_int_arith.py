"""CPU emulation of the carry-free integer butterflies (phantom-fhe-boot_amd/csrc/arith.h,
PHX_INT_NOCARRY) against the plain forms they replace, in exact 64-bit wrapping arithmetic, at the
C4 chain's 59/60-bit primes and the extreme values of the lazy ranges ([0, 8q) forward,
[0, 4q) inverse).  The butterfly structure follows the reference's include/butterfly.cuh:10-37."""
import random

M64 = (1 << 64) - 1


def hi32(x):
    return x >> 32


def lo32(x):
    return x & 0xFFFFFFFF


def csub(x, m):  # arith.h csub: signed test of x - m
    t = (x - m) & M64
    return x if t >> 63 else t


def csub_n(x, m, nm):  # arith.h csub_n: add of the negated constant, select by sign mask
    t = (x + nm) & M64
    s = 0xFFFFFFFF if hi32(t) >> 31 else 0
    return (t + ((hi32(m) & s) << 32 | (lo32(m) & s))) & M64


def mulhi_approx(a, s):
    a0, a1, s0, s1 = lo32(a), hi32(a), lo32(s), hi32(s)
    return (a1 * s1 + ((a1 * s0) >> 32) + ((a0 * s1) >> 32)) & M64


def shoup_plain(a, w, ws, q):
    return (a * w - mulhi_approx(a, ws) * q) & M64


def shoup_nocarry(a, w, ws, q):
    return (a * w + mulhi_approx(a, ws) * ((-q) & M64)) & M64


def ct_plain(x, y, w, ws, q):
    t = shoup_plain(y, w, ws, q)
    u = csub(x, q << 2)
    return (u + t) & M64, (u + (q << 2) - t) & M64


def ct_nocarry(x, y, w, ws, q):
    q4 = q << 2
    t = shoup_nocarry(y, w, ws, q)
    u = csub_n(x, q4, (-q4) & M64)
    return (u + t) & M64, (u + q4 - t) & M64


def gs_plain(x, y, w, ws, q):
    q4 = q << 2
    d = (x + q4 - y) & M64
    return csub((x + y) & M64, q4), shoup_plain(d, w, ws, q)


def gs_nocarry(x, y, w, ws, q):
    q4 = q << 2
    d = (x + q4 - y) & M64
    return csub_n((x + y) & M64, q4, (-q4) & M64), shoup_nocarry(d, w, ws, q)


def reduce8_nocarry(v, q):
    v = csub_n(v, q << 2, (-(q << 2)) & M64)
    v = csub_n(v, q << 1, (-(q << 1)) & M64)
    return csub_n(v, q, (-q) & M64)


# largest primes of the C4 chain's sizes and the MOD_BIT_COUNT_MAX bound (q < 2^61)
PRIMES = [(1 << 60) - 93, (1 << 59) - 55, (1 << 61) - 1]


def _samples(rng, hi, k):
    return [0, 1, hi - 1, hi // 2] + [rng.randrange(hi) for _ in range(k)]


def test_csub_n_matches_csub():
    rng = random.Random(7)
    for q in PRIMES:
        for m in (q, q << 1, q << 2):
            for x in _samples(rng, 8 * q, 400):
                assert csub_n(x, m, (-m) & M64) == csub(x, m)


def test_butterflies_bit_identical():
    rng = random.Random(11)
    for q in PRIMES:
        for _ in range(300):
            w = rng.randrange(q)
            ws = (w << 64) // q
            x, y = rng.randrange(8 * q), rng.randrange(8 * q)
            assert ct_nocarry(x, y, w, ws, q) == ct_plain(x, y, w, ws, q)
            xi, yi = rng.randrange(4 * q), rng.randrange(4 * q)
            assert gs_nocarry(xi, yi, w, ws, q) == gs_plain(xi, yi, w, ws, q)
        # the lazy-range extremes
        w = q - 1
        ws = (w << 64) // q
        for x in (0, 8 * q - 1):
            for y in (0, 8 * q - 1):
                assert ct_nocarry(x, y, w, ws, q) == ct_plain(x, y, w, ws, q)
                r = ct_nocarry(x, y, w, ws, q)
                assert r[0] < 8 * q and r[1] < 8 * q
                assert (r[0] - r[1] - 2 * y * w) % q == 0 and (r[0] + r[1] - 2 * x) % q == 0


def test_reduce8_canonical():
    rng = random.Random(13)
    for q in PRIMES:
        for v in _samples(rng, 8 * q, 400):
            assert reduce8_nocarry(v, q) == v % q
