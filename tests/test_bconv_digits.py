"""CPU checks of the matrix-core base conversion's arithmetic (csrc/rns.hip bconv_mfma_kernel,
rns.h bconv_mfma_tables), emulated in numpy: signed base-256 digits, the 8 exact int8 products
T_b, the int32 pair bounds, and the reassembly (low 64 bits + FP32 nearest-quotient estimate +
one conditional add), checked against exact modular arithmetic (Python integers) on random and
extreme inputs.  The GPU kernel itself is checked bit-exactly in tests/test_gpu_bconv.py."""
import numpy as np
import pytest

import oracle_lib as O

K80 = 0x8080808080808080
M64 = (1 << 64) - 1


def signed_digits(t):
    """the kernel's (t + 0x80..80) ^ 0x80..80, read as 8 int8 digits (little endian)"""
    u = ((t + K80) & M64) ^ K80
    return [((u >> (8 * a)) & 0xFF) - (256 if (u >> (8 * a)) & 0x80 else 0) for a in range(8)]


@pytest.mark.parametrize("t", [0, 1, 127, 128, 255, 256, (1 << 61) - 1, (1 << 60) + 12345, 0x7F7F7F7F7F7F7F])
def test_signed_digits_identity(t):
    d = signed_digits(t)
    assert all(-128 <= x <= 127 for x in d)
    assert sum(x * 256 ** a for a, x in enumerate(d)) == t


def test_signed_digits_random():
    rng = np.random.default_rng(7)
    for t in rng.integers(0, 1 << 61, size=2000, dtype=np.uint64):
        t = int(t)
        assert sum(x * 256 ** a for a, x in enumerate(signed_digits(t))) == t


def f32(x):
    return np.float32(x)


def fmaf(a, b, c):
    # a * b is exact in float64 (24 + 24 bits); one rounding to float32 as the hardware's fmaf
    return np.float32(np.float64(a) * np.float64(b) + np.float64(c))


def emulate(x, ibase, obase):
    """x: [ib][n] residues; returns [ob][n] as the kernel computes it (prescaled inputs)"""
    ib, ob, n = len(ibase), len(obase), x.shape[1]
    qhat = []
    for i in range(ib):
        row = []
        for j in range(ob):
            pr = 1
            for k in range(ib):
                if k != i:
                    pr = pr * ibase[k] % obase[j]
            row.append(pr)
        qhat.append(row)
    # constants m_{s,a,j} = c_sj 256^a mod p_j as signed digits e_b: E[b][j][(s, a)]
    E = np.zeros((8, ob, ib * 8), dtype=np.int64)
    for s in range(ib):
        for a in range(8):
            for j in range(ob):
                m = qhat[s][j] * 256 ** a % obase[j]
                for b, e in enumerate(signed_digits(m)):
                    E[b, j, s * 8 + a] = e
    D = np.zeros((ib * 8, n), dtype=np.int64)
    for s in range(ib):
        for k in range(n):
            D[s * 8:(s + 1) * 8, k] = signed_digits(int(x[s, k]))
    T = np.einsum("bjk,kn->bjn", E, D)  # exact int64 here; the kernel's int32 must hold it
    assert np.abs(T).max() <= 128 * 8 * ib * 128, "T_b bound"
    assert np.abs(T).max() < 2 ** 21 + 1
    out = np.zeros((ob, n), dtype=np.uint64)
    for j in range(ob):
        p = obase[j]
        inv = 1.0 / p
        fx, fy, fz, fw = f32(inv * 2.0 ** 48), f32(inv * 2.0 ** 32), f32(inv * 2.0 ** 16), f32(inv)
        for k in range(n):
            t = [int(T[b, j, k]) for b in range(8)]
            lo_a, lo_b = t[0] + 256 * t[1], t[2] + 256 * t[3]
            hi_a, hi_b = t[4] + 256 * t[5], t[6] + 256 * t[7]
            for v in (lo_a, lo_b, hi_a, hi_b):
                assert -(1 << 31) <= v < (1 << 31), "int32 pair"
            y_exact = lo_a + (lo_b << 16) + (hi_a << 32) + (hi_b << 48)
            L = y_exact & M64
            est = fmaf(f32(hi_b), fx, fmaf(f32(hi_a), fy, fmaf(f32(lo_b), fz, np.float32(f32(lo_a) * fw))))
            qt = int(np.rint(est))
            assert abs(y_exact / p - qt) < 0.5 + 2 ** -6, "quotient estimate"
            y = (L - qt * p) & M64
            if y >= 1 << 63:
                y = (y + p) & M64
            out[j, k] = y
    return out


SHAPES = [
    ([50] * 15, [50] * 6),       # C3 digit
    ([59] * 10, [60] * 4),       # C4
    ([61] * 4, [30] * 5),        # 61-bit inputs, 30-bit outputs
    ([30, 31], [61] * 3),        # small inputs, 61-bit outputs
    ([60] * 16, [60] * 2),       # the largest ibase
]


@pytest.mark.parametrize("ib_bits,ob_bits", SHAPES)
def test_emulated_conversion_matches_exact(ib_bits, ob_bits):
    n = 24
    mods = O.coeff_modulus_create(1024, ib_bits + ob_bits)
    ibase, obase = mods[: len(ib_bits)], mods[len(ib_bits):]
    rng = np.random.default_rng(11)
    x = np.stack([rng.integers(0, q, size=n, dtype=np.uint64) for q in ibase])
    x[:, 0] = [q - 1 for q in ibase]  # extremes
    x[:, 1] = 0
    got = emulate(x, ibase, obase)
    for j, p in enumerate(obase):
        for k in range(n):
            want = 0
            for s, q in enumerate(ibase):
                pr = 1
                for t, qt in enumerate(ibase):
                    if t != s:
                        pr = pr * qt % p
                want += int(x[s, k]) * pr
            assert int(got[j, k]) == want % p
