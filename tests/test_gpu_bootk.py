"""Bit-exact GPU parity of every integer kernel the bootstrap launches, at config C4's size
(N = 2^16, Q = {60, 29 x 59}, P = 10 x 60: bootstrapping_example.cu:69-116), through the C-ABI,
against the CPU oracle (oracle/oracle.c, which restates the reference functions named below):

  lt_bsgs            EvalMultExt + EvalAddExtInPlace inner sums (bootstrap.cu:1322-1332)
  keyswitch_ext      KeySwitchExt (evaluate.cu:3876-3940)
  fast_rotation_ext  EvalFastRotationExt + its fused P c0 / automorphism epilogue (evaluate.cu:3660-3755)
  rotate_ext_acc     a giant step: moddown + modup + inner product + automorphism + accumulate
  tensor_lin         tensor product with MulAddRescale's linear epilogue
  lin_comb / mul_scalar / leaf_combine   EvalMultConst / EvalLinearWSumMutable forms (evaluate.cu:2299-3600)
  automorphism, ModRaise lift at 40 / 30 limbs; the NTT tables against the oracle's tables.

Operands are uniform random residues (parity is a property of the arithmetic, not of key or
ciphertext structure)."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
import phantom_amd as PA
from gpu_util import ptr, stream, to_dev, to_host

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


def _keys(rng, ctx):
    dnum = -(-ctx.size_Q // ctx.size_P)
    keys = [_rand(rng, ctx.moduli, 2) for _ in range(dnum)]
    return keys, [to_dev(k) for k in keys]


def _vp(ts):
    return PA.ptr_array([ptr(t) for t in ts])


@pytest.mark.parametrize("chain,g,b", [(1, 16, 4), (17, 8, 8), (3, 32, 8), (17, 32, 5)])
def test_lt_bsgs(c4, rng, chain, g, b):
    em = _ext_mods(c4, chain)
    babies = [_rand(rng, em, 2) for _ in range(g)]
    pts = [_rand(rng, em) for _ in range(g * b)]
    pts[3] = np.zeros_like(pts[3])  # an absent diagonal reads the zero plaintext
    db, dp = [to_dev(x) for x in babies], [to_dev(x) for x in pts]
    douts = [to_dev(np.zeros(2 * len(em) * N, dtype=np.uint64)) for _ in range(b)]
    PA.check(_lib().phantom_lt_bsgs(c4.handle, chain, _vp(db), g, _vp(dp), b, _vp(douts), stream()))
    want = [np.zeros(2 * len(em) * N, dtype=np.uint64) for _ in range(b)]
    O.lib().or_lt_bsgs(O.ptrs(babies), g, O.ptrs(pts), b, O.ptrs(want), N, len(c4.ql(chain)), c4.size_Q, c4.size_P,
                       O.P(O.arr(c4.moduli)))
    for i in range(b):
        assert np.array_equal(to_host(douts[i]), want[i]), i


@pytest.mark.parametrize("bits,g,b", [(61, 32, 8), (61, 16, 4), (61, 32, 3), (59, 32, 8)])
def test_lt_bsgs_moduli(rng, bits, g, b):
    """the inner sums' 30-bit split partial sums at their bounds: N = 4096, 8 + 2 moduli of `bits`
    bits.  61-bit moduli make a high-half product reach 2^62, so the sums fold every 4 products
    (LtArgs::q60 = 0); below 2^60 every 8 (tile kernel) or 16 (lt_bsgs_kernel).  == or_lt_bsgs"""
    n, size_p, chain = 1 << 12, 2, 1
    ctx = PA.Context(n, O.coeff_modulus_create(n, [bits] * 10), size_p)
    em = ctx.ql(chain) + ctx.moduli[ctx.size_Q:]
    rand = lambda polys: np.concatenate([O.random_limbs(rng, n, em) for _ in range(polys)])
    babies = [rand(2) for _ in range(g)]
    pts = [rand(1) for _ in range(g * b)]
    db, dp = [to_dev(x) for x in babies], [to_dev(x) for x in pts]
    douts = [to_dev(np.zeros(2 * len(em) * n, dtype=np.uint64)) for _ in range(b)]
    PA.check(_lib().phantom_lt_bsgs(ctx.handle, chain, _vp(db), g, _vp(dp), b, _vp(douts), stream()))
    want = [np.zeros(2 * len(em) * n, dtype=np.uint64) for _ in range(b)]
    O.lib().or_lt_bsgs(O.ptrs(babies), g, O.ptrs(pts), b, O.ptrs(want), n, len(ctx.ql(chain)), ctx.size_Q,
                       ctx.size_P, O.P(O.arr(ctx.moduli)))
    for i in range(b):
        assert np.array_equal(to_host(douts[i]), want[i]), (bits, i)


@pytest.mark.parametrize("chain", [1, 17])
def test_keyswitch_ext(c4, rng, chain):
    ql = c4.ql(chain)
    ct = _rand(rng, ql, 2)
    dout = to_dev(np.full(2 * (len(ql) + SIZE_P) * N, 7, dtype=np.uint64))
    dct = to_dev(ct)  # every device operand held until the result is read back
    PA.check(_lib().phantom_keyswitch_ext(c4.handle, chain, ptr(dct), ptr(dout), stream()))
    want = np.zeros(2 * (len(ql) + SIZE_P) * N, dtype=np.uint64)
    O.lib().or_keyswitch_ext(O.P(ct), O.P(want), N, len(ql), c4.size_Q, c4.size_P, O.P(O.arr(c4.moduli)))
    assert np.array_equal(to_host(dout), want)


@pytest.mark.parametrize("chain,elt_kind,add_first", [(1, "rot", 1), (1, "conj", 0), (3, "rot", 1)])
def test_fast_rotation_ext(c4, rng, chain, elt_kind, add_first):
    ql = c4.ql(chain)
    em = _ext_mods(c4, chain)
    beta = -(-len(ql) // SIZE_P)
    elt = pow(5, 77, 2 * N) if elt_kind == "rot" else 2 * N - 1
    c0 = _rand(rng, ql)
    digits = _rand(rng, em, beta)
    keys, dkeys = _keys(rng, c4)
    dout = to_dev(np.zeros(2 * len(em) * N, dtype=np.uint64))
    dc0, ddig = to_dev(c0), to_dev(digits)
    PA.check(_lib().phantom_fast_rotation_ext(c4.handle, chain, ptr(dc0), ptr(ddig), _vp(dkeys),
                                              len(dkeys), elt, add_first, ptr(dout), stream()))
    want = np.zeros(2 * len(em) * N, dtype=np.uint64)
    O.lib().or_fast_rotation_ext(O.P(c0), O.P(digits), O.ptrs(keys), elt, add_first, O.P(want), N, len(ql),
                                 c4.size_Q, c4.size_P, O.P(O.arr(c4.moduli)))
    assert np.array_equal(to_host(dout), want)


@pytest.mark.parametrize("shape,chain,count,identity_at", [("c4", 1, 9, 4), ("c4", 3, 4, None), ("c4", 17, 32, 16),
                                                             ("n512", 1, 7, 2), ("q61", 1, 5, 0)])
def test_fast_rotation_ext_batch(c4, rng, shape, chain, count, identity_at):
    """one launch of `count` baby steps == the per-rotation EvalFastRotationExt / KeySwitchExt
    (c4: full 1024-index blocks, beta 3 / 2; n512: the any-size kernel, beta 4; q61: the full
    kernel at N = 4096 with 61-bit moduli and beta 4, the split partial sums' bounds)"""
    if shape == "c4":
        ctx, n, size_p = c4, N, SIZE_P
    elif shape == "q61":
        n, size_p = 1 << 12, 2
        ctx = PA.Context(n, O.coeff_modulus_create(n, [61] * 10), size_p)
    else:
        n, size_p = 512, 2
        ctx = PA.Context(n, O.coeff_modulus_create(n, [50] * 10), size_p)
    ql = ctx.ql(chain)
    em = _ext_mods(ctx, chain)
    beta = -(-len(ql) // size_p)
    rand = lambda mods, polys=1: np.concatenate([O.random_limbs(rng, n, mods) for _ in range(polys)])
    ct = rand(ql, 2)
    digits = rand(em, beta)
    elts = [pow(5, 3 * k + 1, 2 * n) for k in range(count)]
    elts[-1] = 2 * n - 1  # a conjugation among the rotations
    dnum = -(-ctx.size_Q // size_p)
    distinct = []  # host memory: three key sets shared round robin
    for _ in range(3):
        keys = [rand(ctx.moduli, 2) for _ in range(dnum)]
        distinct.append((keys, [to_dev(k) for k in keys]))
    keysets = [distinct[k % 3] for k in range(count)]
    dct, ddig = to_dev(ct), to_dev(digits)
    douts = [to_dev(np.full(2 * len(em) * n, 5, dtype=np.uint64)) for _ in range(count)]
    key_arrays = [None if k == identity_at else _vp(keysets[k][1]) for k in range(count)]
    kk = (ctypes.POINTER(ctypes.c_void_p) * count)(*[ctypes.cast(a, ctypes.POINTER(ctypes.c_void_p)) if a is not None
                                                     else None for a in key_arrays])
    el = (ctypes.c_uint32 * count)(*elts)
    PA.check(_lib().phantom_fast_rotation_ext_batch(ctx.handle, chain, ptr(dct), ptr(ddig), kk, dnum, el, count,
                                                    _vp(douts), stream()))
    mods = O.P(O.arr(ctx.moduli))
    for k in range(count):
        want = np.zeros(2 * len(em) * n, dtype=np.uint64)
        if k == identity_at:
            O.lib().or_keyswitch_ext(O.P(ct), O.P(want), n, len(ql), ctx.size_Q, ctx.size_P, mods)
        else:
            O.lib().or_fast_rotation_ext(O.P(ct), O.P(digits), O.ptrs(keysets[k][0]), elts[k], 1, O.P(want), n,
                                         len(ql), ctx.size_Q, ctx.size_P, mods)
        assert np.array_equal(to_host(douts[k]), want), k


@pytest.mark.parametrize("chain,accumulate", [(2, 0), (2, 1)])
def test_rotate_ext_accumulate(c4, rng, chain, accumulate):
    ql = c4.ql(chain)
    em = _ext_mods(c4, chain)
    ext = _rand(rng, em, 2)
    acc = _rand(rng, em, 2)
    keys, dkeys = _keys(rng, c4)
    elt = pow(5, 1024, 2 * N)
    dext, dacc = to_dev(ext), to_dev(acc)
    PA.check(_lib().phantom_rotate_ext_accumulate(c4.handle, chain, ptr(dext), _vp(dkeys), len(dkeys), elt,
                                                  ptr(dacc), accumulate, stream()))
    want = acc.copy()
    O.lib().or_rotate_ext_accumulate(O.P(ext.copy()), O.ptrs(keys), elt, O.P(want), accumulate, N, len(ql),
                                     c4.size_Q, c4.size_P, O.P(O.arr(c4.moduli)))
    assert np.array_equal(to_host(dacc), want)


@pytest.mark.parametrize("with_f,with_t", [(True, True), (False, True), (True, False), (False, False)])
def test_tensor_lin(c4, rng, with_f, with_t):
    chain = 16
    ql = c4.ql(chain)
    L = len(ql)
    a, b = _rand(rng, ql, 2), _rand(rng, ql, 2)
    tl = c4.ql(chain - 2)  # a term with more limbs than the product (read at its own stride)
    t = _rand(rng, tl, 2)
    f = O.arr([int(x) for x in rng.integers(0, 2 ** 62, size=L, dtype=np.uint64)])
    c = O.arr([int(x) for x in rng.integers(0, 2 ** 62, size=L, dtype=np.uint64)])
    dout = to_dev(np.zeros(3 * L * N, dtype=np.uint64))
    dt, da, dbb = to_dev(t), to_dev(a), to_dev(b)
    PA.check(_lib().phantom_tensor_lin(c4.handle, chain, ptr(da), ptr(dbb), ptr(dout),
                                       f.ctypes.data if with_f else None, ptr(dt) if with_t else None,
                                       len(tl) * N, c.ctypes.data if with_t else None, stream()))
    mods = O.arr(ql)
    fr = O.arr([int(x) % q for x, q in zip(f, ql)])
    cr = O.arr([int(x) % q for x, q in zip(c, ql)])
    want = np.zeros(3 * L * N, dtype=np.uint64)
    O.lib().or_tensor_lin(O.P(a), O.P(b), O.P(want), N, L, O.P(mods), O.P(fr) if with_f else None,
                          O.P(t) if with_t else None, len(tl) * N, O.P(cr) if with_t else None)
    assert np.array_equal(to_host(dout), want)


@pytest.mark.parametrize("chain", [4, 16])
def test_tensor_lin_batch(c4, rng, chain):
    """the EvalMod products' batched tensors (tensor_lin_batch_kernel: 2 elements per thread, the
    factor 2 as a modular doubling) == or_tensor_lin per job: factors 1, 2 and 3, with and without
    a term and a constant"""
    ql = c4.ql(chain)
    L = len(ql)
    mods = O.arr(ql)
    tl = c4.ql(chain - 2)
    jobs = [(1, True, True), (2, True, False), (2, False, True), (3, True, True), (1, False, False), (2, True, True)]
    cnt = len(jobs)
    A = [_rand(rng, ql, 2) for _ in range(cnt)]
    B = [_rand(rng, ql, 2) for _ in range(cnt)]
    T = [_rand(rng, tl, 2) for _ in range(cnt)]
    C = [O.arr([int(x) % q for x, q in zip(rng.integers(0, 2 ** 62, size=L, dtype=np.uint64), ql)]) for _ in range(cnt)]
    K = [O.arr([int(x) % q for x, q in zip(rng.integers(0, 2 ** 62, size=L, dtype=np.uint64), ql)]) for _ in range(cnt)]
    dA, dB, dT = [to_dev(x) for x in A], [to_dev(x) for x in B], [to_dev(x) for x in T]
    dout = [to_dev(np.zeros(3 * L * N, dtype=np.uint64)) for _ in range(cnt)]
    vp = lambda xs: PA.ptr_array(list(xs))
    facs = O.arr([f for f, _, _ in jobs])
    PA.check(_lib().phantom_tensor_lin_batch(
        c4.handle, chain, cnt, vp(ptr(x) for x in dA), vp(ptr(x) for x in dB), vp(ptr(x) for x in dout),
        facs.ctypes.data, vp(ptr(dT[k]) if jobs[k][1] else 0 for k in range(cnt)), len(tl) * N,
        vp(C[k].ctypes.data if jobs[k][1] else 0 for k in range(cnt)),
        vp(K[k].ctypes.data if jobs[k][2] else 0 for k in range(cnt)), stream()))
    for k, (f, with_t, with_c) in enumerate(jobs):
        want = np.zeros(3 * L * N, dtype=np.uint64)
        fr = O.arr([f % q for q in ql])
        O.lib().or_tensor_lin(O.P(A[k]), O.P(B[k]), O.P(want), N, L, O.P(mods), O.P(fr) if f != 1 else None,
                              O.P(T[k]) if with_t else None, len(tl) * N, O.P(C[k]) if with_t else None)
        if with_c:
            w0 = want[:L * N].reshape(L, N)
            for l in range(L):
                w0[l] = (w0[l] + np.uint64(K[k][l])) % np.uint64(ql[l])
        assert np.array_equal(to_host(dout[k]), want), k


def test_lin_comb_and_mul_scalar(c4, rng):
    chain = 20
    ql = c4.ql(chain)
    L = len(ql)
    mods = O.arr(ql)
    d = _rand(rng, ql, 2)
    tl = c4.ql(chain - 3)
    t = _rand(rng, tl, 2)
    ca = O.arr([int(x) % q for x, q in zip(rng.integers(0, 2 ** 62, size=L, dtype=np.uint64), ql)])
    cb = O.arr([int(x) % q for x, q in zip(rng.integers(0, 2 ** 62, size=L, dtype=np.uint64), ql)])
    dd, dtt = to_dev(d), to_dev(t)
    PA.check(_lib().phantom_lin_comb(c4.handle, chain, ptr(dd), 2, ca.ctypes.data, ptr(dtt), 2, len(tl) * N,
                                     cb.ctypes.data, stream()))
    want = d.copy()
    O.lib().or_lin_comb(O.P(want), 2, O.P(ca), O.P(t), 2, len(tl) * N, O.P(cb), N, L, O.P(mods))
    assert np.array_equal(to_host(dd), want)
    # mul_scalar reading the leading L limbs of longer polynomials, accumulating
    acc = _rand(rng, ql, 2)
    dout = to_dev(np.zeros(2 * L * N, dtype=np.uint64))
    dacc = to_dev(acc)
    PA.check(_lib().phantom_mul_scalar(c4.handle, chain, ptr(dtt), len(tl) * N, ca.ctypes.data,
                                       ptr(dacc), ptr(dout), 2, stream()))
    want = np.zeros(2 * L * N, dtype=np.uint64)
    O.lib().or_mul_scalar_acc(O.P(t), len(tl) * N, O.P(ca), O.P(acc), O.P(want), 2, N, L, O.P(mods))
    assert np.array_equal(to_host(dout), want)


@pytest.mark.parametrize("K,M", [(15, 4), (7, 8), (1, 1)])
def test_leaf_combine(c4, rng, K, M):
    chain = 12
    ql = c4.ql(chain)
    L = len(ql)
    ins, strides = [], []
    for k in range(K):
        lk = c4.ql(chain - (k % 3))  # inputs at the product's level or above
        ins.append(_rand(rng, lk, 2))
        strides.append(len(lk) * N)
    coef = O.arr([int(x) % ql[i % L] for i, x in enumerate(rng.integers(0, 2 ** 62, size=M * K * L, dtype=np.uint64))])
    cadd = O.arr([int(x) % ql[i % L] for i, x in enumerate(rng.integers(0, 2 ** 62, size=M * L, dtype=np.uint64))])
    dins = [to_dev(x) for x in ins]
    douts = [to_dev(np.zeros(2 * L * N, dtype=np.uint64)) for _ in range(M)]
    st = (PA.sz * K)(*strides)
    PA.check(_lib().phantom_leaf_combine(c4.handle, chain, _vp(dins), st, K, coef.ctypes.data, cadd.ctypes.data,
                                         _vp(douts), M, stream()))
    want = [np.zeros(2 * L * N, dtype=np.uint64) for _ in range(M)]
    ost = (O.sz * K)(*strides)
    O.lib().or_leaf_combine(O.ptrs(ins), ost, K, O.P(coef), O.P(cadd), O.ptrs(want), M, N, L, O.P(O.arr(ql)))
    for m in range(M):
        assert np.array_equal(to_host(douts[m]), want[m]), m


@pytest.mark.parametrize("elt", [pow(5, 3, 2 * N), pow(5, 16384, 2 * N), 2 * N - 1])
def test_automorphism_c4_size(c4, rng, elt):
    L = 40  # Ql u P at chain 1
    a = _rand(rng, c4.moduli[:L])
    dout = to_dev(np.zeros(L * N, dtype=np.uint64))
    da = to_dev(a)
    PA.check(_lib().phantom_apply_galois_ntt(c4.handle, elt, ptr(da), ptr(dout), L, stream()))
    want = np.zeros(L * N, dtype=np.uint64)
    O.lib().or_apply_galois_ntt(O.P(a), O.P(want), N, L, elt)
    assert np.array_equal(to_host(dout), want)


def test_raise_c4_size(c4, rng):
    q0 = c4.moduli[0]
    L = c4.size_Q
    x = rng.integers(0, q0, size=N, dtype=np.uint64)
    x[:4] = [0, 1, q0 // 2, q0 // 2 + 1]  # both sides of the centered lift
    dout = to_dev(np.zeros(L * N, dtype=np.uint64))
    dx = to_dev(x)
    PA.check(_lib().phantom_switch_modulus_raise(c4.handle, ptr(dx), ptr(dout), L, stream()))
    want = np.zeros(L * N, dtype=np.uint64)
    O.lib().or_switch_modulus_raise(O.P(x), O.P(want), N, q0, O.P(O.arr(c4.moduli[:L])), L)
    assert np.array_equal(to_host(dout), want)


@pytest.mark.parametrize("idx", [0, 1, 29, 30, 39])
def test_ntt_tables_match_oracle(c4, idx):
    """phantom_ntt_tables_host (the device tables, DNTTTable of include/ntt.cuh:36-129) equals the
    oracle's restatement of src/host/ntt.cu:11-56 for C4 primes (60- and 59-bit)."""
    q = c4.moduli[idx]
    t = PA.NttTables(N, [q])
    got = [np.zeros(N, dtype=np.uint64) for _ in range(4)]
    ninv = np.zeros(1, dtype=np.uint64)
    PA.check(_lib().phantom_ntt_tables_host(t.handle, 0, *[g.ctypes.data_as(PA.u64p) for g in got],
                                            ninv.ctypes.data_as(PA.u64p)))
    want, want_ninv = O.ntt_tables(N, q)
    # tw, tw_shoup identical.  itw differs at index 1 only: the reference folds n^-1 into
    # itwiddle[1] (src/host/ntt.cu:53-55) for its last GS stage; this engine's integer INTT
    # multiplies every output by n^-1 instead (csrc/ntt.hip), so it stores psi^(-n/2) there.
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    for g, w in ((got[2], want[2]), (got[3], want[3])):
        assert np.array_equal(np.delete(g, 1), np.delete(w, 1))
    assert O.lib().or_mulmod(int(got[2][1]), want_ninv, q) == int(want[2][1])
    assert int(ninv[0]) == want_ninv
    t.close()


@pytest.mark.parametrize("chain,count", [(4, 2), (12, 4), (20, 2)])
def test_relinearize_rescale_batch_c4(c4, rng, chain, count):
    """EvalMod's batched products at C4 chains (the real and imaginary halves, a ladder
    generation): phantom_relinearize_rescale_batch bit-exact vs the oracle composition per product
    (tests/ks_oracle.py; src/evaluate.cu:1552-1647, src/rns_bconv.cu:530-843)."""
    import ks_oracle as KO
    L = len(c4.ql(chain))
    cts = [_rand(rng, c4.ql(chain), 3) for _ in range(count)]
    keys, dkeys = _keys(rng, c4)
    d = to_dev(np.concatenate(cts))
    s_out = 2 * (L - 1) * N
    dout = to_dev(np.zeros(count * s_out, dtype=np.uint64))
    PA.check(_lib().phantom_relinearize_rescale_batch(c4.handle, chain, ptr(d), 3 * L * N, count, ptr(dout), s_out,
                                                      _vp(dkeys), len(dkeys), stream()))
    got = to_host(dout)
    for k in range(count):
        assert np.array_equal(got[k * s_out:(k + 1) * s_out], KO.relinearize_rescale(c4, chain, cts[k], keys)), k
