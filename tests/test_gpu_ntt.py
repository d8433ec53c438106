"""GPU parity of the NTT launchers against the CPU oracle (bit-exact), through the C-ABI."""
import numpy as np
import pytest

import oracle_lib as O
import phantom_amd as PA
from gpu_util import ptr, stream, to_dev, to_host

pytestmark = pytest.mark.gpu

C3_BITS = [60] + [50] * 44 + [60] * 15


@pytest.fixture(scope="module")
def c3():
    n = 1 << 16
    mods = O.coeff_modulus_create(n, C3_BITS)
    return n, mods, PA.NttTables(n, mods)


def _fwd(tables, d, L, start=0):
    PA.check(PA.load().phantom_nwt_forward_inplace(ptr(d), tables.handle, L, start, stream()))


def _inv(tables, d, L, start=0):
    PA.check(PA.load().phantom_nwt_backward_inplace(ptr(d), tables.handle, L, start, stream()))


def test_c1_ntt_4096_single_prime(rng):
    # config 1: test/ntt_test.cu at N = 4096, one 50-bit prime; constant-2 and uniform inputs
    n = 4096
    mods = O.coeff_modulus_create(n, [50])
    t = PA.NttTables(n, mods)
    for a in (np.full(n, 2, dtype=np.uint64), O.random_limbs(rng, n, mods)):
        d = to_dev(a)
        _fwd(t, d, 1)
        got = to_host(d)
        assert np.array_equal(got, O.ntt_fwd(a, n, mods))
        _inv(t, d, 1)
        assert np.array_equal(to_host(d), a)


@pytest.mark.parametrize("log_n", list(range(8, 18)))
@pytest.mark.parametrize("batch", [1, 10])
def test_ntt_all_degrees(rng, log_n, batch):
    n = 1 << log_n
    mods = O.coeff_modulus_create(n, [50] * (batch - 1) + [60])
    t = PA.NttTables(n, mods)
    a = O.random_limbs(rng, n, mods)
    d = to_dev(a)
    _fwd(t, d, batch)
    f = to_host(d)
    assert np.array_equal(f, O.ntt_fwd(a, n, mods))
    _inv(t, d, batch)
    assert np.array_equal(to_host(d), a)
    # inverse of arbitrary canonical data matches the oracle's inverse
    d2 = to_dev(a)
    _inv(t, d2, batch)
    assert np.array_equal(to_host(d2), O.ntt_inv(a, n, mods))


def test_c2_forward_inverse_n65536_l44(rng, c3):
    # config 2: N = 2^16, limbs 0..43 of the C3 chain, uniform mt-style inputs
    n, mods, t = c3
    L = 44
    a = O.random_limbs(rng, n, mods[:L])
    d = to_dev(a)
    _fwd(t, d, L)
    f = to_host(d)
    assert np.array_equal(f, O.ntt_fwd(a, n, mods[:L]))
    _inv(t, d, L)
    assert np.array_equal(to_host(d), a)


def test_c2_batches_on_three_streams(rng, c3):
    """bench.py's C2 stepping: independent [44][65536] batches dealt round-robin to 3 HIP streams
    (the tables shared). Every batch's forward equals the oracle's and its inverse restores it."""
    import torch
    n, mods, t = c3
    L = 44
    lib = PA.load()
    batches = [O.random_limbs(rng, n, mods[:L]) for _ in range(6)]
    devs = [to_dev(a) for a in batches]
    streams = [torch.cuda.Stream() for _ in range(3)]
    cur = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(cur)
    for i, d in enumerate(devs):
        PA.check(lib.phantom_nwt_forward_inplace(ptr(d), t.handle, L, 0, streams[i % 3].cuda_stream))
    torch.cuda.synchronize()
    for a, d in zip(batches[:2], devs[:2]):  # the oracle's forward is slow: two of them
        assert np.array_equal(to_host(d), O.ntt_fwd(a, n, mods[:L]))
    for i, d in enumerate(devs):
        PA.check(lib.phantom_nwt_backward_inplace(ptr(d), t.handle, L, 0, streams[i % 3].cuda_stream))
    torch.cuda.synchronize()
    for a, d in zip(batches, devs):
        assert np.array_equal(to_host(d), a)


def test_start_modulus_idx_offsets_data_and_tables(rng, c3):
    n, mods, t = c3
    L, start = 5, 40
    a = O.random_limbs(rng, n, mods[:start + L])
    d = to_dev(a)
    _fwd(t, d, L, start)
    got = to_host(d)
    assert np.array_equal(got[:start * n], a[:start * n])
    assert np.array_equal(got[start * n:], O.ntt_fwd(a[start * n:], n, mods[start:start + L]))


def test_backward_scale_and_out_of_place(rng, c3):
    n, mods, t = c3
    L = 15
    a = O.random_limbs(rng, n, mods[:L])
    scale = [int(x) % q for x, q in zip(rng.integers(1, 2 ** 62, L), mods[:L])]
    shoup = [(s << 64) // q for s, q in zip(scale, mods[:L])]
    din, dout = to_dev(a), to_dev(np.zeros_like(a))
    ds, dss = to_dev(O.arr(scale)), to_dev(O.arr(shoup))
    PA.check(PA.load().phantom_nwt_backward_scale(ptr(dout), ptr(din), t.handle, L, 0, ptr(ds), ptr(dss), stream()))
    want = O.ntt_inv(a, n, mods[:L])
    for l in range(L):
        want[l * n:(l + 1) * n] = (want[l * n:(l + 1) * n].astype(object) * scale[l] % mods[l]).astype(np.uint64)
    assert np.array_equal(to_host(dout), want)
    assert np.array_equal(to_host(din), a)


def test_special_mod_exclude_range(rng, c3):
    # modup's NTT over a QlP buffer: Ql limbs then the P limbs, skipping the digit's own limbs
    n, mods, t = c3
    size_QP, size_P, size_Ql = 60, 15, 20
    qlp = mods[:size_Ql] + mods[size_QP - size_P:]
    a = O.random_limbs(rng, n, qlp)
    d = to_dev(a)
    PA.check(PA.load().phantom_nwt_forward_include_special_mod_exclude_range(
        ptr(d), t.handle, size_Ql + size_P, 0, size_QP, size_P, 15, 20, stream()))
    got = to_host(d)
    for i, q in enumerate(qlp):
        sl = slice(i * n, (i + 1) * n)
        want = a[sl] if 15 <= i < 20 else O.ntt_fwd(a[sl], n, [q])
        assert np.array_equal(got[sl], want), i
    # inverse on the P part only (moddown_from_NTT, rns_bconv.cu:804-807)
    d = to_dev(got)
    PA.check(PA.load().phantom_nwt_backward_inplace_include_special_mod(
        ptr(d), t.handle, size_P, size_Ql, size_QP, size_P, stream()))
    back = to_host(d)
    for i, q in enumerate(qlp):
        sl = slice(i * n, (i + 1) * n)
        want = got[sl] if i < size_Ql else O.ntt_inv(got[sl], n, [q])
        assert np.array_equal(back[sl], want), i


def test_invalid_exclude_range_is_rejected(c3):
    n, mods, t = c3
    import torch
    d = torch.zeros(4 * n, dtype=torch.int64, device="cuda")
    rc = PA.load().phantom_nwt_forward_include_special_mod_exclude_range(
        ptr(d), t.handle, 4, 2, 60, 1, 0, 3, stream())
    assert rc == 1 and b"Excluded range" in PA.load().phantom_last_error()


@pytest.mark.parametrize("log_n", [8, 9, 10, 11])
@pytest.mark.parametrize("batch", [1, 10])
def test_nwt_1d(rng, log_n, batch):
    """test/ntt_test.cu test_nwt_1d (:7-69): fnwt_1d / inwt_1d at n = 2^8 .. 2^11 with 50-bit primes,
    the reference's constant-1 input and uniform inputs: INTT(NTT(x)) = x, and both directions
    bit-exact against the oracle."""
    n = 1 << log_n
    mods = O.coeff_modulus_create(n, [50] * batch)
    t = PA.NttTables(n, mods)
    lib = PA.load()
    for a in (np.ones(batch * n, dtype=np.uint64), O.random_limbs(rng, n, mods)):
        d = to_dev(a)
        PA.check(lib.phantom_fnwt_1d(ptr(d), t.handle, batch, 0, stream()))
        assert np.array_equal(to_host(d), O.ntt_fwd(a, n, mods))
        PA.check(lib.phantom_inwt_1d(ptr(d), t.handle, batch, 0, None, None, stream()))
        assert np.array_equal(to_host(d), a)
    t.close()


def test_backward_inplace_scale(rng, c3):
    n, mods, t = c3
    L = 7
    a = O.random_limbs(rng, n, mods[:L])
    scale = [int(x) % q for x, q in zip(rng.integers(1, 2 ** 62, L), mods[:L])]
    shoup = [(s << 64) // q for s, q in zip(scale, mods[:L])]
    d = to_dev(a)
    ds, dss = to_dev(O.arr(scale)), to_dev(O.arr(shoup))
    PA.check(PA.load().phantom_nwt_backward_inplace_scale(ptr(d), t.handle, L, 0, ptr(ds), ptr(dss), stream()))
    want = O.ntt_inv(a, n, mods[:L])
    for l in range(L):
        want[l * n:(l + 1) * n] = (want[l * n:(l + 1) * n].astype(object) * scale[l] % mods[l]).astype(np.uint64)
    assert np.array_equal(to_host(d), want)


def test_forward_include_special_mod(rng, c3):
    n, mods, t = c3
    size_QP, size_P, size_Ql = 60, 15, 9
    qlp = mods[:size_Ql] + mods[size_QP - size_P:]
    a = O.random_limbs(rng, n, qlp)
    d = to_dev(a)
    PA.check(PA.load().phantom_nwt_forward_include_special_mod(ptr(d), t.handle, size_Ql + size_P, 0, size_QP,
                                                               size_P, stream()))
    got = to_host(d)
    for i, q in enumerate(qlp):
        sl = slice(i * n, (i + 1) * n)
        assert np.array_equal(got[sl], O.ntt_fwd(a[sl], n, [q])), i


def test_forward_fuse_moddown(rng, c3):
    """nwt_2d_radix8_forward_inplace_fuse_moddown: ct = (cx - NTT(delta)) * P^-1 per limb."""
    n, mods, t = c3
    L = 12
    cx = O.random_limbs(rng, n, mods[:L])
    delta = O.random_limbs(rng, n, mods[:L])
    pinv = [int(x) % q for x, q in zip(rng.integers(1, 2 ** 62, L), mods[:L])]
    pinvs = [(s << 64) // q for s, q in zip(pinv, mods[:L])]
    dct, dcx, ddl = to_dev(np.zeros_like(cx)), to_dev(cx), to_dev(delta)
    dp, dps = to_dev(O.arr(pinv)), to_dev(O.arr(pinvs))
    PA.check(PA.load().phantom_nwt_forward_fuse_moddown(ptr(dct), ptr(dcx), ptr(dp), ptr(dps), ptr(ddl), t.handle, L,
                                                        0, stream()))
    nd = O.ntt_fwd(delta, n, mods[:L])
    want = np.zeros_like(cx)
    for l, q in enumerate(mods[:L]):
        sl = slice(l * n, (l + 1) * n)
        diff = (cx[sl].astype(object) - nd[sl].astype(object)) % q
        want[sl] = (diff * pinv[l] % q).astype(np.uint64)
    assert np.array_equal(to_host(dct), want)


@pytest.mark.parametrize("limbs,bits", [(264, 59), (256, 60)])
def test_ntt_large_integer_batches(rng, limbs, bits):
    """a C5-sized launch (a lockstep group's 256-480 limbs) of integer-only limbs below 2^60 (the
    IO kernels), in place: forward, inverse of the result, and inverse of arbitrary canonical data
    == the oracle (a one-workgroup-per-limb kernel, round 6, passed this and was slower: removed,
    profiles/r06/ntt_limb/)"""
    n = 1 << 16
    mods = O.coeff_modulus_create(n, [bits] * limbs)
    t = PA.NttTables(n, mods)
    a = O.random_limbs(rng, n, mods)
    d = to_dev(a)
    _fwd(t, d, limbs)
    assert np.array_equal(to_host(d), O.ntt_fwd(a, n, mods))
    _inv(t, d, limbs)
    assert np.array_equal(to_host(d), a)
    d2 = to_dev(a)
    _inv(t, d2, limbs)
    assert np.array_equal(to_host(d2), O.ntt_inv(a, n, mods))
