"""Ciphertext byte format of the reference's PhantomCiphertext::save / load
(include/ciphertext.h:184-225): the header fields written one by one with no padding —
chain_index, size, poly_modulus_degree, coeff_modulus_size (size_t), scale (double),
correction_factor (uint64_t), noiseScaleDeg (size_t), is_ntt_form, is_asymmetric (bool) —
then the words.  The expected bytes are built here with struct from that field list; the
library's serializer (host-only C-ABI) must produce and accept exactly them.  CPU only."""
import ctypes
import struct

import numpy as np
import pytest

import phantom_amd as PA


class Hdr(ctypes.Structure):
    _fields_ = [("chain_index", ctypes.c_uint64), ("size", ctypes.c_uint64),
                ("poly_modulus_degree", ctypes.c_uint64), ("coeff_modulus_size", ctypes.c_uint64),
                ("scale", ctypes.c_double), ("correction_factor", ctypes.c_uint64),
                ("noise_scale_deg", ctypes.c_uint64), ("is_ntt_form", ctypes.c_int), ("is_asymmetric", ctypes.c_int)]


def _reference_bytes(chain, size, n, L, scale, corr, deg, ntt, asym, data):
    return struct.pack("<QQQQdQQ??", chain, size, n, L, scale, corr, deg, ntt, asym) + data.astype("<u8").tobytes()


@pytest.mark.parametrize("ntt,asym", [(True, False), (False, True)])
def test_ciphertext_bytes_match_reference_layout(ntt, asym):
    lib = PA.load()
    rng = np.random.default_rng(7)
    n, L, size = 16, 3, 2
    data = rng.integers(0, 2**60, size=size * L * n, dtype=np.uint64)
    h = Hdr(5, size, n, L, 2.0 ** 40 + 0.25, 1, 2, int(ntt), int(asym))
    want = _reference_bytes(5, size, n, L, 2.0 ** 40 + 0.25, 1, 2, ntt, asym, data)
    assert len(want) == 58 + 8 * data.size
    written = ctypes.c_size_t(0)
    out = (ctypes.c_uint8 * len(want))()
    PA.check(lib.phantom_ciphertext_serialize(ctypes.byref(h), data.ctypes.data, out, len(want), ctypes.byref(written)))
    assert written.value == len(want)
    assert bytes(out) == want

    back = Hdr()
    words = ctypes.c_size_t(0)
    got = np.zeros(data.size, dtype=np.uint64)
    PA.check(lib.phantom_ciphertext_deserialize(want, len(want), ctypes.byref(back), got.ctypes.data, got.size,
                                                 ctypes.byref(words)))
    assert words.value == data.size and np.array_equal(got, data)
    assert (back.chain_index, back.size, back.poly_modulus_degree, back.coeff_modulus_size) == (5, size, n, L)
    assert back.scale == 2.0 ** 40 + 0.25 and back.noise_scale_deg == 2
    assert bool(back.is_ntt_form) == ntt and bool(back.is_asymmetric) == asym


def test_short_buffers_are_rejected():
    lib = PA.load()
    data = np.arange(2 * 2 * 8, dtype=np.uint64)
    h = Hdr(1, 2, 8, 2, 1.0, 1, 1, 1, 0)
    written = ctypes.c_size_t(0)
    small = (ctypes.c_uint8 * 10)()
    assert lib.phantom_ciphertext_serialize(ctypes.byref(h), data.ctypes.data, small, 10, ctypes.byref(written)) != 0
    assert written.value == 58 + 8 * data.size  # the size needed
    blob = _reference_bytes(1, 2, 8, 2, 1.0, 1, 1, True, False, data)
    back, words = Hdr(), ctypes.c_size_t(0)
    # truncated payload
    assert lib.phantom_ciphertext_deserialize(blob[:-1], len(blob) - 1, ctypes.byref(back), None, 0,
                                              ctypes.byref(words)) != 0
    # header only: parse without copying
    PA.check(lib.phantom_ciphertext_deserialize(blob, len(blob), ctypes.byref(back), None, 0, ctypes.byref(words)))
    assert words.value == data.size


def test_galois_key_bytes_match_reference_layout():
    """PhantomGaloisKey::save (include/secretkey.h:195-205): size_t count, then per key a
    PhantomRelinKey record (:130-141): size_t dnum, then dnum PhantomPublicKey records, each the
    key-level ciphertext pk_ (include/ciphertext.h:184-201) — packed here field by field."""
    import ctypes
    import struct

    import numpy as np

    import phantom_amd as PA
    n, qp, dnum, count = 16, 3, 2, 3
    rng = np.random.default_rng(9)
    keys = rng.integers(0, 2**60, size=count * dnum * 2 * qp * n, dtype=np.uint64)
    want = struct.pack("<Q", count)
    for k in range(count):
        want += struct.pack("<Q", dnum)
        for d in range(dnum):
            want += struct.pack("<QQQQdQQ??", 0, 2, n, qp, 1.0, 1, 1, True, False)
            off = (k * dnum + d) * 2 * qp * n
            want += keys[off: off + 2 * qp * n].tobytes()
    lib = PA.load()
    written = ctypes.c_size_t(0)
    out = (ctypes.c_uint8 * len(want))()
    PA.check(lib.phantom_galois_key_serialize(n, qp, dnum, count, keys.ctypes.data, out, len(want),
                                              ctypes.byref(written)))
    assert written.value == len(want) and bytes(out) == want
    # a short buffer reports the size and fails
    small = (ctypes.c_uint8 * 8)()
    assert lib.phantom_galois_key_serialize(n, qp, dnum, count, keys.ctypes.data, small, 8, ctypes.byref(written)) != 0
    assert written.value == len(want)
