"""C-ABI boundary checks that need no GPU: the library loads, exports every symbol
include/phantom_amd.h declares, and its host-side parameter generation matches the oracle."""
import ctypes

import pytest

import oracle_lib as O
import phantom_amd as PA


def test_library_loads_and_reports_version():
    lib = PA.load()
    assert b"gfx950" in lib.phantom_version()


def test_every_declared_symbol_is_exported():
    lib = PA.load()
    names = PA.declared_symbols()
    assert len(names) >= 10
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_status_strings():
    lib = PA.load()
    assert lib.phantom_status_string(0) == b"ok"
    assert lib.phantom_status_string(1) == b"invalid argument"


@pytest.mark.parametrize("n,bits", [
    (4096, [50]),
    (65536, [60] + [50] * 44 + [60] * 15),          # C3 chain, examples/3_ckks.cu:796-803
    (65536, [60] + [59] * 29 + [60] * 10),          # C4 chain, bootstrapping_example.cu:69-116
    (8192, [60, 40, 40, 60]),
])
def test_coeff_modulus_create_matches_oracle(n, bits):
    assert PA.coeff_modulus_create(n, bits) == O.coeff_modulus_create(n, bits)


def test_coeff_modulus_create_rejects_bad_sizes():
    lib = PA.load()
    bs = (ctypes.c_int * 1)(61)
    out = (ctypes.c_uint64 * 1)()
    assert lib.phantom_coeff_modulus_create(4096, bs, 1, out) == 1
    assert b"bit_sizes" in lib.phantom_last_error()
    bs = (ctypes.c_int * 1)(50)
    assert lib.phantom_coeff_modulus_create(3000, bs, 1, out) == 1


# ---- ChaCha20 (csrc/chacha.h) and its numpy restatement, pinned to RFC 8439 -------------------

def _lib_block(key, counter, nonce):
    lib = PA.load()
    k = (ctypes.c_uint32 * 8)(*key)
    out = (ctypes.c_uint32 * 16)()
    PA.check(lib.phantom_chacha20_block(k, counter, nonce, out))
    return list(out)


# RFC 8439 section 2.3.2: key 00 01 .. 1f, nonce 00:00:00:09:00:00:00:4a:00:00:00:00, counter 1
# (serialized output 10 f1 e7 e4 d1 3b 59 15 50 0f dd 1f ...; state words 12..15 = 1, 0x09000000, 0x4a000000, 0 = counter 1 | 0x09000000 << 32, nonce 0x4a000000)
RFC_KEY = [0x03020100, 0x07060504, 0x0B0A0908, 0x0F0E0D0C, 0x13121110, 0x17161514, 0x1B1A1918, 0x1F1E1D1C]
RFC_BLOCK = [0xE4E7F110, 0x15593BD1, 0x1FDD0F50, 0xC47120A3, 0xC7F4D1C7, 0x0368C033, 0x9AAA2204, 0x4E6CD4C3,
             0x466482D2, 0x09AA9F07, 0x05D7C214, 0xA2028BD9, 0xD19C12B5, 0xB94E16DE, 0xE883D0CB, 0x4E3C50A2]
# RFC 8439 appendix A.1 test vector 1: all-zero key, nonce and counter: keystream 76 b8 e0 ad a0 f1 3d 90 ...
ZERO_BLOCK_HEAD = [0xADE0B876, 0x903DF1A0, 0xE56A5D40, 0x28BD8653]


def test_chacha20_block_matches_rfc8439():
    assert _lib_block(RFC_KEY, 1 | (0x09000000 << 32), 0x4A000000) == RFC_BLOCK
    assert _lib_block([0] * 8, 0, 0)[:4] == ZERO_BLOCK_HEAD


def test_numpy_chacha_matches_rfc8439_and_library():
    import chacha_np as C
    b = C.blocks(RFC_KEY, [1 | (0x09000000 << 32)], 0x4A000000)[0]
    assert [int(x) for x in b] == RFC_BLOCK
    assert [int(x) for x in C.blocks([0] * 8, [0], 0)[0][:4]] == ZERO_BLOCK_HEAD
    key = [0xDEADBEEF, 1, 2, 3, 4, 5, 6, 0xFFFFFFFF]
    for counter, nonce in [(0, 0), (7, 3), (2**32 + 5, 2**40 + 9)]:
        assert [int(x) for x in C.blocks(key, [counter], nonce)[0]] == _lib_block(key, counter, nonce)
