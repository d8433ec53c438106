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
