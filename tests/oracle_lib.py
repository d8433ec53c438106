"""ctypes binding of the CPU oracle (oracle/liboracle.so) — the parity checker.

Test infrastructure only: tests/, bench.py's cpu_baseline leg and __graft_entry__.smoke()
use it; the product never does.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

u64 = ctypes.c_uint64
u64p = ctypes.POINTER(ctypes.c_uint64)
u32p = ctypes.POINTER(ctypes.c_uint32)
u8p = ctypes.POINTER(ctypes.c_uint8)
sz = ctypes.c_size_t

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_PATH):
            import subprocess
            subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(ORACLE_PATH)
        sig = {
            "or_mulmod": (u64, [u64, u64, u64]),
            "or_powmod": (u64, [u64, u64, u64]),
            "or_invmod": (u64, [u64, u64]),
            "or_is_prime": (ctypes.c_int, [u64]),
            "or_shoup": (u64, [u64, u64]),
            "or_coeff_modulus_create": (ctypes.c_int, [sz, ctypes.POINTER(ctypes.c_int), sz, u64p]),
            "or_minimal_primitive_root": (u64, [u64, u64]),
            "or_ntt_tables": (ctypes.c_int, [sz, u64, u64p, u64p, u64p, u64p, u64p, u64p]),
            "or_ntt_fwd": (None, [u64p, sz, sz, u64p]),
            "or_ntt_inv": (None, [u64p, sz, sz, u64p]),
            "or_ntt_fwd_naive": (None, [u64p, u64p, sz, u64]),
            "or_ntt_plan_create": (ctypes.c_void_p, [sz, sz, u64p]),
            "or_ntt_plan_destroy": (None, [ctypes.c_void_p]),
            "or_ntt_plan_fwd": (None, [ctypes.c_void_p, u64p, sz, ctypes.c_int]),
            "or_ntt_plan_inv": (None, [ctypes.c_void_p, u64p, sz, ctypes.c_int]),
            "or_poly_add": (None, [u64p, u64p, u64p, sz, sz, u64p]),
            "or_poly_sub": (None, [u64p, u64p, u64p, sz, sz, u64p]),
            "or_poly_negate": (None, [u64p, u64p, sz, sz, u64p]),
            "or_poly_mul": (None, [u64p, u64p, u64p, sz, sz, u64p]),
            "or_poly_mul_scalar": (None, [u64p, u64p, u64p, sz, sz, u64p]),
            "or_tensor_prod_2x2": (None, [u64p, u64p, u64p, sz, sz, u64p]),
            "or_salsa20_core": (None, [u32p, u32p]),
            "or_salsa20_block": (None, [ctypes.c_char_p, ctypes.c_uint64, u32p]),
            "or_sample_uniform_seeded": (None, [ctypes.c_char_p, u64p, sz, sz, u64p]),
            "or_tensor_square_2x2": (None, [u64p, u64p, sz, sz, u64p]),
            "or_bconv": (None, [u64p, u64p, sz, u64p, sz, u64p, sz]),
            "or_modup": (None, [u64p, u64p, sz, u64p, sz, u64p, sz]),
            "or_keyswitch_inner_prod": (None, [u64p, ctypes.POINTER(u64p), u64p, sz, sz, sz, sz, sz, u64p]),
            "or_moddown_from_ntt": (None, [u64p, u64p, sz, u64p, sz, u64p, sz]),
            "or_keyswitch_add": (None, [u64p, u64p, ctypes.POINTER(u64p), sz, sz, sz, sz, u64p]),
            "or_relinearize": (None, [u64p, sz, sz, sz, sz, ctypes.POINTER(u64p), u64p]),
            "or_rescale_ntt": (None, [u64p, u64p, sz, sz, sz, u64p]),
            "or_mod_switch_drop_ntt": (None, [u64p, u64p, sz, sz, sz]),
            "or_galois_perm_ntt": (None, [ctypes.c_uint32, sz, ctypes.POINTER(ctypes.c_uint32)]),
            "or_apply_galois_ntt": (None, [u64p, u64p, sz, sz, ctypes.c_uint32]),
            "or_switch_modulus_raise": (None, [u64p, u64p, sz, u64, u64p, sz]),
            "or_monomial_ntt": (None, [u64p, sz, sz, u64p, ctypes.c_uint32]),
            "or_lt_bsgs": (None, [ctypes.POINTER(u64p), sz, ctypes.POINTER(u64p), sz, ctypes.POINTER(u64p), sz, sz, sz,
                                  sz, u64p]),
            "or_keyswitch_ext": (None, [u64p, u64p, sz, sz, sz, sz, u64p]),
            "or_fast_rotation_ext": (None, [u64p, u64p, ctypes.POINTER(u64p), ctypes.c_uint32, ctypes.c_int, u64p, sz,
                                            sz, sz, sz, u64p]),
            "or_rotate_ext_accumulate": (None, [u64p, ctypes.POINTER(u64p), ctypes.c_uint32, u64p, ctypes.c_int, sz,
                                                sz, sz, sz, u64p]),
            "or_mul_scalar_acc": (None, [u64p, sz, u64p, u64p, u64p, sz, sz, sz, u64p]),
            "or_tensor_lin": (None, [u64p, u64p, u64p, sz, sz, u64p, u64p, u64p, sz, u64p]),
            "or_lin_comb": (None, [u64p, sz, u64p, u64p, sz, sz, u64p, sz, sz, u64p]),
            "or_leaf_combine": (None, [ctypes.POINTER(u64p), ctypes.POINTER(sz), sz, u64p, u64p, ctypes.POINTER(u64p),
                                       sz, sz, sz, u64p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def P(a):
    """uint64 numpy array -> u64 pointer (array must stay alive)."""
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(u64p)


def arr(values):
    return np.ascontiguousarray(np.array(values, dtype=np.uint64))


def coeff_modulus_create(n, bit_sizes):
    out = np.zeros(len(bit_sizes), dtype=np.uint64)
    bs = (ctypes.c_int * len(bit_sizes))(*bit_sizes)
    assert lib().or_coeff_modulus_create(n, bs, len(bit_sizes), P(out)) == 0
    return [int(x) for x in out]


def ntt_tables(n, q):
    t = [np.zeros(n, dtype=np.uint64) for _ in range(4)]
    ni = np.zeros(1, dtype=np.uint64)
    nis = np.zeros(1, dtype=np.uint64)
    assert lib().or_ntt_tables(n, q, P(t[0]), P(t[1]), P(t[2]), P(t[3]), P(ni), P(nis)) == 0
    return t, int(ni[0])


def ntt_fwd(data, n, moduli):
    d = np.ascontiguousarray(data.copy())
    m = arr(moduli)
    lib().or_ntt_fwd(P(d), n, len(moduli), P(m))
    return d


def ntt_inv(data, n, moduli):
    d = np.ascontiguousarray(data.copy())
    m = arr(moduli)
    lib().or_ntt_inv(P(d), n, len(moduli), P(m))
    return d


def random_limbs(rng, n, moduli):
    """Uniform [0, q_i) limb-major data."""
    out = np.empty(len(moduli) * n, dtype=np.uint64)
    for i, q in enumerate(moduli):
        out[i * n:(i + 1) * n] = rng.integers(0, q, size=n, dtype=np.uint64)
    return out


def ptrs(arrays):
    """host array of u64 pointers to numpy arrays (the arrays must stay alive)"""
    return (u64p * len(arrays))(*[P(a) for a in arrays])
