"""ctypes binding of libphantom_amd.so (include/phantom_amd.h) for tests and bench.py.

The product is the C-ABI library; this module only loads it and declares signatures.
It raises if the library is missing — there is no Python or CPU fallback.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PHANTOM_AMD_LIB: load another build of the same library (tools/build_variants.sh experiments)
LIB_PATH = os.environ.get("PHANTOM_AMD_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libphantom_amd.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "phantom_amd.h")

u64p = ctypes.POINTER(ctypes.c_uint64)
vp = ctypes.c_void_p
sz = ctypes.c_size_t

_SIGS = {
    "phantom_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "phantom_last_error": (ctypes.c_char_p, []),
    "phantom_version": (ctypes.c_char_p, []),
    "phantom_coeff_modulus_create": (ctypes.c_int, [sz, ctypes.POINTER(ctypes.c_int), sz, u64p]),
    "phantom_ntt_tables_create": (ctypes.c_int, [sz, u64p, sz, ctypes.POINTER(vp)]),
    "phantom_ntt_tables_destroy": (ctypes.c_int, [vp]),
    "phantom_ntt_tables_host": (ctypes.c_int, [vp, sz, u64p, u64p, u64p, u64p, u64p]),
    "phantom_nwt_forward_inplace": (ctypes.c_int, [vp, vp, sz, sz, vp]),
    "phantom_nwt_backward_inplace": (ctypes.c_int, [vp, vp, sz, sz, vp]),
    "phantom_nwt_backward": (ctypes.c_int, [vp, vp, vp, sz, sz, vp]),
    "phantom_nwt_backward_scale": (ctypes.c_int, [vp, vp, vp, sz, sz, vp, vp, vp]),
    "phantom_nwt_forward_include_special_mod_exclude_range": (ctypes.c_int, [vp, vp, sz, sz, sz, sz, sz, sz, vp]),
    "phantom_nwt_backward_inplace_include_special_mod": (ctypes.c_int, [vp, vp, sz, sz, sz, sz, vp]),
    "phantom_nwt_backward_inplace_scale": (ctypes.c_int, [vp, vp, sz, sz, vp, vp, vp]),
    "phantom_nwt_forward_include_special_mod": (ctypes.c_int, [vp, vp, sz, sz, sz, sz, vp]),
    "phantom_nwt_forward_fuse_moddown": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, sz, sz, vp]),
    "phantom_fnwt_1d": (ctypes.c_int, [vp, vp, sz, sz, vp]),
    "phantom_inwt_1d": (ctypes.c_int, [vp, vp, sz, sz, vp, vp, vp]),
    "phantom_context_create": (ctypes.c_int, [sz, u64p, sz, sz, ctypes.POINTER(vp)]),
    "phantom_context_destroy": (ctypes.c_int, [vp]),
    "phantom_context_coeff_modulus_size": (sz, [vp, sz]),
    "phantom_context_set_unbiased_moddown": (ctypes.c_int, [vp, ctypes.c_int]),
    "phantom_multiply": (ctypes.c_int, [vp, sz, vp, vp, vp, vp]),
    "phantom_square": (ctypes.c_int, [vp, sz, vp, vp, vp]),
    "phantom_relinearize": (ctypes.c_int, [vp, sz, vp, ctypes.POINTER(vp), sz, vp]),
    "phantom_relinearize_rescale": (ctypes.c_int, [vp, sz, vp, vp, ctypes.POINTER(vp), sz, vp]),
    "phantom_relinearize_rescale_batch": (ctypes.c_int, [vp, sz, vp, sz, sz, vp, sz, ctypes.POINTER(vp), sz, vp]),
    "phantom_keyswitch": (ctypes.c_int, [vp, sz, vp, vp, ctypes.POINTER(vp), sz, vp]),
    "phantom_modup": (ctypes.c_int, [vp, sz, vp, vp, vp]),
    "phantom_keyswitch_inner_prod": (ctypes.c_int, [vp, sz, vp, ctypes.POINTER(vp), sz, vp, vp]),
    "phantom_moddown_from_ntt": (ctypes.c_int, [vp, sz, vp, vp, vp]),
    "phantom_fast_bconv": (ctypes.c_int, [u64p, sz, u64p, sz, vp, vp, sz, ctypes.c_int, vp]),
    "phantom_bconv_create": (ctypes.c_int, [u64p, sz, u64p, sz, vp, ctypes.POINTER(vp)]),
    "phantom_bconv_run": (ctypes.c_int, [vp, vp, vp, sz, ctypes.c_int, vp]),
    "phantom_bconv_destroy": (ctypes.c_int, [vp]),
    "phantom_moddown_modup": (ctypes.c_int, [vp, sz, vp, vp, vp]),
    "phantom_moddown_modup_batch": (ctypes.c_int, [vp, sz, vp, sz, sz, vp, vp]),
    "phantom_ciphertext_serialize": (ctypes.c_int, [vp, vp, vp, sz, vp]),
    "phantom_ciphertext_deserialize": (ctypes.c_int, [vp, sz, vp, vp, sz, vp]),
    "phantom_moddown_rescale": (ctypes.c_int, [vp, sz, vp, vp, sz, vp]),
    "phantom_rescale_to_next": (ctypes.c_int, [vp, sz, vp, vp, sz, vp]),
    "phantom_apply_galois_ntt": (ctypes.c_int, [vp, ctypes.c_uint32, vp, vp, sz, vp]),
    "phantom_poly_op": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, vp, sz, sz, vp]),
    "phantom_switch_modulus_raise": (ctypes.c_int, [vp, vp, vp, sz, vp]),
    "phantom_chacha20_block": (ctypes.c_int, [vp, ctypes.c_uint64, ctypes.c_uint64, vp]),
    "phantom_sample_poly": (ctypes.c_int, [vp, ctypes.c_int, vp, ctypes.c_uint64, vp, sz, vp]),
    "phantom_boot_session_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.c_uint32,
                                                   ctypes.c_uint32, ctypes.c_uint32, vp, ctypes.POINTER(vp)]),
    "phantom_boot_session_destroy": (ctypes.c_int, [vp]),
    "phantom_traffic_read": (ctypes.c_int, [vp]),
    "phantom_traffic_reset": (ctypes.c_int, []),
    "phantom_pool_stats": (ctypes.c_int, [vp]),
    "phantom_pool_reset_peak": (ctypes.c_int, []),
    "phantom_lt_bsgs": (ctypes.c_int, [vp, sz, ctypes.POINTER(vp), sz, ctypes.POINTER(vp), sz, ctypes.POINTER(vp), vp]),
    "phantom_keyswitch_ext": (ctypes.c_int, [vp, sz, vp, vp, vp]),
    "phantom_fast_rotation_ext": (ctypes.c_int, [vp, sz, vp, vp, ctypes.POINTER(vp), sz, ctypes.c_uint32, ctypes.c_int,
                                                 vp, vp]),
    "phantom_fast_rotation_ext_batch": (ctypes.c_int, [vp, sz, vp, vp, ctypes.POINTER(ctypes.POINTER(vp)), sz,
                                                       ctypes.POINTER(ctypes.c_uint32), sz, ctypes.POINTER(vp), vp]),
    "phantom_rotate_ext_accumulate": (ctypes.c_int, [vp, sz, vp, ctypes.POINTER(vp), sz, ctypes.c_uint32, vp,
                                                     ctypes.c_int, vp]),
    "phantom_lt_bsgs_group": (ctypes.c_int, [vp, sz, sz, ctypes.POINTER(vp), sz, sz, ctypes.POINTER(vp), sz,
                                             ctypes.POINTER(vp), ctypes.POINTER(vp), sz, vp]),
    "phantom_fast_rotation_ext_batch_group": (ctypes.c_int, [vp, sz, sz, ctypes.POINTER(vp), ctypes.POINTER(vp),
                                                             ctypes.POINTER(ctypes.POINTER(vp)), sz,
                                                             ctypes.POINTER(ctypes.c_uint32), sz, ctypes.POINTER(vp),
                                                             vp]),
    "phantom_rotate_ext_accumulate_group": (ctypes.c_int, [vp, sz, sz, ctypes.POINTER(vp), ctypes.POINTER(vp), sz,
                                                           ctypes.c_uint32, ctypes.POINTER(vp), ctypes.c_int, vp]),
    "phantom_tensor_lin": (ctypes.c_int, [vp, sz, vp, vp, vp, vp, vp, sz, vp, vp]),
    "phantom_tensor_lin_batch": (ctypes.c_int, [vp, sz, sz, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp),
                                                vp, ctypes.POINTER(vp), sz, ctypes.POINTER(vp), ctypes.POINTER(vp), vp]),
    "phantom_lin_comb": (ctypes.c_int, [vp, sz, vp, sz, vp, vp, sz, sz, vp, vp]),
    "phantom_mul_scalar": (ctypes.c_int, [vp, sz, vp, sz, vp, vp, vp, sz, vp]),
    "phantom_leaf_combine": (ctypes.c_int, [vp, sz, ctypes.POINTER(vp), vp, sz, vp, vp, ctypes.POINTER(vp), sz, vp]),
    "phantom_eval_mod_coefficients": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, vp]),
    "phantom_boot_encrypt": (ctypes.c_int, [vp, vp, sz, sz, vp, sz, ctypes.POINTER(sz)]),
    "phantom_boot_output_bytes": (ctypes.c_int, [vp, ctypes.POINTER(sz)]),
    "phantom_galois_key_serialize": (ctypes.c_int, [sz, sz, sz, sz, vp, vp, sz, vp]),
    "phantom_salsa20_block": (ctypes.c_int, [vp, ctypes.c_uint64, vp]),
    "phantom_sample_uniform_seeded": (ctypes.c_int, [vp, vp, vp, sz, vp]),
    "phantom_boot_layout": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.c_uint32,
                                           ctypes.c_uint32, sz, ctypes.POINTER(sz), ctypes.POINTER(sz),
                                           ctypes.POINTER(sz)]),
    "phantom_boot_run": (ctypes.c_int, [vp, vp, sz, sz, vp, sz, ctypes.c_int]),
    "phantom_boot_run_grouped": (ctypes.c_int, [vp, vp, sz, sz, vp, sz, ctypes.c_int, ctypes.c_int]),
    "phantom_boot_decrypt": (ctypes.c_int, [vp, vp, sz, vp]),
}

_lib = None


class PhantomError(RuntimeError):
    pass


def load():
    """Load libphantom_amd.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch bundles its own libamdhip64 (soname
        # libamdhip64.so.7).  Loading torch first makes this library bind to that same
        # runtime instead of pulling a second copy from /opt/rocm.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise PhantomError(f"{LIB_PATH} missing: run __graft_entry__.build() (no fallback path exists)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            if hasattr(lib, name):
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
        _lib = lib
    return _lib


def check(status):
    if status != 0:
        lib = load()
        raise PhantomError(f"{lib.phantom_status_string(status).decode()}: {lib.phantom_last_error().decode()}")


def declared_symbols(header=HEADER_PATH):
    """Names of every function declared in include/phantom_amd.h."""
    import re
    txt = open(header).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(phantom_[a-z0-9_]+)\s*\(", txt)))


def u64_array(values):
    arr = (ctypes.c_uint64 * len(values))(*values)
    return arr


def coeff_modulus_create(n, bit_sizes):
    lib = load()
    bs = (ctypes.c_int * len(bit_sizes))(*bit_sizes)
    out = (ctypes.c_uint64 * len(bit_sizes))()
    check(lib.phantom_coeff_modulus_create(n, bs, len(bit_sizes), out))
    return list(out)


class Context:
    """Owning handle of a phantom_context (CKKS PhantomContext over a key-level chain)."""

    def __init__(self, n, moduli, special_modulus_size):
        lib = load()
        self.n = n
        self.moduli = list(moduli)
        self.size_P = special_modulus_size
        self.size_Q = len(self.moduli) - special_modulus_size
        h = vp()
        check(lib.phantom_context_create(n, u64_array(self.moduli), len(self.moduli), special_modulus_size,
                                         ctypes.byref(h)))
        self.handle = h

    def ql(self, chain_index):
        return self.moduli[:self.size_Q - (chain_index - 1)]

    def set_unbiased_moddown(self, on):
        """Opt-in mean-unbiased moddowns (phantom_context_set_unbiased_moddown); off by default."""
        check(load().phantom_context_set_unbiased_moddown(self.handle, 1 if on else 0))

    def close(self):
        if self.handle:
            load().phantom_context_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def ptr_array(ptrs):
    return (vp * len(ptrs))(*ptrs)


class NttTables:
    """Owning handle of a phantom_ntt_tables (device NTT tables for a modulus list)."""

    def __init__(self, n, moduli):
        lib = load()
        self.n = n
        self.moduli = list(moduli)
        h = vp()
        check(lib.phantom_ntt_tables_create(n, u64_array(self.moduli), len(self.moduli), ctypes.byref(h)))
        self.handle = h

    def close(self):
        if self.handle:
            load().phantom_ntt_tables_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def boot_layout(chain_index, log_n=16, depth=29, special=10, level_budget=(2, 2), num_slots=0, iterations=1):
    """(input bytes at chain_index, output bytes, output chain index) of a bootstrap session's
    serialized ciphertexts, computed on the host from the parameters (phantom_boot_layout)."""
    lb = (ctypes.c_uint32 * 2)(*level_budget)
    a, b, c = sz(0), sz(0), sz(0)
    check(load().phantom_boot_layout(log_n, depth, special, lb, num_slots, iterations, chain_index,
                                     ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
    return a.value, b.value, c.value


class BootSession:
    """Owning handle of a phantom_boot_session (the SimpleBootstrapExample set-up; C4/C5)."""

    def __init__(self, seed, log_n=16, depth=29, special=10, level_budget=(2, 2), num_slots=0, iterations=1,
                 precision=0):
        lib = load()
        assert len(seed) == 32
        self.seed = bytes(seed)
        lb = (ctypes.c_uint32 * 2)(*level_budget)
        h = vp()
        check(lib.phantom_boot_session_create(log_n, depth, special, lb, num_slots, iterations, precision,
                                              self.seed, ctypes.byref(h)))
        self.handle = h
        self.n = 1 << log_n
        self.slots = num_slots or self.n // 2
        self.depth = depth
        self.params = dict(log_n=log_n, depth=depth, special=special, level_budget=tuple(level_budget),
                           num_slots=num_slots, iterations=iterations)

    def output_bytes(self):
        b = sz(0)
        check(load().phantom_boot_output_bytes(self.handle, ctypes.byref(b)))
        return b.value

    def input_bytes(self, chain_index):
        return boot_layout(chain_index, **self.params)[0]

    def encrypt(self, values, chain_index, dev_ptr, stride):
        """values: float64 [count, slots]; writes serialized ciphertexts at dev_ptr + i * stride."""
        import numpy as np
        v = np.ascontiguousarray(values, dtype=np.float64)
        if v.ndim != 2 or v.shape[1] != self.slots:
            raise ValueError(f"values must be [count, {self.slots}], got shape {v.shape}")
        b = sz(0)
        check(load().phantom_boot_encrypt(self.handle, v.ctypes.data, v.shape[0], chain_index, dev_ptr, stride,
                                          ctypes.byref(b)))
        return b.value

    def run(self, dev_in, in_stride, count, dev_out, out_stride, lanes=4, group=None):
        """group: at most this many ciphertexts per lane in lockstep (1..8; a lane's m ciphertexts form
        ceil(m / group) groups of near-equal size); None = the library default (8)."""
        if group is None:
            check(load().phantom_boot_run(self.handle, dev_in, in_stride, count, dev_out, out_stride, lanes))
        else:
            check(load().phantom_boot_run_grouped(self.handle, dev_in, in_stride, count, dev_out, out_stride, lanes,
                                                  group))

    def decrypt(self, dev_ptr, capacity):
        import numpy as np
        out = np.zeros(self.slots, dtype=np.float64)
        check(load().phantom_boot_decrypt(self.handle, dev_ptr, capacity, out.ctypes.data))
        return out

    def close(self):
        if self.handle:
            load().phantom_boot_session_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pool_stats():
    """the device allocator's {held, live, peak_live, peak_held} bytes (phantom_pool_stats)"""
    out = (ctypes.c_uint64 * 4)()
    check(load().phantom_pool_stats(out))
    return dict(zip(("held", "live", "peak_live", "peak_held"), (int(x) for x in out)))


def pool_reset_peak():
    check(load().phantom_pool_reset_peak())


def traffic():
    """algorithmic bytes counted since the last reset: {"keys", "plaintexts", "ciphertexts", "total"}"""
    out = (ctypes.c_uint64 * 3)()
    check(load().phantom_traffic_read(out))
    d = {"keys": out[0], "plaintexts": out[1], "ciphertexts": out[2]}
    d["total"] = sum(d.values())
    return d


def traffic_reset():
    check(load().phantom_traffic_reset())


def bit_precision(ref, actual):
    """compute_bit_precision of bootstrapping_example.cu:17-41: mean of -log2 relative error."""
    import numpy as np
    ref = np.asarray(ref, dtype=np.float64)
    actual = np.asarray(actual, dtype=np.float64)
    keep = np.abs(ref) >= 1e-20
    rel = np.abs(ref[keep] - actual[keep]) / np.abs(ref[keep])
    rel = np.maximum(rel, 1e-40)
    return float(np.mean(-np.log2(rel))) if rel.size else 0.0
