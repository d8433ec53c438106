"""One rank of the C5 data-path test (tests/test_bench_dist.py): the multi-GPU scatter / gather of
bench.py's C5 leg (phantom-fhe-boot_amd/py/shard.py) on CPU over gloo.  Rank 0 serializes a batch
of ciphertexts in the reference's byte format (host C-ABI, include/ciphertext.h:184-225),
scatters them, every rank deserializes its slice, applies a host stand-in for the bootstrap
(reverses the words, chain_index + 1, scale x 2, correction_factor = 1 + rank), reserializes,
and rank 0 gathers and checks every result against its input and the rank that owned it.
Prints one JSON line on rank 0."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "phantom-fhe-boot_amd", "py"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import phantom_amd as PA  # noqa: E402
import shard  # noqa: E402


class Hdr(ctypes.Structure):
    _fields_ = [("chain_index", ctypes.c_uint64), ("size", ctypes.c_uint64),
                ("poly_modulus_degree", ctypes.c_uint64), ("coeff_modulus_size", ctypes.c_uint64),
                ("scale", ctypes.c_double), ("correction_factor", ctypes.c_uint64),
                ("noise_scale_deg", ctypes.c_uint64), ("is_ntt_form", ctypes.c_int), ("is_asymmetric", ctypes.c_int)]


def serialize(lib, h, data, stride):
    out = (ctypes.c_uint8 * stride)()
    written = ctypes.c_size_t(0)
    PA.check(lib.phantom_ciphertext_serialize(ctypes.byref(h), data.ctypes.data, out, stride, ctypes.byref(written)))
    return np.frombuffer(bytes(out), dtype=np.uint8)


def deserialize(lib, row):
    b = bytes(row.tolist())
    h, words = Hdr(), ctypes.c_size_t(0)
    PA.check(lib.phantom_ciphertext_deserialize(b, len(b), ctypes.byref(h), None, 0, ctypes.byref(words)))
    data = np.zeros(words.value, dtype=np.uint64)
    PA.check(lib.phantom_ciphertext_deserialize(b, len(b), ctypes.byref(h), data.ctypes.data, data.size,
                                                ctypes.byref(words)))
    return h, data


def main():
    dist.init_process_group("gloo")
    world, rank = dist.get_world_size(), dist.get_rank()
    lib = PA.load()
    total, n, L = 6 * world, 16, 3
    words = 2 * L * n
    stride = (58 + 8 * words + 63) // 64 * 64
    seed = shard.broadcast_seed(dist, "cpu")
    rng = np.random.default_rng(5)
    inputs = [rng.integers(0, 2**62, size=words, dtype=np.uint64) for _ in range(total)]
    full = None
    if rank == 0:
        full = torch.zeros((total, stride), dtype=torch.uint8)
        for i, d in enumerate(inputs):
            full[i] = torch.from_numpy(serialize(lib, Hdr(3, 2, n, L, 2.0 ** 40, 1, 1, 1, 0), d, stride).copy())
    local = shard.scatter_rows(dist, full, total // world, stride, "cpu")
    out = torch.zeros_like(local)
    for j in range(local.shape[0]):
        h, d = deserialize(lib, local[j].numpy())
        h.chain_index += 1
        h.scale *= 2.0
        h.correction_factor = 1 + rank
        out[j] = torch.from_numpy(serialize(lib, h, d[::-1].copy(), stride).copy())
    gathered = shard.gather_rows(dist, out, "cpu")
    if rank == 0:
        ok = True
        for i in range(total):
            h, d = deserialize(lib, gathered[i].numpy())
            ok &= np.array_equal(d, inputs[i][::-1]) and h.chain_index == 4 and h.scale == 2.0 ** 41
            ok &= h.correction_factor == 1 + i // (total // world)
        print(json.dumps({"ok": bool(ok), "world": world, "total": total, "seed_bytes": len(seed)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
