"""One rank of the C5 data-path test (tests/test_bench_dist.py): bench.py's multi-GPU scatter /
gather (phantom-fhe-boot_amd/py/shard.py) on CPU over gloo, with the session's real serialized
ciphertexts.

Shapes and strides are those of the C5 job (bench.py c5_leg): the bootstrap session of
bootstrapping_example.cu:69-116 (N = 2^16, Q = {60, 29 x 59}, P = 10 x 60, levelBudget {2, 2}),
inputs at chain index 26 and outputs at the session's output chain, sizes from
phantom_boot_layout (the same numbers phantom_boot_encrypt / phantom_boot_output_bytes give on a
GPU), rows rounded up to 256 B as bench.py does.  Rank 0 serializes a batch in the reference's
byte format (include/ciphertext.h:184-225) with the header phantom_boot_encrypt writes (chain, size
2, N, limbs, the level's FLEXIBLEAUTO scale, correction 1, degree 1, NTT form, symmetric) and
scatters it; every rank parses and checks its rows, and in place of the bootstrap (which needs a
GPU) writes output ciphertexts of the session's output shape derived from each input and its own
rank; rank 0 gathers and checks every byte, the order and the owning rank.  One JSON line on rank 0.
"""
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

LOG_N, DEPTH, SPECIAL, CHAIN = 16, 29, 10, 26
ALIGN = 256


class Hdr(ctypes.Structure):
    _fields_ = [("chain_index", ctypes.c_uint64), ("size", ctypes.c_uint64),
                ("poly_modulus_degree", ctypes.c_uint64), ("coeff_modulus_size", ctypes.c_uint64),
                ("scale", ctypes.c_double), ("correction_factor", ctypes.c_uint64),
                ("noise_scale_deg", ctypes.c_uint64), ("is_ntt_form", ctypes.c_int), ("is_asymmetric", ctypes.c_int)]


def serialize(lib, h, data, stride):
    out = (ctypes.c_uint8 * stride)()
    written = ctypes.c_size_t(0)
    PA.check(lib.phantom_ciphertext_serialize(ctypes.byref(h), data.ctypes.data, out, stride, ctypes.byref(written)))
    return np.frombuffer(bytes(out), dtype=np.uint8), written.value


def deserialize(lib, row):
    b = row.tobytes()
    h, words = Hdr(), ctypes.c_size_t(0)
    PA.check(lib.phantom_ciphertext_deserialize(b, len(b), ctypes.byref(h), None, 0, ctypes.byref(words)))
    data = np.zeros(words.value, dtype=np.uint64)
    PA.check(lib.phantom_ciphertext_deserialize(b, len(b), ctypes.byref(h), data.ctypes.data, data.size,
                                                ctypes.byref(words)))
    return h, data


def scaling_factors(moduli, size_q):
    """PreComputeScale (include/ciphertext.h:320-367): sf[0] = q_last, sf[k] = sf[k-1]^2 / q_(Q-k)"""
    sf = [float(moduli[size_q - 1])]
    for k in range(1, size_q):
        sf.append(sf[k - 1] * sf[k - 1] / float(moduli[size_q - k]))
    return sf


def stand_in(data, n, limbs_in, limbs_out, moduli, owner):
    """the rank's output for one input: limb l of each polynomial = input limb l mod limbs_in,
    plus owner + l, reduced mod q_l"""
    src = data.reshape(2, limbs_in, n)
    out = np.empty((2, limbs_out, n), dtype=np.uint64)
    for l in range(limbs_out):
        q = np.uint64(moduli[l])
        out[:, l] = (src[:, l % limbs_in] % q + np.uint64(owner + l)) % q
    return out.reshape(-1)


def main():
    dist.init_process_group("gloo")
    world, rank = dist.get_world_size(), dist.get_rank()
    lib = PA.load()
    n = 1 << LOG_N
    in_bytes, out_bytes, out_chain = PA.boot_layout(CHAIN, log_n=LOG_N, depth=DEPTH, special=SPECIAL)
    sin, sout = -(-in_bytes // ALIGN) * ALIGN, -(-out_bytes // ALIGN) * ALIGN
    moduli = PA.coeff_modulus_create(n, [60] + [59] * DEPTH + [60] * SPECIAL)
    size_q = DEPTH + 1
    l_in, l_out = size_q - (CHAIN - 1), size_q - (out_chain - 1)
    sf = scaling_factors(moduli, size_q)
    per = 2
    total = per * world
    seed = shard.broadcast_seed(dist, "cpu")
    rng = np.random.default_rng(5)
    inputs = [np.concatenate([rng.integers(0, q, size=n, dtype=np.uint64) for _ in range(2) for q in moduli[:l_in]])
              for _ in range(total)]
    full = None
    ok = True
    if rank == 0:
        full = torch.zeros((total, sin), dtype=torch.uint8)
        for i, d in enumerate(inputs):
            row, written = serialize(lib, Hdr(CHAIN, 2, n, l_in, sf[CHAIN - 1], 1, 1, 1, 0), d, sin)
            ok &= written == in_bytes
            full[i] = torch.from_numpy(row.copy())
    local = shard.scatter_rows(dist, full, per, sin, "cpu")
    out = torch.zeros((per, sout), dtype=torch.uint8)
    for j in range(per):
        h, d = deserialize(lib, local[j].numpy())
        ok &= (h.chain_index, h.size, h.poly_modulus_degree, h.coeff_modulus_size) == (CHAIN, 2, n, l_in)
        ok &= h.scale == sf[CHAIN - 1] and h.noise_scale_deg == 1 and h.is_ntt_form == 1 and h.is_asymmetric == 0
        ok &= np.array_equal(d, inputs[rank * per + j])
        res = stand_in(d, n, l_in, l_out, moduli, rank)
        row, written = serialize(lib, Hdr(out_chain, 2, n, l_out, sf[out_chain - 1], 1, 1, 1, 0), res, sout)
        ok &= written == out_bytes
        out[j] = torch.from_numpy(row.copy())
    gathered = shard.gather_rows(dist, out, "cpu")
    # bench.py's per-rank C5 figures (wall time, pool): every rank sees every rank's values in order
    stats = shard.gather_stats(dist, [1.5 + rank, 10.0 * rank], "cpu")
    ok &= stats == [[1.5 + r, 10.0 * r] for r in range(world)]
    if rank == 0:
        for i in range(total):
            h, d = deserialize(lib, gathered[i].numpy())
            ok &= (h.chain_index, h.coeff_modulus_size) == (out_chain, l_out) and h.scale == sf[out_chain - 1]
            ok &= np.array_equal(d, stand_in(inputs[i], n, l_in, l_out, moduli, i // per))
        print(json.dumps({"ok": bool(ok), "world": world, "total": total, "seed_bytes": len(seed),
                          "in_bytes": in_bytes, "out_bytes": out_bytes, "out_chain": out_chain}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
