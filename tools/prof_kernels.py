"""Profiling driver (tools only): MODE=ntt50 | ntt60 | ntt60fi | c3.  ntt50/ntt60: forward NTT of [L][2^16]
(ntt60fi: forward then inverse)
(44 50-bit primes / the C4 chain's 40 primes) over a ring of 15 buffers; c3: relinearize of a
45-limb ciphertext (P = 15, dnum 3) with random keys.  Used under rocprofv3 (kernel trace, PMC)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("PHX_PY", os.path.join(ROOT, "phantom-fhe-boot_amd", "py")))  # PHX_PY: a variant build
import torch  # noqa: E402
import phantom_amd as PA  # noqa: E402

N = 1 << 16
iters = int(os.environ.get("ITERS", "20"))
mode = os.environ.get("MODE", "ntt50")
lib = PA.load()
s = torch.cuda.current_stream().cuda_stream
rng = np.random.default_rng(1)


def limbs(ms, polys=1):
    a = np.concatenate([rng.integers(0, q, size=N, dtype=np.uint64) for _ in range(polys) for q in ms])
    return torch.from_numpy(a.view(np.int64)).cuda()


if mode in ("ntt50", "ntt60", "ntt60fi"):
    if mode != "ntt50":
        mods = PA.coeff_modulus_create(N, [60] + [59] * 29 + [60] * 10)
    else:
        mods = PA.coeff_modulus_create(N, [60] + [50] * 44 + [60] * 15)[:44]
    L = len(mods)
    t = PA.NttTables(N, mods)
    ring = [limbs(mods) for _ in range(15)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(iters):
        PA.check(lib.phantom_nwt_forward_inplace(ring[i % 15].data_ptr(), t.handle, L, 0, s))
        if mode == "ntt60fi":
            PA.check(lib.phantom_nwt_backward_inplace(ring[i % 15].data_ptr(), t.handle, L, 0, s))
    torch.cuda.synchronize()
else:
    mods = PA.coeff_modulus_create(N, [60] + [50] * 44 + [60] * 15)
    ctx = PA.Context(N, mods, 15)
    ql = mods[:45]
    keys = [limbs(mods, 2) for _ in range(3)]
    kp = PA.ptr_array([k.data_ptr() for k in keys])
    prods = [limbs(ql, 3) for _ in range(4)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(iters):
        PA.check(lib.phantom_relinearize(ctx.handle, 1, prods[i % 4].data_ptr(), kp, 3, s))
    torch.cuda.synchronize()
print(f"{mode}: {(time.perf_counter() - t0) / iters * 1e6:.1f} us per iteration (incl. launch)")
