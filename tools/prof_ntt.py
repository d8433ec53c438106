"""Profiling driver: forward (and optionally inverse) NTT, N=2^16, L=44, ring of buffers.
Used under rocprofv3 (kernel trace / PMC passes); prints mean per-call time."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "phantom-fhe-boot_amd", "py"))
import torch  # noqa: E402
import phantom_amd as PA  # noqa: E402

N, L = 1 << 16, 44
iters = int(os.environ.get("ITERS", "30"))
inverse = os.environ.get("INV", "1") == "1"
lib = PA.load()
# BITS=60: 44 60-bit primes (the integer Shoup path every C4 bootstrap limb takes)
if os.environ.get("BITS", "50") == "60":
    mods = PA.coeff_modulus_create(N, [60] * L)
elif os.environ.get("BITS") == "c4":  # the 40-limb C4 chain (Q = {60, 29 x 59}, P = 10 x 60)
    mods = PA.coeff_modulus_create(N, [60] + [59] * 29 + [60] * 10)
else:
    mods = PA.coeff_modulus_create(N, [60] + [50] * 44 + [60] * 15)[:L]
mods = mods * int(os.environ.get("REP", "1"))  # REP times as many limbs (the same primes) per launch
L = len(mods)
t = PA.NttTables(N, mods)
rng = np.random.default_rng(1)
base = np.concatenate([rng.integers(0, q, size=N, dtype=np.uint64) for q in mods])
ring = [torch.from_numpy(base.view(np.int64)).cuda() for _ in range(15)]
s = torch.cuda.current_stream().cuda_stream
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(iters):
    d = ring[i % 15].data_ptr()
    PA.check(lib.phantom_nwt_forward_inplace(d, t.handle, L, 0, s))
    if inverse:
        PA.check(lib.phantom_nwt_backward_inplace(d, t.handle, L, 0, s))
torch.cuda.synchronize()
print(f"{(time.perf_counter() - t0) / iters * 1e6:.1f} us per iteration (incl. launch)")
