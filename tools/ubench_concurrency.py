"""Concurrency probe (tools only): does a second stream fill the SIMDs a small NTT launch leaves
idle?  C4-chain primes, [L][2^16] buffers.  For L in LIMBS: time ITERS x (forward NTT of A; of B)
on one stream, the same split over two streams, and one launch over 2L limbs (A and B adjacent).
Prints µs per pair."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "phantom-fhe-boot_amd", "py"))
import torch  # noqa: E402
import phantom_amd as PA  # noqa: E402

N = 1 << 16
iters = int(os.environ.get("ITERS", "200"))
lib = PA.load()
mods = PA.coeff_modulus_create(N, [60] + [59] * 29 + [60] * 10)
rng = np.random.default_rng(1)


def limbs(ms):
    a = np.concatenate([rng.integers(0, q, size=N, dtype=np.uint64) for q in ms])
    return torch.from_numpy(a.view(np.int64)).cuda()


def timed(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


s0 = torch.cuda.current_stream()
s1 = torch.cuda.Stream()
for L in [int(x) for x in os.environ.get("LIMBS", "10,20,40").split(",")]:
    ms = mods[:L] * 2
    t = PA.NttTables(N, ms)
    ab = limbs(ms)  # A = limbs [0, L), B = limbs [L, 2L) (same moduli)
    a, b = ab.data_ptr(), ab.data_ptr() + L * N * 8
    for name, inv in (("fwd", False), ("inv", True)):
        f = lib.phantom_nwt_backward_inplace if inv else lib.phantom_nwt_forward_inplace
        def one(p, st):
            PA.check(f(p, t.handle, L, 0, st.cuda_stream))

        def serial():
            one(a, s0)
            one(b, s0)

        def two_streams():
            ev = torch.cuda.Event()
            ev.record(s0)
            s1.wait_event(ev)
            one(a, s0)
            one(b, s1)
            ev2 = torch.cuda.Event()
            ev2.record(s1)
            s0.wait_event(ev2)

        def fused():
            PA.check(f(a, t.handle, 2 * L, 0, s0.cuda_stream))
        print(f"L={L:3d} {name}: serial {timed(serial):7.2f} us  two streams {timed(two_streams):7.2f} us  "
              f"one launch of 2L {timed(fused):7.2f} us", flush=True)
    t.close()
