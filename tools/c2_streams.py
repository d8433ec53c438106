"""C2 throughput (forward + inverse NTT of independent [44][65536] batches) with the steps dealt
round-robin to 1, 2 or 3 HIP streams: how much of a transform's launch ramp and store tail the
next batch's transform can fill (profiles/r03/ntt_experiments/timeline_*.txt)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, sys.argv[1] if len(sys.argv) > 1 else "phantom-fhe-boot_amd/py")
import phantom_amd as PA  # noqa: E402

N, L = 1 << 16, 44
lib = PA.load()
mods = PA.coeff_modulus_create(N, [60] + [50] * 44 + [60] * 15)[:L]
t = PA.NttTables(N, mods)
rng = np.random.default_rng(0x5EED)
base = np.concatenate([rng.integers(0, q, size=N, dtype=np.uint64) for q in mods])
ring = [torch.from_numpy(base.view(np.int64).copy()).cuda() for _ in range(12)]  # 12: each buffer stays on one stream for 1, 2, 3 or 4 streams
BYTES = 2 * 16 * N * L  # fwd + inv, 16 B per coefficient per transform


def run(nstreams, steps=400, warm=40):
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    cur = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(cur)

    def step(i):
        s = streams[i % nstreams]
        d = ring[i % 12].data_ptr()
        PA.check(lib.phantom_nwt_forward_inplace(d, t.handle, L, 0, s.cuda_stream))
        PA.check(lib.phantom_nwt_backward_inplace(d, t.handle, L, 0, s.cuda_stream))

    for i in range(warm):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return steps * BYTES / dt / 1e9, dt / steps * 1e6


for k in (1, 2, 3, 4, 1, 2, 3, 4):
    gbs, us = run(k)
    print(f"streams {k}: {gbs:8.1f} GB/s  {us:6.2f} us/step", flush=True)
h = ring[0].cpu().numpy().view(np.uint64)
print("round trip exact:", bool(np.array_equal(h, base)))
