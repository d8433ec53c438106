"""Host-side enqueue time of each C3 op (bench.c3_leg's calls) while the device works: the mean
wall time of each C-ABI call over `ITERS` chained multiply -> relinearize -> rescale sequences,
without synchronising inside the loop, plus the device time of the whole chain."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "phantom-fhe-boot_amd", "py"))
import torch  # noqa: E402
import bench  # noqa: E402
import phantom_amd as PA  # noqa: E402

lib = PA.load()
N = bench.N
mods = PA.coeff_modulus_create(N, bench.C3_BITS)
ctx = PA.Context(N, mods, 15)
rng = np.random.default_rng(1)
rand = lambda ms, p: torch.from_numpy(np.concatenate([rng.integers(0, q, size=N, dtype=np.uint64) for _ in range(p) for q in ms]).view(np.int64)).cuda()
ct1, ct2 = rand(mods[:45], 2), rand(mods[:45], 2)
keys = [rand(mods, 2) for _ in range(3)]
kp = PA.ptr_array([k.data_ptr() for k in keys])
prod = torch.empty(3 * 45 * N, dtype=torch.int64, device="cuda")
resc = torch.empty(2 * 44 * N, dtype=torch.int64, device="cuda")
sh = torch.cuda.current_stream().cuda_stream
ops = [("multiply", lambda: lib.phantom_multiply(ctx.handle, 1, ct1.data_ptr(), ct2.data_ptr(), prod.data_ptr(), sh)),
       ("relinearize", lambda: lib.phantom_relinearize(ctx.handle, 1, prod.data_ptr(), kp, 3, sh)),
       ("rescale", lambda: lib.phantom_rescale_to_next(ctx.handle, 1, prod.data_ptr(), resc.data_ptr(), 2, sh))]
for _ in range(5):
    for _, f in ops:
        f()
torch.cuda.synchronize()
iters = int(os.environ.get("ITERS", "50"))
host = {k: 0.0 for k, _ in ops}
t0 = time.perf_counter()
for _ in range(iters):
    for k, f in ops:
        a = time.perf_counter()
        f()
        host[k] += time.perf_counter() - a
t_enq = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
print({"host_us_per_call": {k: round(v / iters * 1e6, 2) for k, v in host.items()},
       "enqueue_us_per_chain": round(t_enq / iters * 1e6, 2), "wall_us_per_chain": round(t_all / iters * 1e6, 2)})
