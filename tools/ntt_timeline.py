"""Per-wave timeline of the forward NTT passes from a PHX_NTT_STAMP=1 build (diagnostic only).

usage: python tools/ntt_timeline.py tools/variants/stamp/py [BITS]
Each wave of the forward column and row passes stamps s_memrealtime (10 ns ticks, chip-wide) at
entry, data arrived, butterflies done, stores issued and stores complete (csrc/ntt.hip
PHX_NTT_STAMP).  Prints per pass: the span, phase-duration percentiles, and a 0.5 us binned count of
waves in each phase (waiting for data / computing / storing), i.e. how much of the pass overlaps
memory with compute.
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, sys.argv[1])
import torch  # noqa: E402
import phantom_amd as PA  # noqa: E402

BITS = sys.argv[2] if len(sys.argv) > 2 else "50"
N = 1 << 16
lib = PA.load()
if BITS == "60":
    L = 40
    mods = PA.coeff_modulus_create(N, [60] + [59] * 29 + [60] * 10)
else:
    L = 44
    mods = PA.coeff_modulus_create(N, [60] + [50] * 44 + [60] * 15)[:L]
t = PA.NttTables(N, mods)
rng = np.random.default_rng(1)
base = np.concatenate([rng.integers(0, q, size=N, dtype=np.uint64) for q in mods])
ring = [torch.from_numpy(base.view(np.int64)).cuda() for _ in range(15)]
s = torch.cuda.current_stream().cuda_stream
for i in range(30):
    PA.check(lib.phantom_nwt_forward_inplace(ring[i % 15].data_ptr(), t.handle, L, 0, s))
torch.cuda.synchronize()
lib.phantom_debug_ntt_stamps_clear.restype = ctypes.c_int
lib.phantom_debug_ntt_stamps.restype = ctypes.c_int
lib.phantom_debug_ntt_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
SLOTS, ROW = 32768, 16384
assert lib.phantom_debug_ntt_stamps_clear() == 0
torch.cuda.synchronize()
# back to back (a busy GPU, as in the bench); the last forward's stamps remain
BACK = int(os.environ.get("BACK", "8"))
for i in range(BACK):
    PA.check(lib.phantom_nwt_forward_inplace(ring[i % 15].data_ptr(), t.handle, L, 0, s))
torch.cuda.synchronize()
buf = np.zeros(SLOTS * 8, dtype=np.uint64)
assert lib.phantom_debug_ntt_stamps(buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(SLOTS, 8)


def report(name, rows):
    rows = rows[rows[:, 0] > 0]
    if len(rows) == 0:
        print(name, "no stamps")
        return
    t0 = rows[:, 0].min()
    tt = (rows[:, :5].astype(np.int64) - int(t0)) * 0.01  # us
    span = tt[:, 4].max()
    wait, comp, issue, drain = tt[:, 1] - tt[:, 0], tt[:, 2] - tt[:, 1], tt[:, 3] - tt[:, 2], tt[:, 4] - tt[:, 3]
    pct = lambda a: " ".join(f"{np.percentile(a, p):6.2f}" for p in (5, 50, 95))
    print(f"== {name}: {len(rows)} waves, span {span:.2f} us")
    print(f"   entry     p5/50/95 {pct(tt[:, 0])}")
    print(f"   data wait          {pct(wait)}")
    print(f"   compute            {pct(comp)}")
    print(f"   store issue        {pct(issue)}")
    print(f"   store drain        {pct(drain)}")
    print(f"   done               {pct(tt[:, 4])}")
    cu = (rows[:, 6].astype(np.int64) << 16) | ((rows[:, 5].astype(np.int64) >> 8) & 0xFF)
    print(f"   distinct (xcc, se/sh/cu): {len(np.unique(cu))}")
    print("   bin(us)  waiting computing storing done")
    for b in np.arange(0, span + 0.5, 0.5):
        mid = b + 0.25
        w = np.sum((tt[:, 0] <= mid) & (tt[:, 1] > mid))
        c = np.sum((tt[:, 1] <= mid) & (tt[:, 2] > mid))
        so = np.sum((tt[:, 2] <= mid) & (tt[:, 4] > mid))
        d = np.sum(tt[:, 4] <= mid)
        print(f"   {b:5.1f}  {w:7d} {c:9d} {so:7d} {d:5d}")


report("column pass", st[:ROW])
report("row pass", st[ROW:])
