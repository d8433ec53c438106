"""A/B timing of one forward / inverse NTT across library builds, one process per build and
repetition (alternating, so box drift hits every build alike).  Per build: median of
HIP-event-bracketed single transforms on one stream over a 15-buffer ring (cold HBM), the
back-to-back means, and a checksum of the forward output (equal = bit-identical) plus an exact
round-trip flag.  NTT_BITS=60 uses the 40-limb C4 chain (integer path), 50 the C2 batch.

  python tools/ntt_ab.py <py dir of build A> <py dir of build B> ...
A build may carry environment settings: <py dir>@NAME=value,NAME2=value (e.g. a run-time knob of one
library).  NTT_REP=k repeats the moduli k times (a k times larger launch of the same primes).
"""
import json
import os
import subprocess
import sys

CODE = r'''
import sys, os, time, numpy as np, torch
sys.path.insert(0, sys.argv[1])
import phantom_amd as PA
N, L = 1 << 16, 44
lib = PA.load()
if os.environ.get("NTT_BITS", "50") == "60":
    L = 40
    mods = PA.coeff_modulus_create(N, [60] + [59] * 29 + [60] * 10)
else:
    mods = PA.coeff_modulus_create(N, [60] + [50] * 44 + [60] * 15)[:L]
mods = mods * int(os.environ.get("NTT_REP", "1"))
L = len(mods)
t = PA.NttTables(N, mods)
rng = np.random.default_rng(1)
base = np.concatenate([rng.integers(0, q, size=N, dtype=np.uint64) for q in mods])
NB = 15  # 15 x 23 MB > 256 MB Infinity Cache
ring = [torch.from_numpy(base.view(np.int64)).cuda() for _ in range(NB)]
s = torch.cuda.current_stream()
F, I = lib.phantom_nwt_forward_inplace, lib.phantom_nwt_backward_inplace
def single(fn, iters=80):
    evs = []
    for i in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s); PA.check(fn(ring[i % NB].data_ptr(), t.handle, L, 0, s.cuda_stream)); b.record(s)
        evs.append((a, b))
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in evs[10:])
    return ts[len(ts) // 2]
def b2b(fns, iters=200):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(10):
        for fn in fns: PA.check(fn(ring[i % NB].data_ptr(), t.handle, L, 0, s.cuda_stream))
    torch.cuda.synchronize()
    h0 = time.perf_counter()
    a.record(s)
    for i in range(iters):
        for fn in fns: PA.check(fn(ring[i % NB].data_ptr(), t.handle, L, 0, s.cuda_stream))
    b.record(s)
    host = (time.perf_counter() - h0) * 1e6 / iters
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters, host
chk = torch.from_numpy(base.view(np.int64)).cuda()
PA.check(F(chk.data_ptr(), t.handle, L, 0, s.cuda_stream))
torch.cuda.synchronize()
h = chk.cpu().numpy().view(np.uint64)
csum = int(np.bitwise_xor.reduce(h * np.arange(1, len(h) + 1, dtype=np.uint64)))
PA.check(I(chk.data_ptr(), t.handle, L, 0, s.cuda_stream))
torch.cuda.synchronize()
rt = bool(np.array_equal(chk.cpu().numpy().view(np.uint64), base))
fs, is_ = single(F), single(I)
fb, fh = b2b([F]); ib, ih = b2b([I]); sb, sh = b2b([F, I])
print("RESULT", fs, is_, fb, ib, sb, fh, sh, csum & 0xffffffff, int(rt))
'''


def main():
    dirs = sys.argv[1:]
    res = {d: [] for d in dirs}
    for rep in range(int(os.environ.get("REPS", "3"))):
        for d in dirs:
            path, _, envs = d.partition("@")
            env = dict(os.environ)
            env.update(dict(kv.split("=", 1) for kv in envs.split(",") if kv))
            out = subprocess.run([sys.executable, "-c", CODE, path], capture_output=True, text=True, timeout=240, env=env)
            line = [l for l in out.stdout.splitlines() if l.startswith("RESULT")]
            if not line:
                print(d, "ERROR", out.stderr[-600:], flush=True)
                sys.exit(1)
            v = line[0].split()[1:]
            r = dict(zip(["fwd_us", "inv_us", "fwd_b2b_us", "inv_b2b_us", "step_b2b_us", "host_fwd_us", "host_step_us"],
                         [round(float(x), 2) for x in v[:7]]))
            r["checksum"] = int(v[7])
            r["round_trip"] = bool(int(v[8]))
            res[d].append(r)
            print(json.dumps({"build": d, "rep": rep, **r}), flush=True)
    print(json.dumps({"bits": os.environ.get("NTT_BITS", "50"), "summary": {
        d: {k: sorted(x[k] for x in rs) for k in ("fwd_us", "inv_us", "step_b2b_us")} for d, rs in res.items()}}))


if __name__ == "__main__":
    main()
