"""Time one forward / inverse NTT under different limb-chunk pipelines (PHX_NTT_PIPE, csrc/ntt.hip),
one process per setting.  Per setting: median of HIP-event-bracketed single transforms on one
caller stream, the back-to-back mean, the fwd+inv step rate on one stream, and a checksum of the
forward output (equal = bit-identical).  NTT_BITS=60 uses the 40-limb C4 chain.

  python tools/ntt_pipe.py "0" "2,2" "3,3" "4,2" ...
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
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
    settings = sys.argv[1:] or ["0", "2,2", "3,3", "4,2", "4,4"]
    py = os.path.join(ROOT, "phantom-fhe-boot_amd", "py")
    res = {}
    for rep in range(int(os.environ.get("REPS", "2"))):
        for st in settings:
            env = dict(os.environ, PHX_NTT_PIPE=st)
            out = subprocess.run([sys.executable, "-c", CODE, py], capture_output=True, text=True, timeout=240, env=env)
            line = [l for l in out.stdout.splitlines() if l.startswith("RESULT")]
            if not line:
                print(st, "ERROR", out.stderr[-600:], flush=True)
                sys.exit(1)
            v = line[0].split()[1:]
            r = {"fwd_us": round(float(v[0]), 2), "inv_us": round(float(v[1]), 2), "fwd_b2b_us": round(float(v[2]), 2),
                 "inv_b2b_us": round(float(v[3]), 2), "step_b2b_us": round(float(v[4]), 2),
                 "host_fwd_us": round(float(v[5]), 2), "host_step_us": round(float(v[6]), 2),
                 "check": v[7], "roundtrip": v[8] == "1"}
            res.setdefault(st, []).append(r)
            print(f"rep {rep} pipe {st:>8}: {r}", flush=True)
    tag = os.environ.get("NTT_BITS", "50")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", f"ntt_pipe_{tag}.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
