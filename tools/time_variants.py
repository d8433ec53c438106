"""Time the forward/inverse NTT of each library variant under tools/variants/ (one process each)."""
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
BITS = os.environ.get("NTT_BITS", "50")
if BITS == "60":  # the C4 chain: Q = {60, 29 x 59}, P = 10 x 60 (bootstrapping_example.cu:69-116)
    L = 40
    mods = PA.coeff_modulus_create(N, [60] + [59] * 29 + [60] * 10)
else:
    mods = PA.coeff_modulus_create(N, [60] + [50] * 44 + [60] * 15)[:L]
t = PA.NttTables(N, mods)
rng = np.random.default_rng(1)
base = np.concatenate([rng.integers(0, q, size=N, dtype=np.uint64) for q in mods])
ring = [torch.from_numpy(base.view(np.int64)).cuda() for _ in range(15)]
s = torch.cuda.current_stream()
def run(fn, iters=60):
    evs = []
    for i in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s); PA.check(fn(ring[i % 15].data_ptr(), t.handle, L, 0, s.cuda_stream)); b.record(s)
        evs.append((a, b))
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in evs[10:])
    return ts[len(ts) // 2]
fwd = run(lib.phantom_nwt_forward_inplace)
inv = run(lib.phantom_nwt_backward_inplace)
def b2b(fn, iters=150):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(10): PA.check(fn(ring[i % 15].data_ptr(), t.handle, L, 0, s.cuda_stream))
    a.record(s)
    for i in range(iters): PA.check(fn(ring[i % 15].data_ptr(), t.handle, L, 0, s.cuda_stream))
    b.record(s); torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters
chk = torch.from_numpy(base.view(np.int64)).cuda()
PA.check(lib.phantom_nwt_forward_inplace(chk.data_ptr(), t.handle, L, 0, s.cuda_stream))
torch.cuda.synchronize()
h = chk.cpu().numpy().view(np.uint64)
csum = int(np.bitwise_xor.reduce(h * np.arange(1, len(h) + 1, dtype=np.uint64)))
print("CHECK", csum)
print("RESULT", fwd, inv, b2b(lib.phantom_nwt_forward_inplace), b2b(lib.phantom_nwt_backward_inplace))
'''
res = {}
for name in sorted(os.listdir(os.path.join(ROOT, "tools", "variants"))):
    py = os.path.join(ROOT, "tools", "variants", name, "py")
    out = subprocess.run([sys.executable, "-c", CODE, py], capture_output=True, text=True, timeout=300, env=dict(os.environ))
    line = [l for l in out.stdout.splitlines() if l.startswith("RESULT")]
    if line:
        f, i, fb, ib = map(float, line[0].split()[1:])
        res[name] = {"fwd_us": round(f, 2), "inv_us": round(i, 2), "fwd_b2b_us": round(fb, 2), "inv_b2b_us": round(ib, 2)}
        chk = [l for l in out.stdout.splitlines() if l.startswith("CHECK")]
        res[name]["check"] = chk[0].split()[1][-8:] if chk else None
    else:
        res[name] = {"error": out.stderr[-500:]}
    print(name, res[name], flush=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "variants_%s.json" % os.environ.get("NTT_BITS", "50")), "w"), indent=1)
