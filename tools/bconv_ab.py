"""A/B timing of the base conversion across library builds (one process per build and repetition,
alternating): phantom_bconv_run through one kept converter, median of HIP-event-timed calls over a
ring of inputs larger than the Infinity Cache, per shape; GB/s = (ibase + obase) limbs x n x 8 B /
time, and a checksum of the output (equal = bit-identical).

  python tools/bconv_ab.py <py dir of build A> <py dir of build B> ...
"""
import json
import os
import subprocess
import sys

CODE = r'''
import ctypes, sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
import phantom_amd as PA
lib = PA.load()
n = 1 << 16
s = torch.cuda.current_stream()
# (ibase bits, obase bits): the C3 digit (15 -> 45), the C4 digit at Ql 30 (10 -> 30) and the
# moddown P -> Ql of C4 (10 -> 30), the C3 moddown (15 -> 45 over 2 polys as one call of 2n)
shapes = [("c3_digit", [50] * 15, [50] * 30 + [60] * 15, 1), ("c4_digit", [59] * 10, [59] * 20 + [60] * 10, 1),
          ("c4_moddown_2polys", [60] * 10, [59] * 30, 2)]
res = {}
for name, ib_bits, ob_bits, polys in shapes:
    mods = PA.coeff_modulus_create(n, ib_bits + ob_bits)
    ib = np.array(mods[:len(ib_bits)], dtype=np.uint64)
    ob = np.array(mods[len(ib_bits):], dtype=np.uint64)
    h = ctypes.c_void_p()
    PA.check(lib.phantom_bconv_create(ib.ctypes.data_as(PA.u64p), len(ib), ob.ctypes.data_as(PA.u64p), len(ob),
                                      s.cuda_stream, ctypes.byref(h)))
    rng = np.random.default_rng(7)
    nn = n * polys
    # inputs: polys x [ib][n] laid out as [ib][nn] (the conversion reads limb-major rows of nn)
    ring_n = max(2, (600 << 20) // ((len(ib) + len(ob)) * nn * 8))
    ins = []
    for _ in range(ring_n):
        x = np.concatenate([rng.integers(0, q, size=nn, dtype=np.uint64) for q in ib])
        ins.append(torch.from_numpy(x.view(np.int64)).cuda())
    outs = [torch.empty(len(ob) * nn, dtype=torch.int64, device="cuda") for _ in range(ring_n)]
    for i in range(10):
        PA.check(lib.phantom_bconv_run(h, ins[i % ring_n].data_ptr(), outs[i % ring_n].data_ptr(), nn, 1, s.cuda_stream))
    torch.cuda.synchronize()
    ts = []
    for i in range(120):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        PA.check(lib.phantom_bconv_run(h, ins[i % ring_n].data_ptr(), outs[i % ring_n].data_ptr(), nn, 1, s.cuda_stream))
        b.record(s)
        ts.append((a, b))
    torch.cuda.synchronize()
    us = sorted(a.elapsed_time(b) * 1e3 for a, b in ts)[len(ts) // 2]
    o = outs[0].cpu().numpy().view(np.uint64)
    csum = int(np.bitwise_xor.reduce(o * np.arange(1, len(o) + 1, dtype=np.uint64))) & 0xffffffff
    res[name] = {"us": round(us, 2), "GBps": round((len(ib) + len(ob)) * nn * 8 / us / 1e3, 1), "checksum": csum}
    PA.check(lib.phantom_bconv_destroy(h))
print("RESULT " + __import__("json").dumps(res))
'''


def main():
    dirs = sys.argv[1:]
    allres = {d: [] for d in dirs}
    for rep in range(int(os.environ.get("REPS", "3"))):
        for d in dirs:
            out = subprocess.run([sys.executable, "-c", CODE, d], capture_output=True, text=True, timeout=240)
            line = [l for l in out.stdout.splitlines() if l.startswith("RESULT")]
            if not line:
                print(d, "ERROR", out.stderr[-800:], flush=True)
                sys.exit(1)
            r = json.loads(line[0][7:])
            allres[d].append(r)
            print(json.dumps({"build": d, "rep": rep, **r}), flush=True)
    print(json.dumps({"summary": {d: {k: sorted(x[k]["us"] for x in rs) for k in rs[0]} for d, rs in allres.items()}}))


if __name__ == "__main__":
    main()
