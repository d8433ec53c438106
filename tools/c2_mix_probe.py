"""Does the C2 batch's one 60-bit limb (integer path, about twice the VALU of an FP64 limb) set
the forward NTT's duration?  Median single-launch time (HIP events, 15-buffer cold ring) of the
forward and inverse NTT over: the C2 moduli (q0 60-bit + 43 x 50-bit), 44 x 50-bit, 43 x 50-bit,
and the 60-bit limb alone."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, sys.argv[1] if len(sys.argv) > 1 else "phantom-fhe-boot_amd/py")
import phantom_amd as PA  # noqa: E402

N = 1 << 16
lib = PA.load()
allm = PA.coeff_modulus_create(N, [60] + [50] * 44 + [60] * 15)
cases = {"c2_mixed_44": allm[:44], "fp64_44": allm[1:45], "fp64_43": allm[1:44], "int_1": allm[:1],
         "int_first_then_fp64_44": allm[:45]}
s = torch.cuda.current_stream()
F, I = lib.phantom_nwt_forward_inplace, lib.phantom_nwt_backward_inplace
out = {}
for rep in range(3):
    for name, mods in cases.items():
        L = len(mods)
        t = PA.NttTables(N, mods)
        rng = np.random.default_rng(1)
        base = np.concatenate([rng.integers(0, q, size=N, dtype=np.uint64) for q in mods])
        ring = [torch.from_numpy(base.view(np.int64)).cuda() for _ in range(15)]

        def single(fn, iters=80):
            evs = []
            for i in range(iters):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                PA.check(fn(ring[i % 15].data_ptr(), t.handle, L, 0, s.cuda_stream))
                b.record(s)
                evs.append((a, b))
            torch.cuda.synchronize()
            ts = sorted(a.elapsed_time(b) * 1e3 for a, b in evs[10:])
            return ts[len(ts) // 2]
        out.setdefault(name, []).append((round(single(F), 2), round(single(I), 2)))
        del ring
        t.close()
        torch.cuda.synchronize()
print(json.dumps(out))
