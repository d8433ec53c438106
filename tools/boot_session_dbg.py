"""Debug driver: one bootstrap through the session C-ABI (num_slots / iterations from argv)."""
import sys
import os
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "phantom-fhe-boot_amd", "py"))
import numpy as np
import torch
import phantom_amd as PA

slots = int(sys.argv[1]) if len(sys.argv) > 1 else 0
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 1
prec = int(sys.argv[3]) if len(sys.argv) > 3 else 0
lanes = int(sys.argv[4]) if len(sys.argv) > 4 else 1
count = int(sys.argv[5]) if len(sys.argv) > 5 else 1
t = time.time()
s = PA.BootSession(bytes(range(32)), num_slots=slots, iterations=iters, precision=prec)
print("setup", round(time.time() - t, 2), "slots", s.slots, flush=True)
rng = np.random.default_rng(1)
vals = rng.uniform(1, 5, size=(count, s.slots))
sin, sout = s.input_bytes(26), s.output_bytes()
di = torch.empty((count, sin), dtype=torch.uint8, device="cuda")
do = torch.empty((count, sout), dtype=torch.uint8, device="cuda")
s.encrypt(vals, 26, di.data_ptr(), sin)
print("in bits", PA.bit_precision(vals[0], s.decrypt(di[0].data_ptr(), sin)), flush=True)
for rep in range(2):
    t = time.time()
    s.run(di.data_ptr(), sin, count, do.data_ptr(), sout, lanes)
    torch.cuda.synchronize()
    print("run", rep, round((time.time() - t) * 1e3, 1), "ms", flush=True)
print("out bits", [round(PA.bit_precision(vals[i], s.decrypt(do[i].data_ptr(), sout)), 2) for i in range(count)], flush=True)
s.close()
