"""Distribution of the two-iteration bootstrap's precision over fresh encryptions (the encryptor
draws from OS entropy; the key seed is the tests' bytes(range(32))).  One BootSession per setting,
`COUNT` ciphertexts each.  usage: python tools/two_iter_dist.py [COUNT]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "phantom-fhe-boot_amd", "py"))
import phantom_amd as PA  # noqa: E402


def run(iterations, precision, count, chain=26, lanes=2):
    sess = PA.BootSession(bytes(range(32)), num_slots=0, iterations=iterations, precision=precision)
    rng = np.random.default_rng(0xB0 + iterations)
    vals = rng.uniform(1.0, 5.0, size=(count, sess.slots))
    sin, sout = sess.input_bytes(chain), sess.output_bytes()
    dev_in = torch.empty((count, sin), dtype=torch.uint8, device="cuda")
    dev_out = torch.empty((count, sout), dtype=torch.uint8, device="cuda")
    assert sess.encrypt(vals, chain, dev_in.data_ptr(), sin) == sin
    sess.run(dev_in.data_ptr(), sin, count, dev_out.data_ptr(), sout, lanes)
    torch.cuda.synchronize()
    bits = [PA.bit_precision(vals[i], sess.decrypt(dev_out[i].data_ptr(), sout)) for i in range(count)]
    sess.close()
    return bits


if __name__ == "__main__":
    torch.cuda.set_device(0)
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    for it, prec in ((1, 0), (2, 8)):
        b = run(it, prec, count)
        print(json.dumps({"iterations": it, "precision": prec, "count": count, "min": round(min(b), 2),
                          "median": round(float(np.median(b)), 2), "max": round(max(b), 2),
                          "bits": [round(x, 2) for x in sorted(b)]}), flush=True)
