"""The reference's examples/3_ckks.cu through this engine's C++ façade
(phantom-fhe-boot_amd/examples/ckks_example.cpp): the same calls in the same order —
PhantomSecretKey(context) + gen_publickey, encode/decode, encrypt_symmetric / encrypt_asymmetric,
add / sub, multiply_plain, the x*y*x HomMul with relinearize_inplace / rescale_to_next_inplace /
mod_switch_to_next_inplace, EvalRotateKeyGen + EvalRotateFused / EvalConjFused, and the
small-parameter apply_galois_inplace, and the seed-compressed save_symmetric /
load_symmetric round trip, and (ckks_api) the rest of include/evaluate.cuh's CKKS surface: add_many,
add/sub_plain, the squaring branch of multiply (bit-identical to the product of two copies),
multiply_and_relin, plaintext mod_switch_to(_next), hoisting_inplace, NAF-composed rotations,
save_symmetric refusing a rewritten c1, from_seed keys with independent encryption randomness — each checked with the reference's own rule (every slot
within 1e-3, 3_ckks.cu:19,33-41).  Keys come from the OS entropy path (no test seed)."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "phantom-fhe-boot_amd", "bin", "ckks_example")
EXAMPLES = ["ckks_enc", "ckks_add", "ckks_save_symmetric", "ckks_mul_plain", "ckks_mul", "ckks_rotation", "ckks_api"]


@pytest.mark.parametrize("alpha", [15, 1, 3])
def test_3_ckks_examples(alpha):
    """alpha 15: the C3 chain (N = 2^16, Q = {60, 44 x 50}, P = 15 x 60); alpha 1 and 3: the
    reference's N = 2^15, 40-bit-prime sets with 1 and 3 special primes (dnum 19 and 5)."""
    out = subprocess.run([BIN, str(alpha), "--seed", str(alpha)], capture_output=True, text=True, timeout=110)
    rows = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    got = {r["example"]: r for r in rows if "example" in r}
    assert out.returncode == 0, (rows, out.stderr[-2000:])
    for name in EXAMPLES:
        assert got[name]["ok"] and got[name]["alpha"] == alpha, got[name]
    assert got["ckks_small_param"]["ok"], got["ckks_small_param"]
    # PhantomGaloisKey::save / load in the reference's bytes (secretkey.h:195-220), parsed field by field
    assert got["ckks_galois_key_layout"]["ok"], got["ckks_galois_key_layout"]
