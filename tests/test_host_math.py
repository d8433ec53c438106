"""CPU-only checks of the bootstrap's host mathematics (phantom-fhe-boot_amd/examples/host_math_test.cpp):
canonical embedding round trip, the SlotToCoeff / CoeffToSlot stage factorisation against the
encoder's embedding, grouped stage composition, and the EvalMod Chebyshev + double-angle
approximation of sin(2 pi K y) / (2 pi) (K = 512, r = 6, degree 88: the reference's
bootstrap.cuh:201-255 parameters).  No GPU is touched."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "phantom-fhe-boot_amd", "bin", "host_math_test")


def test_bootstrap_host_math():
    out = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert out.returncode == 0 and res["ok"], res
    assert res["stc_stages"] < 1e-9 and res["cts_stages"] < 1e-9
    assert res["evalmod_after_double_angle"] < 1e-8
