"""The runtime switches that select alternative product code, each exercised once against its
oracle tests in a child process with the switch set (each is read once per process):

  PHX_KS_EPI=0        the key-switch inner product as its own kernel instead of inside the moddown's
                      INTT prologue / NTT epilogue            -> relinearize / key-switch tests
  PHX_FUSED_BCONV=1   base conversion as the NTT column pass's prologue
                                                              -> modup / moddown / relinearize tests
  PHX_BCONV_MFMA=0    every base conversion on the VALU kernel -> base-conversion + relinearize tests
  PHX_LT_SQUARE=1     the square baby-step / giant-step split  -> full bootstrap precision and levels

Debug aids (PHX_BOOT_TRACE, PHX_DEBUG_SYNC) change no results and are not listed."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pytest(env_kv, *args):
    env = dict(os.environ, **env_kv)
    cmd = [sys.executable, "-m", "pytest", "-q", "-m", "gpu", "-p", "no:cacheprovider", *args]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    tail = (out.stdout + out.stderr)[-3000:]
    assert out.returncode == 0, tail
    assert " passed" in out.stdout and " failed" not in out.stdout, tail


def test_ks_inner_product_kernel():
    _pytest({"PHX_KS_EPI": "0"}, "tests/test_gpu_ckks.py", "-k", "relinearize or keyswitch")


def test_fused_bconv_prologue():
    _pytest({"PHX_FUSED_BCONV": "1"}, "tests/test_gpu_ckks.py", "-k", "modup or moddown or relinearize")


def test_bconv_valu_everywhere():
    _pytest({"PHX_BCONV_MFMA": "0"}, "tests/test_gpu_bconv.py", "tests/test_gpu_ckks.py", "-k",
            "bconv or relinearize or moddown")


def test_lt_square_split_bootstrap():
    env = dict(os.environ, PHX_LT_SQUARE="1")
    exe = os.path.join(ROOT, "phantom-fhe-boot_amd", "bin", "bootstrapping_example")
    out = subprocess.run([exe, "boot", "16", "1"], env=env, capture_output=True, text=True, timeout=200)
    assert out.returncode == 0, out.stderr[-2000:]
    rows = [json.loads(l) for l in out.stdout.splitlines() if l.startswith('{"stage": "bootstrap"')]
    assert rows and rows[0]["avg_bits"] > 9.85 and rows[0]["levels_after"] == 11, rows
