"""EvalChebyshevSeries through the reference's Paterson-Stockmeyer split (host/chebyshev_ps.cpp:
src/evaluate.cu:2998-3535, src/util.cu:15-312) at every degree 5..119 on three intervals, N = 2^13
on the C4 modulus shape: the levels it consumes (a pending rescale counted) equal the reference's
GetDepthByDegree(d) (src/util.cu:44-71) whenever the affine map runs, and one less on [-1, 1] where
the reference skips it (src/evaluate.cu:3282-3297); the decrypted value matches the host evaluation
of the same interpolant."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "phantom-fhe-boot_amd", "bin", "bootstrapping_example")


def test_chebyshev_series_levels_match_get_depth_by_degree():
    out = subprocess.run([EXE, "chebdepth", "13"], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    rows = [json.loads(l) for l in out.stdout.splitlines() if l.startswith('{"cheb"')]
    assert len(rows) == 3 * 115
    for r in rows:
        unit = (r["a"], r["b"]) == (-1, 1)
        assert r["levels_used"] == r["depth_by_degree"] - (1 if unit else 0), r
        assert r["max_abs_err"] < 1e-9, r
