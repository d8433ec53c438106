"""Generates tests/golden/eval_mod_coefficients.json: the two Chebyshev coefficient tables the
reference ships for EvalMod (include/bootstrap.cuh:217-255, g_coefficientsSparse and
g_coefficientsUniform, originally from OpenFHE), read from the reference tree as numeric data.
Run in the build container (the GPU box has no /root/reference):
    python tests/golden/make_eval_mod_coefficients.py /root/reference/include/bootstrap.cuh"""
import json
import os
import re
import sys


def table(text, name):
    m = re.search(name + r"\s*\{([^}]*)\}", text)
    if not m:
        raise SystemExit(f"{name} not found")
    return [float(x) for x in re.findall(r"[-+]?\d+\.\d+(?:[eE][-+]?\d+)?", m.group(1))]


def main(path):
    text = open(path).read()
    out = {
        "source": "include/bootstrap.cuh:217-255 of alexlee838/phantom-fhe-boot",
        "convention": "p(y) = c[0]/2 + sum_{k>=1} c[k] T_k(y) (src/evaluate.cu:3259 adds coefficients[0] / 2)",
        "uniform": {"K": 512, "double_angle_iterations": 6, "coefficients": table(text, "g_coefficientsUniform")},
        "sparse": {"K": 28, "double_angle_iterations": 3, "coefficients": table(text, "g_coefficientsSparse")},
    }
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "eval_mod_coefficients.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(dst, len(out["uniform"]["coefficients"]), len(out["sparse"]["coefficients"]))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/include/bootstrap.cuh")
