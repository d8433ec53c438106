"""Summarise `bootstrapping_example tail` output (per-coefficient bootstrap error probe).

Per key: s(zeta) (the secret at the first slot's root), the median error of coefficient 0 (the
input's mean), the errors of coefficients 0 and N/2 (the two halves of CoeffToSlot's slot 0) when
one of them has overflow I = 0, the error of the other coefficients with I = 0, and the
precision range.  Across keys: how those slot-0 offsets follow s(zeta).

  python tools/tail_analysis.py gpurun_out/.../tail_keys.txt
"""
import json
import sys

import numpy as np


def main():
    keys, rows = {}, []
    for line in open(sys.argv[1]):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if "s_zeta" in d:
            keys[d["key"]] = d
        elif "tail" in d:
            rows.append(d)
    out = []
    for k, kd in sorted(keys.items()):
        rs = [r for r in rows if r["key"] == k]
        if not rs:
            continue
        e0 = np.array([r["e0"] for r in rs])
        med = float(np.median(e0))
        i0 = [r["e0"] - med for r in rs if r["I0"] == 0]
        ih = [r["e_half"] for r in rs if r["I_half"] == 0]
        ih0 = [r["e0"] - med for r in rs if r["I_half"] == 0]
        zo = [r["I_zero_others"] for r in rs]
        rec = {
            "key": k, "s_zeta": kd["s_zeta"], "ciphertexts": len(rs),
            "bits_min": min(r["avg_bits"] for r in rs), "bits_mean": round(float(np.mean([r["avg_bits"] for r in rs])), 3),
            "e0_median": med,
            "I0_is_0": {"n": len(i0), "e0_minus_median": [round(x, 5) for x in i0],
                        "e_half": [round(r["e_half"], 5) for r in rs if r["I0"] == 0]},
            "Ihalf_is_0": {"n": len(ih), "e_half": [round(x, 5) for x in ih], "e0_minus_median": [round(x, 5) for x in ih0]},
            "other_I0_coeffs_mean_max": [float(np.mean([z[1] for z in zo])), float(max(z[2] for z in zo))],
            "repeat_unequal": sum(not r["repeat_equal"] for r in rs),
            "reencrypted_e0_median": float(np.median([r["e0_reencrypted"] for r in rs])),
            "top_share_median": float(np.median([r["top_err_share"] for r in rs])),
        }
        out.append(rec)
        print(json.dumps(rec))
    bits = [r["avg_bits"] for r in rows]
    worst = sorted(rows, key=lambda r: r["avg_bits"])[:10]
    print(json.dumps({"ciphertexts": len(rows), "bits_min": min(bits), "bits_mean": round(float(np.mean(bits)), 3),
                      "worst": [{"key": r["key"], "bits": r["avg_bits"], "I0": r["I0"], "I_half": r["I_half"],
                                 "e0": r["e0"], "e_half": r["e_half"]} for r in worst],
                      "worst_with_I0_or_Ihalf_zero": sum(r["I0"] == 0 or r["I_half"] == 0 for r in worst)}))


if __name__ == "__main__":
    main()
