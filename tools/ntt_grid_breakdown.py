"""NTT launches of the last warm window of a rocprofv3 csv kernel trace, grouped by kernel and
workgroup count (16 workgroups per 2^16 limb at S1 = S2 = 256): calls, mean duration, µs per limb.

usage: python tools/ntt_grid_breakdown.py run_kernel_trace.csv [gap_us]"""
import collections
import csv
import re
import sys


def main(path, gap_us=300.0):
    ks = []
    for r in csv.DictReader(open(path)):
        ks.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])))
    ks.sort(key=lambda k: k[1])
    cut, run_end = 0, ks[0][2]
    for i in range(1, len(ks)):
        if ks[i][1] - run_end > gap_us * 1e3:
            cut = i
        run_end = max(run_end, ks[i][2])
    agg = collections.defaultdict(lambda: [0, 0])
    tot_all = sum(e - s for _, s, e, _ in ks[cut:])
    for name, s, e, wg in ks[cut:]:
        m = re.search(r"(ntt_(?:col|row)<[^>]*>)", name)
        if not m:
            continue
        agg[(m.group(1), wg)][0] += 1
        agg[(m.group(1), wg)][1] += e - s
    tot = sum(t for _, t in agg.values())
    print(f"# NTT {tot / 1e6:.2f} ms of {tot_all / 1e6:.2f} ms kernel time in the window")
    for (k, wg), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:36s} limbs={wg / 16:5.1f} calls={c:4d} avg={t / c / 1e3:7.2f}us "
              f"per_limb={t / c / 1e3 / (wg / 16):5.2f}us total={t / 1e6:6.2f}ms")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 300.0)
