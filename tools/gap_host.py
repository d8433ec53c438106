"""What the host did during the long idle gaps of one window of a kernel + HIP runtime trace
(rocprofv3 --kernel-trace --hip-runtime-trace, CSV): for every gap longer than `min_us` before
kernel K, the HIP API calls of K's launching thread between the previous kernel's end and K's
launch call, with their host durations, and the host time not spent in any HIP call.

usage: gap_host.py <trace dir> <window index> [min_us] [gap_ms]"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_windows import windows  # noqa: E402


def main():
    d = sys.argv[1]
    wi = int(sys.argv[2])
    min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 10.0
    gap_ms = float(sys.argv[4]) if len(sys.argv) > 4 else 20.0
    kt = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0])))
    api = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0])))
    by_corr = {a["Correlation_Id"]: a for a in api}
    api_by_thread = collections.defaultdict(list)
    for a in api:
        api_by_thread[a["Thread_Id"]].append((int(a["Start_Timestamp"]), int(a["End_Timestamp"]), a["Function"]))
    for v in api_by_thread.values():
        v.sort()
    ks = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Correlation_Id"]) for r in kt),
                key=lambda k: k[1])
    w = windows([k[:3] + (k[3],) for k in ks], gap_ms * 1e6)[wi]
    w.sort(key=lambda k: k[1])
    totals = collections.Counter()
    end = w[0][2]
    for i, k in enumerate(w[1:], 1):
        gap = (k[1] - end) / 1e3
        if gap > min_us and k[3] in by_corr:
            la = by_corr[k[3]]
            t1 = int(la["Start_Timestamp"])
            calls = [c for c in api_by_thread[la["Thread_Id"]] if end <= c[0] < t1]
            agg = collections.Counter()
            for s, e, f in calls:
                agg[f] += (e - s) / 1e3
            in_api = sum(agg.values())
            launch_lag = (k[1] - t1) / 1e3
            top = ", ".join(f"{f} {t:.0f}" for f, t in agg.most_common(4))
            print(f"gap {gap:7.1f} us before #{i} {k[0].split('(')[0][-45:]}: host {(t1 - end) / 1e3:7.1f} us "
                  f"({len(calls)} calls, {in_api:.0f} us in HIP: {top}), launch->start {launch_lag:.1f} us")
            for f, t in agg.items():
                totals[f] += t
        end = max(end, k[2])
    print("HIP time inside long gaps by function (us):", dict(totals.most_common(10)))


if __name__ == "__main__":
    main()
