"""Per-kernel stats of every run in a rocprofv3 kernel trace, the runs separated by idle gaps longer
than `gap_ms` (bootstrapping_example prof sleeps 100 ms between its runs).  Writes one CSV per
window (prefix_w<i>.csv, the format of rocprofv3 --stats) and prints a summary line per window.

usage: prof_windows.py <trace dir | .db | kernel_trace.csv> <out prefix> [gap_ms]"""
import csv
import glob
import sqlite3
import statistics
import sys


def load(path):
    ks = []
    if path.endswith(".csv"):
        for r in csv.DictReader(open(path)):
            ks.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    else:
        dbs = glob.glob(path + "/**/*.db", recursive=True) if not path.endswith(".db") else [path]
        for db in dbs:
            ks += list(sqlite3.connect(db).execute("select name, start, end from kernels"))
        if not dbs:
            for f in glob.glob(path + "/**/*kernel_trace.csv", recursive=True):
                ks += load(f)
    ks.sort(key=lambda r: r[1])
    return ks


def windows(ks, gap_ns):
    out, cur, run_end = [], [ks[0]], ks[0][2]
    for k in ks[1:]:
        if k[1] - run_end > gap_ns:
            out.append(cur)
            cur = []
        cur.append(k)
        run_end = max(run_end, k[2])
    out.append(cur)
    return out


def stats(win):
    t0, t1 = win[0][1], max(e for _, _, e in win)
    busy, cs, ce = 0, None, None
    for _, s, e in win:
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    rows = {}
    for name, s, e in win:
        rows.setdefault(name, []).append(e - s)
    return t1 - t0, busy, rows


def main(path, prefix, gap_ms=20.0):
    ks = load(path)
    for i, w in enumerate(windows(ks, gap_ms * 1e6)):
        span, busy, rows = stats(w)
        tot = sum(sum(v) for v in rows.values())
        with open(f"{prefix}_w{i}.csv", "w") as f:
            f.write(f"# window {i}: {len(w)} kernels, wall span {span / 1e6:.3f} ms, GPU busy (union) {busy / 1e6:.3f} ms, "
                    f"sum of kernel durations {tot / 1e6:.3f} ms\n")
            f.write('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n')
            for name, d in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
                sd = statistics.pstdev(d) if len(d) > 1 else 0.0
                f.write(f'"{name}",{len(d)},{sum(d)},{sum(d)/len(d):.1f},{100*sum(d)/tot:.2f},{min(d)},{max(d)},{sd:.1f}\n')
        print(f"window {i}: {len(w)} kernels, span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, "
              f"kernel sum {tot / 1e6:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], float(sys.argv[3]) if len(sys.argv) > 3 else 20.0)
