"""Per-kernel stats of the LAST warm run in a rocprofv3 kernel-trace database (or csv trace): the trace is cut at
the last idle gap longer than `gap_us` (the host synchronises between runs), so setup, key
generation and earlier runs are excluded.  Prints kernel stats CSV for that window plus the
window's wall span and the union of kernel intervals (GPU busy time)."""
import glob
import sqlite3
import statistics
import sys


def main(path, gap_us=300.0):
    ks = []
    if path.endswith(".csv"):  # --output-format csv: run_kernel_trace.csv
        import csv
        for r in csv.DictReader(open(path)):
            ks.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    else:
        dbs = glob.glob(path + "/**/*.db", recursive=True) if not path.endswith(".db") else [path]
        for db in dbs:
            c = sqlite3.connect(db)
            ks += list(c.execute("select name, start, end from kernels"))
    ks.sort(key=lambda r: r[1])
    # walk back from the end to the last gap > gap_us between the running max end and the next start
    cut = 0
    run_end = ks[0][2]
    for i in range(1, len(ks)):
        if ks[i][1] - run_end > gap_us * 1e3:
            cut = i
        run_end = max(run_end, ks[i][2])
    win = ks[cut:]
    t0, t1 = win[0][1], max(e for _, _, e in win)
    busy, cur_s, cur_e = 0, None, None
    for _, s, e in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    rows = {}
    for name, s, e in win:
        rows.setdefault(name, []).append(e - s)
    tot = sum(sum(v) for v in rows.values())
    print(f"# window: {len(win)} kernels, wall span {(t1 - t0) / 1e6:.3f} ms, GPU busy (union) {busy / 1e6:.3f} ms, "
          f"sum of kernel durations {tot / 1e6:.3f} ms")
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"')
    for name, d in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        sd = statistics.pstdev(d) if len(d) > 1 else 0.0
        print(f'"{name}",{len(d)},{sum(d)},{sum(d)/len(d):.1f},{100*sum(d)/tot:.2f},{min(d)},{max(d)},{sd:.1f}')


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 300.0)
