"""Summarise a rocprofv3 SQLite output (kernels view) as per-kernel duration stats (CSV-like),
the same columns as rocprofv3 --stats kernel_stats.csv."""
import glob
import sqlite3
import statistics
import sys


def main(path):
    dbs = glob.glob(path + "/**/*.db", recursive=True) if not path.endswith(".db") else [path]
    rows = {}
    for db in dbs:
        c = sqlite3.connect(db)
        for name, start, end in c.execute("select name, start, end from kernels"):
            rows.setdefault(name, []).append(end - start)
    tot = sum(sum(v) for v in rows.values())
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"')
    for name, d in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        sd = statistics.pstdev(d) if len(d) > 1 else 0.0
        print(f'"{name}",{len(d)},{sum(d)},{sum(d)/len(d):.1f},{100*sum(d)/tot:.2f},{min(d)},{max(d)},{sd:.1f}')


if __name__ == "__main__":
    main(sys.argv[1])
