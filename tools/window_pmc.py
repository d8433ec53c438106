"""PMC counters per kernel instantiation over the last window of a bootstrapping_example `prof` run
(the lockstep group): any number of rocprofv3 --kernel-trace --pmc passes over the same program,
joined by dispatch id.  FETCH_SIZE is reported as read bytes with the gfx950 correction
(2 x FETCH_SIZE KiB, MI355X_MICROARCH.md), WRITE_SIZE as write bytes (x KiB); other counters are
summed as they are (TCC_HIT_sum, TCC_MISS_sum -> hit rate).  Durations: the first pass's trace.

usage: python tools/window_pmc.py [--per K] <pass dir> [<pass dir> ...] > out.json
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = n.split("(")[0].replace("void ", "")
    return n.replace("phx::", "").replace("nttd::", "")


def last_window(d):
    trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    wins, cur = [], [rows[0]]
    for a, b in zip(rows, rows[1:]):
        if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) > 20e6:
            wins.append(cur)
            cur = []
        cur.append(b)
    wins.append(cur)
    return wins[-1]


def counters(d):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(cc)):
        vals[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return vals


def main():
    args = sys.argv[1:]
    per = 8
    if args[0] == "--per":
        per, args = int(args[1]), args[2:]
    wins = [last_window(d) for d in args]
    # the same program in every pass: the k-th dispatch of the window is the same kernel
    names = [r["Kernel_Name"] for r in wins[0]]
    for w in wins[1:]:
        if [r["Kernel_Name"] for r in w] != names:
            raise SystemExit("passes differ in their last window's dispatch sequence")
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for d, w in zip(args, wins):
        vals = counters(d)
        for i, r in enumerate(w):
            a = agg[short(r["Kernel_Name"])]
            if d == args[0]:
                a["calls"] += 1
                a["ms"] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            for c, v in vals.items():
                x = v.get(r["Dispatch_Id"], 0.0)
                if c == "FETCH_SIZE":
                    a["read_GB"] += 2048.0 * x / 1e9
                elif c == "WRITE_SIZE":
                    a["write_GB"] += 1024.0 * x / 1e9
                else:
                    a[c] += x
    out = {"source": "rocprofv3 --kernel-trace --pmc, one pass per counter set, last window (%d bootstraps)" % per,
           "correction": "gfx950: read = 2 x FETCH_SIZE KiB, write = WRITE_SIZE KiB", "kernels": {}}
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["ms"]):
        e = {kk: (round(v, 3) if isinstance(v, float) else v) for kk, v in a.items()}
        e["calls"] = int(a["calls"])
        e["ms_per_bootstrap"] = round(a["ms"] / per, 3)
        if "read_GB" in a and "write_GB" in a and a["write_GB"]:
            e["read_over_write"] = round(a["read_GB"] / a["write_GB"], 3)
        h, m = a.get("TCC_HIT_sum"), a.get("TCC_MISS_sum")
        if h is not None and m is not None and h + m:
            e["tcc_hit_rate"] = round(h / (h + m), 4)
        out["kernels"][k] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
