"""EvalMod's kernels in a rocprofv3 kernel trace of the bootstrap example: the window from the first
to the last tensor_lin / leaf_combine dispatch (only MulAddRescale and the Chebyshev leaves launch
those) of the last bootstrap; prints span, kernel-busy time, per-kernel totals and optionally the
timeline.

  python tools/evalmod_window.py run_kernel_trace.csv [--timeline]
"""
import csv
import re
import sys


def name(r):
    return re.sub(r"\(.*", "", r["Kernel_Name"].replace("phx::(anonymous namespace)::", "").replace("void ", ""))


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "tensor_lin" in name(r) or "leaf_combine" in name(r)]
    last = marks[-1]
    t_last = int(rows[last]["Start_Timestamp"])
    first = [i for i in marks if int(rows[i]["Start_Timestamp"]) > t_last - 15_000_000][0]
    seg = rows[first:last + 1]
    t0 = int(seg[0]["Start_Timestamp"])
    end = max(int(r["End_Timestamp"]) for r in seg)
    tot, cnt = {}, {}
    for r in seg:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        tot[name(r)] = tot.get(name(r), 0) + d
        cnt[name(r)] = cnt.get(name(r), 0) + 1
    print(f"span {(end - t0) / 1e6:.3f} ms, kernel busy {sum(tot.values()) / 1e6:.3f} ms, {len(seg)} dispatches")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{k:60s} {cnt[k]:5d} {v / 1e3:9.1f} us  avg {v / cnt[k] / 1e3:7.1f}")
    if "--timeline" in sys.argv:
        prev = t0
        for r in seg:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} gap {(s - prev) / 1e3:6.1f}  {name(r)[:70]}")
            prev = max(prev, e)


if __name__ == "__main__":
    main()
