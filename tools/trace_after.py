"""Per-kernel totals from a rocprofv3 kernel_trace.csv restricted to dispatches after the last
dispatch of a marker kernel (e.g. the last key-generation kernel before timed bootstraps),
divided by a run count.  usage: trace_after.py trace.csv MARKER_SUBSTRING RUNS"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marker, runs = sys.argv[2], int(sys.argv[3])
last = max(i for i, r in enumerate(rows) if marker in r["Kernel_Name"])
tot, cnt = {}, {}
for r in rows[last + 1:]:
    name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("phx::(anonymous namespace)::", "").replace("void ", ""))
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot[name] = tot.get(name, 0) + d
    cnt[name] = cnt.get(name, 0) + 1
span = (int(rows[-1]["End_Timestamp"]) - int(rows[last + 1]["Start_Timestamp"])) / runs / 1e6
busy = sum(tot.values()) / runs / 1e6
print(f"per run: span {span:.2f} ms, kernel busy {busy:.2f} ms, {sum(cnt.values()) // runs} dispatches")
for k in sorted(tot, key=lambda k: -tot[k])[:25]:
    print(f"{k:50s} {cnt[k] // runs:6d}/run {tot[k] / runs / 1e6:8.3f} ms/run  avg {tot[k] / cnt[k] / 1e3:7.2f} us")
