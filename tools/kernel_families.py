"""Kernel time by family (template arguments and namespaces stripped) of a rocprofv3 stats CSV or a
tools/prof_windows.py window CSV.  usage: kernel_families.py <csv> [top]"""
import csv
import re
import sys


def family(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("phx::", "")
    n = re.sub(r"\(.*", "", n)
    return n.split("<")[0].strip()


def main(path, top=16):
    lines = [l for l in open(path).read().splitlines() if not l.startswith("#")]
    agg = {}
    for r in csv.DictReader(lines):
        k = family(r["Name"])
        a = agg.setdefault(k, [0, 0])
        a[0] += int(r["Calls"])
        a[1] += int(r["TotalDurationNs"])
    tot = sum(v[1] for v in agg.values())
    print(f"{'family':32s} {'calls':>6s} {'ms':>9s} {'%':>6s}")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{k:32s} {v[0]:6d} {v[1] / 1e6:9.3f} {100 * v[1] / tot:6.1f}")
    print(f"{'total':32s} {sum(v[0] for v in agg.values()):6d} {tot / 1e6:9.3f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 16)
