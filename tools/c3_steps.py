"""Per-launch breakdown of the last C3 step (multiply, relinearize, rescale) in a rocprofv3 kernel
trace of tools/prof_c3.py: kernel, duration and the idle gap before it.
usage: python tools/c3_steps.py <run_kernel_trace.csv>"""
import csv
import re
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").replace("phx::", "").replace("nttd::", "")
    return re.sub(r"\(.*", "", n)


def main(path):
    ks = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(path))
                 if "copyBuffer" not in r["Kernel_Name"]), key=lambda k: k[1])
    idx = [i for i, k in enumerate(ks) if "tensor_kernel" in k[0]]
    i0, i1 = idx[-2], idx[-1]
    prev = None
    for k in ks[i0:i1]:
        gap = (k[1] - prev) / 1e3 if prev else 0.0
        print(f"{short(k[0]):56s} {(k[2] - k[1]) / 1e3:8.2f} us  gap {gap:6.2f}")
        prev = k[2]
    print(f"step span {(ks[i1][1] - ks[i0][1]) / 1e3:.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])
