"""Summarise rocprofv3 --pmc csv passes (tools/gpu_probe.sh) per kernel: mean counter value per
dispatch.  FETCH_SIZE/WRITE_SIZE are in KiB as rocprofv3 reports them (see MI355X_MICROARCH.md
§HBM for the gfx950 FETCH_SIZE correction).

usage: python tools/pmc_summary.py gpurun_out/pmc_r01 > profiles/r01/ntt_pmc_summary.txt
"""
import collections
import csv
import glob
import os
import re
import sys


def main():
    root = sys.argv[1]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(\w+<[^>]*>)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"][:40]
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        print(k)
        for c, v in sorted(d.items()):
            print(f"   {c:24s} {sum(v) / len(v):14.1f}  (dispatches={len(v)})")


if __name__ == "__main__":
    main()
