"""Per-dispatch HBM bytes of the NTT passes from rocprofv3 FETCH_SIZE / WRITE_SIZE passes
(tools/gpu_pmc_traffic.sh), corrected as MI355X_MICROARCH.md §HBM prescribes for gfx950:
FETCH_SIZE (KiB) counts half the bytes of 16-B-per-lane streaming reads, so it is doubled;
WRITE_SIZE (KiB) is taken as is.  Prints JSON: per kernel mean read / write bytes per dispatch,
and the forward-NTT total (column + row pass) that bench.py reports as roofline.traffic.

usage: python tools/pmc_traffic.py gpurun_out/pmc_traffic > profiles/rNN/ntt_pmc_traffic.json
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def main():
    root = sys.argv[1]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(ntt_\w+<[^>]*>)", r["Kernel_Name"])
            if not m:
                continue
            vals[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, tools/prof_ntt.py",
           "correction": "gfx950: read bytes = 2 x FETCH_SIZE x 1024; write bytes = WRITE_SIZE x 1024",
           "kernels": {}}
    for k, d in vals.items():
        rd = 2 * 1024 * sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"]) if d.get("FETCH_SIZE") else None
        wr = 1024 * sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"]) if d.get("WRITE_SIZE") else None
        out["kernels"][k] = {"read_bytes": rd, "write_bytes": wr, "dispatches": len(d.get("FETCH_SIZE", []))}
    def is_fwd(k):  # ntt_col<S1, S2, FWD> / ntt_row<S1, S2, FWD, EPI>
        return k.split("<")[1].rstrip(">").split(",")[2].strip() == "true"
    fwd = [v for k, v in out["kernels"].items() if is_fwd(k)]
    if fwd and all(v["read_bytes"] is not None and v["write_bytes"] is not None for v in fwd):
        out["forward_ntt_bytes_per_launch"] = sum(v["read_bytes"] + v["write_bytes"] for v in fwd)
    inv = [v for k, v in out["kernels"].items() if not is_fwd(k)]
    if inv and all(v["read_bytes"] is not None and v["write_bytes"] is not None for v in inv):
        out["inverse_ntt_bytes_per_launch"] = sum(v["read_bytes"] + v["write_bytes"] for v in inv)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
