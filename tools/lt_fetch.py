"""HBM read bytes of the linear transforms' inner-product kernels in `bootstrapping_example prof`
(one warm bootstrap, then one lockstep group): the last 4 lt_bsgs_wide / lt_bsgs_tile dispatches (the single
bootstrap's 4 levels) against the last 4 lt_bsgs_group dispatches (the group's 4 levels), from a
rocprofv3 --pmc FETCH_SIZE pass (gfx950: bytes = 2 x FETCH_SIZE x 1024, MI355X_MICROARCH.md §HBM).

usage: python tools/lt_fetch.py <rocprofv3 output dir> [group]"""
import csv
import glob
import json
import os
import sys


def main(root, group=4):
    rows = []
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != "FETCH_SIZE":
                continue
            name = r["Kernel_Name"]
            kind = "single" if ("lt_bsgs_wide_kernel" in name or "lt_bsgs_tile_kernel" in name) else "group" if "lt_bsgs_group_kernel" in name else None
            if kind:
                rows.append((int(r["Dispatch_Id"]), kind, 2 * 1024 * float(r["Counter_Value"]),
                             int(r.get("Grid_Size", 0) or 0)))
    rows.sort()
    single = [r for r in rows if r[1] == "single"][-4:]
    grp = [r for r in rows if r[1] == "group"][-4:]
    levels = []
    for i, (s, g) in enumerate(zip(single, grp)):
        levels.append({"level": i, "single_read_bytes": s[2], "group_read_bytes": g[2],
                       "group_over_g_singles": round(g[2] / (group * s[2]), 4)})
    out = {"source": "rocprofv3 --pmc FETCH_SIZE over bootstrapping_example prof 16 %d" % group,
           "correction": "gfx950: read bytes = 2 x FETCH_SIZE x 1024", "group": group, "levels": levels,
           "sum_single_read_bytes": sum(r[2] for r in single), "sum_group_read_bytes": sum(r[2] for r in grp)}
    if single and grp:
        out["group_over_g_singles"] = round(out["sum_group_read_bytes"] / (group * out["sum_single_read_bytes"]), 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4)
