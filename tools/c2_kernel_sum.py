"""Forward-NTT kernel averages from a rocprofv3 kernel_stats.csv of bench.py's C2 command ->
profiles/.../c2_fwd_kernels.json (bench.py KERNEL_SUM_SOURCE: fwd_ms minus this sum is the
column -> row launch gap).

  python tools/c2_kernel_sum.py <kernel_stats.csv> <out.json>
"""
import csv
import json
import re
import sys


def main():
    src, dst = sys.argv[1], sys.argv[2]
    got = {}
    for row in csv.DictReader(open(src)):
        name = row["Name"]
        # forward passes: ntt_col<S1, S2, FWD=true, BCV=false, ...> / ntt_row<S1, S2, FWD=true, EPI=false, ...>
        if re.search(r"ntt_col<\d+, \d+, true, false", name):
            got["ntt_col_fwd_us"] = float(row["AverageNs"]) / 1e3
            got["ntt_col_fwd_calls"] = int(row["Calls"])
        elif re.search(r"ntt_row<\d+, \d+, true, false", name):
            got["ntt_row_fwd_us"] = float(row["AverageNs"]) / 1e3
            got["ntt_row_fwd_calls"] = int(row["Calls"])
    if "ntt_col_fwd_us" not in got or "ntt_row_fwd_us" not in got:
        sys.exit("forward NTT kernels not found in " + src)
    got["sum_us"] = round(got["ntt_col_fwd_us"] + got["ntt_row_fwd_us"], 3)
    got["source"] = src
    json.dump(got, open(dst, "w"), indent=1)
    print(json.dumps(got))


if __name__ == "__main__":
    main()
