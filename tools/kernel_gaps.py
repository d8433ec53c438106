"""Idle gaps between consecutive kernels of one window of a rocprofv3 kernel trace (the windows as
tools/prof_windows.py cuts them: runs separated by > gap_ms of idle).  For a single-stream window
(one bootstrap) every gap is the device-side hand-off between dependent kernels plus any host
stall; the distribution tells which of the two the idle time is.

usage: kernel_gaps.py <trace dir | kernel_trace.csv> <window index (negative: from the end)> [gap_ms]"""
import statistics
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_windows import load, windows  # noqa: E402


def main():
    ks = load(sys.argv[1])
    gap_ms = float(sys.argv[3]) if len(sys.argv) > 3 else 20.0
    w = windows(ks, gap_ms * 1e6)[int(sys.argv[2])]
    w.sort(key=lambda k: k[1])
    gaps, busy_end = [], w[0][2]
    for k in w[1:]:
        gaps.append(max(0, k[1] - busy_end) / 1e3)  # us; overlap (several streams) counts as 0
        busy_end = max(busy_end, k[2])
    span = (max(k[2] for k in w) - w[0][1]) / 1e6
    gs = sorted(gaps)
    q = lambda p: gs[min(len(gs) - 1, int(p * len(gs)))]
    print({"kernels": len(w), "span_ms": round(span, 3), "idle_ms": round(sum(gaps) / 1e3, 3),
           "gap_us_median": round(statistics.median(gs), 2), "p10": round(q(0.1), 2), "p90": round(q(0.9), 2),
           "p99": round(q(0.99), 2), "max": round(gs[-1], 1), "gaps_over_10us": sum(g > 10 for g in gs),
           "idle_in_gaps_over_10us_ms": round(sum(g for g in gs if g > 10) / 1e3, 3)})


if __name__ == "__main__":
    main()
