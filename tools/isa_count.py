"""Static instruction mix of device kernels in a hipcc -S assembly file.

usage: python tools/isa_count.py file.s [substring-of-kernel-name ...]
Counts instructions per class (VALU f64, VALU int, VMEM, LDS, SALU, waitcnt, barrier) in each
matching kernel body.  Static counts only (loops are counted once) — a guide for where the
cycles of a fully unrolled kernel go.
"""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_") and "f64" in op:
        return "valu_f64"
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_load"
    if op.startswith(("global_store", "buffer_store", "flat_store")):
        return "vmem_store"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "lds_read"
    if op.startswith("ds_write") or op.startswith("ds_store"):
        return "lds_write"
    if op.startswith("ds_"):
        return "lds_other"
    if op == "s_waitcnt":
        return "waitcnt"
    if op == "s_barrier":
        return "barrier"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    cur, counts, ops = None, {}, {}
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            cur = m.group(1) if (not pats or any(p in m.group(1) for p in pats)) else None
            if cur:
                counts[cur] = Counter()
                ops[cur] = Counter()
            continue
        if cur is None:
            continue
        s = line.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        if op == "s_endpgm":
            cur = None
            continue
        counts[cur][classify(op)] += 1
        ops[cur][op] += 1
    for k, c in counts.items():
        print(k)
        print("  ", dict(sorted(c.items())), "total", sum(c.values()))
        print("   top:", ops[k].most_common(14))


if __name__ == "__main__":
    main()
