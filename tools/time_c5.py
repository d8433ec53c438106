"""C5 throughput of a library variant: bench.c5_leg (C5_TOTAL bootstraps, default 384, on C5_LANES lanes, default 3, 8 verified) on the
variant's ctypes binding.  usage: python tools/time_c5.py tools/variants/<name>/py"""
import os
import sys

sys.path.insert(0, sys.argv[1])
import phantom_amd as PA  # noqa: E402,F401  (the variant's binding, loaded first)
import torch  # noqa: E402

sys.path.insert(1, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

torch.cuda.set_device(0)
lanes = int(os.environ.get("C5_LANES", "3"))
group = int(os.environ["C5_GROUP"]) if os.environ.get("C5_GROUP") else None
r = bench.c5_leg(None, torch, 1, 0, 0, total=int(os.environ.get("C5_TOTAL", "384")), lanes=lanes, verify=8, group=group)
free, total = torch.cuda.mem_get_info()
print(os.path.basename(os.path.dirname(os.path.abspath(sys.argv[1]))), lanes, r["lockstep_group"], r["bootstraps_per_s"], r["min_avg_bits"],
      "used_GiB %.1f" % ((total - free) / 2**30), flush=True)
