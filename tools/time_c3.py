"""C3 (multiply + relinearize + rescale) per-op times of a library variant: bench.c3_leg on the
variant's ctypes binding.  usage: python tools/time_c3.py tools/variants/<name>/py"""
import os
import sys

sys.path.insert(0, sys.argv[1])
import phantom_amd as PA  # noqa: E402  (the variant's binding, loaded first)
import torch  # noqa: E402

sys.path.insert(1, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

for _ in range(2):
    r = bench.c3_leg(PA, PA.load(), torch)
    print(os.path.basename(os.path.dirname(os.path.abspath(sys.argv[1]))), r["ms"], r["total_ms"], flush=True)
