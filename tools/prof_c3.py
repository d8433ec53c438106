"""Profiling driver: config C3 (multiply + relinearize + rescale, N=2^16, 45 limbs, P=15, dnum 3)
through the C-ABI, `ITERS` times; for rocprofv3 kernel traces / PMC passes."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "phantom-fhe-boot_amd", "py"))
import torch  # noqa: E402
import bench  # noqa: E402
import phantom_amd as PA  # noqa: E402

lib = PA.load()
print(bench.c3_leg(PA, lib, torch, steps=int(os.environ.get("ITERS", "20")), warmup=3))
