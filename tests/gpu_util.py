"""Device-buffer helpers for GPU parity tests (torch is used only for HIP memory/streams)."""
import numpy as np


def torch():
    import torch as _t
    assert _t.cuda.is_available(), "GPU tests need a HIP device"
    return _t


def to_dev(a):
    t = torch()
    return t.from_numpy(np.ascontiguousarray(a).view(np.int64).copy()).cuda()


def to_host(t):
    torch().cuda.synchronize()
    return t.cpu().numpy().view(np.uint64).copy()


def stream():
    return torch().cuda.current_stream().cuda_stream


def ptr(t):
    return t.data_ptr()
