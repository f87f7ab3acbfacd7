"""Device plumbing: PyTorch-ROCm tensors as the device memory container.

PyTorch is used only for allocation, host<->device copies, streams and
``torch.distributed``; every computation runs in libslamhip's HIP kernels.
"""
import numpy as np


def torch():
    import torch as _t
    return _t


def require_gpu():
    t = torch()
    if not t.cuda.is_available():
        raise RuntimeError("slamhip: no ROCm GPU visible (torch.cuda.is_available() is False); "
                           "the HIP path has no CPU fallback")
    return t


def default_device():
    t = require_gpu()
    return t.device("cuda", t.cuda.current_device())


def to_dev(a, dtype, device=None):
    t = require_gpu()
    dev = device if device is not None else default_device()
    arr = np.ascontiguousarray(a, dtype=dtype)
    if not arr.flags.writeable:   # e.g. PoseGraph's cached edge arrays (torch wants writable memory)
        arr = arr.copy()
    return t.from_numpy(arr).to(dev, non_blocking=False)


def empty(shape, dtype, device=None):
    t = require_gpu()
    dev = device if device is not None else default_device()
    tdt = {np.float64: t.float64, np.int64: t.int64, np.int32: t.int32, np.int8: t.int8, np.uint8: t.uint8}[dtype]
    return t.empty(shape, dtype=tdt, device=dev)


def ptr(x):
    return None if x is None else x.data_ptr()


def stream_handle(stream=None):
    t = require_gpu()
    s = stream if stream is not None else t.cuda.current_stream()
    return s.cuda_stream
