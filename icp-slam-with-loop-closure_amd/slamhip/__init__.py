"""slamhip — MI355X-native ICP scan matching and SE(2) pose-graph optimisation.

Hand-written HIP kernels for gfx950 (``csrc/``), reached through a thin ctypes
C-ABI (``include/slamhip.h``); PyTorch-ROCm provides device memory, streams and
``torch.distributed`` only.  The reference-compatible call surface lives in the
sibling ``src`` package (``src.icp``, ``src.pose_graph_optimization``, ...).
"""
from . import se2, synthetic  # noqa: F401  (pure NumPy, no GPU needed)

__all__ = ["se2", "synthetic", "icp", "pgo", "dist", "lib"]


def lib():
    """The loaded libslamhip.so (raises if it has not been built)."""
    from ._abi import lib as _lib
    return _lib()
