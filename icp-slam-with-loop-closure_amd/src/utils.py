"""Drop-in ``src/utils.py``: SE(2) conversions (reference ``src/utils.py:1-44``).

Host-side boundary helpers; the kernels inline the same formulas.
"""
import numpy as np

from slamhip.se2 import mat_to_pose, odom_change_to_mat, pose_to_mat  # noqa: F401


def invert_affine(mat):
    """``src/utils.py:21-26``, kept bug-for-bug: the translation is R^T t
    (the reference omits the minus sign).  Unused by the pipeline."""
    out = np.eye(mat.shape[0])
    rt = mat[:-1, :-1].T
    out[:-1, :-1] = rt
    out[:-1, -1] = rt @ mat[:-1, -1]
    return out


def homogenize(vecs):
    """Stub in the reference (``src/utils.py:38-40``): returns None."""
    return None


def unhomogenize(vecs):
    """Stub in the reference (``src/utils.py:42-44``): returns None."""
    return None
