"""Drop-in ``src/icp.py``: the reference's ICP call surface on MI355X.

Every function keeps the reference signature, return types and side effects
(``/root/reference/src/icp.py``); the arithmetic runs in libslamhip's HIP
kernels (``slam_icp_batch_f64``, ``slam_icp_step_f64``,
``slam_kabsch2d_f64``).  Inputs are the reference's homogeneous (n, 3) float64
clouds (``np.c_[points, ones]``) and SE(2) matrices; a homogeneous coordinate
other than 1 raises ``ValueError`` (the kernels keep it implicit).

Differences from the reference, all within the parity tolerance (1e-9 on
transforms in tests/test_icp_gpu.py): the 2x2 rotation is the closed form of
the SVD route and the reductions use a fixed tree order instead of NumPy's.
Correspondences are bit-identical whenever the transformed query coordinates
are (the transform step reproduces OpenBLAS's FMA order).

New: ``icp_batch`` — B pairs in one launch, the GPU replacement for the
joblib fan-out in ``scripts/main.py:240-247``.
"""
import numpy as np

from slamhip import icp as _k

_DEFAULT_INIT = np.eye(3)   # shared mutable default, as in the reference


def get_closest_point(point, pc):
    """src/icp.py:4-7 — index of pc's row nearest to ``point``."""
    corr = get_correspondences(np.asarray(point, dtype=np.float64).reshape(1, -1), pc)
    return corr[0]


def get_correspondences(pc1, pc2):
    """src/icp.py:10-19 — nearest pc2 row for every pc1 row (int array)."""
    _, corr, _ = _k.icp_step([pc1, pc2], [0], [1], np.eye(3)[None])
    return corr[0].astype(int)


def get_transform(pc1, pc2):
    """src/icp.py:22-46 — SE(2) matrix taking matched rows pc1[i] to pc2[i]."""
    T, _ = _k.kabsch(pc1, pc2)
    return T


def get_error(pc1, pc2):
    """src/icp.py:49-52 — sum of squared differences of matched rows."""
    _, e = _k.kabsch(pc1, pc2)
    return e


def icp_iteration(pc1, pc2, previous_transform, rotation_only=False):
    """src/icp.py:55-69 — returns (transform, correspondences, error)."""
    if rotation_only:
        previous_transform[:2, 2] = 0   # the reference mutates its argument
    T, corr, err = _k.icp_step([pc1, pc2], [0], [1], np.asarray(previous_transform)[None],
                               rotation_only=rotation_only)
    return T[0], corr[0].astype(int), np.float64(err[0])


def icp(pc1, pc2, init_transform=_DEFAULT_INIT, epsilon=0.01, max_iters=100, stopping_thresh=0.0001,
        rotation_only=False):
    """src/icp.py:72-97 — returns (list of 3x3 transforms, error).

    ``transforms[0]`` is the caller's ``init_transform`` object (its
    translation zeroed in place when ``rotation_only``, as the reference does).
    """
    init = np.asarray(init_transform, dtype=np.float64)
    hist, err, _ = _k.icp_pair(pc1, pc2, init, epsilon=epsilon, max_iters=max_iters,
                               stopping_thresh=stopping_thresh, rotation_only=rotation_only)
    if rotation_only:
        init_transform[:2, 2] = 0
    transforms = [init_transform] + [h.copy() for h in hist[1:]]
    return transforms, np.float64(err)


def icp_batch(pc1_list, pc2_list, init_transforms, epsilon=0.01, max_iters=100, stopping_thresh=0.0001,
              rotation_only=False, history=False):
    """B independent ``icp()`` calls in one launch.

    Returns (final transforms (B,3,3), errors (B,), iterations (B,)) and, with
    ``history=True``, a fourth item: the per-pair transform lists.
    """
    res = _k.icp_pairs(list(pc1_list), list(pc2_list), np.asarray(init_transforms, dtype=np.float64),
                       epsilon=epsilon, max_iters=max_iters, stopping_thresh=stopping_thresh,
                       rotation_only=rotation_only, history=history)
    if history:
        return res.tf, res.err, res.iters, [list(h) for h in res.hist]
    return res.tf, res.err, res.iters
