"""CPU oracle for the ICP hot path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product path (``slamhip`` / the drop-in ``src/icp.py``) never calls
into ``oracle/``.

It restates the reference's ICP (``/root/reference/src/icp.py``) in NumPy with
the reference's exact floating-point semantics, vectorised over queries:

* ``correspondences``  — ``get_closest_point`` + ``get_correspondences``
  (``src/icp.py:4-19``): squared distance summed over the 3 homogeneous
  columns in column order, first-minimum ``argmin``;
* ``kabsch``           — ``get_transform`` (``src/icp.py:22-46``): column
  means by ``np.sum(axis=0)/n``, ``S = X @ Y.T``, LAPACK SVD, reflection fix;
* ``sq_error``         — ``get_error`` (``src/icp.py:49-52``): a SUM (not a
  mean) over all n x 3 entries;
* ``icp_iteration``    — ``src/icp.py:55-69`` (incl. the in-place zeroing of
  the previous transform's translation when ``rotation_only``);
* ``icp``              — ``src/icp.py:72-97`` stopping rules: ``err < eps``,
  ``iteration > max_iters`` (so at most max_iters+2 iterations), and
  ``|last_err - err| < stopping_thresh`` from the second iteration on.

Pinning: ``tests/test_oracle_golden.py`` checks this module BIT FOR BIT
against ``tests/golden/icp_unit.npz`` and ``icp_cases.npz``, which
``tests/golden/gen_golden.py`` produced by running the reference itself.
"""
import numpy as np


def correspondences(pc1, pc2, block=256):
    """argmin_j sum_c (pc2[j,c] - pc1[i,c])**2 for every query row i."""
    pc1 = np.asarray(pc1, dtype=np.float64)
    pc2 = np.asarray(pc2, dtype=np.float64)
    out = np.empty(len(pc1), dtype=np.int64)
    for s in range(0, len(pc1), block):
        q = pc1[s:s + block]
        d = ((pc2[None, :, :] - q[:, None, :]) ** 2).sum(axis=2)
        out[s:s + block] = np.argmin(d, axis=1)
    return out


def correspondences_loop(pc1, pc2):
    """The reference's per-query Python loop shape (``src/icp.py:16-17``);
    used as the "ref_loop" CPU timing mode."""
    out = np.zeros(pc1.shape[0], dtype=int)
    for i in range(pc1.shape[0]):
        out[i] = np.argmin(np.sum((pc2 - pc1[i]) ** 2, axis=1))
    return out


def kabsch(a, b):
    """Rigid 2-D transform taking matched rows a -> b (3x3 homogeneous)."""
    n_a, n_b = a.shape[0], b.shape[0]
    mu_a = np.sum(a[:, 0:2], axis=0) / n_a
    mu_b = np.sum(b[:, 0:2], axis=0) / n_b
    xa = (a[:, 0:2] - mu_a).T
    yb = (b[:, 0:2] - mu_b).T
    cross = xa @ yb.T
    u, _, vt = np.linalg.svd(cross)
    v = vt.T
    fix = np.eye(2)
    fix[1, 1] = np.linalg.det(v @ u.T)
    rot = v @ fix @ u.T
    shift = mu_b.reshape((-1, 1)) - rot @ mu_a.reshape((-1, 1))
    out = np.eye(3)
    out[0:2, 0:2] = rot
    out[0, 2] = shift[0, 0]
    out[1, 2] = shift[1, 0]
    return out


def sq_error(a, b):
    return np.sum((a - b) ** 2)


def icp_iteration(pc1, pc2, prev, rotation_only=False, corr_fn=correspondences):
    if rotation_only:
        prev[:2, 2] = 0
    moved = np.dot(prev, pc1.T).T
    corr = corr_fn(moved, pc2)
    matched = pc2[corr]
    step = kabsch(moved, matched)
    if rotation_only:
        step[:2, 2] = 0
    return step @ prev, corr, sq_error(moved, matched)


def icp(pc1, pc2, init_transform=None, epsilon=0.01, max_iters=100, stopping_thresh=0.0001,
        rotation_only=False, corr_fn=correspondences):
    """Returns (list of 3x3 transforms starting with the caller's init, error)."""
    if init_transform is None:
        init_transform = np.eye(3)
    hist = [init_transform]
    k = 0
    prev_err = None
    while True:
        nxt, _, err = icp_iteration(pc1, pc2, hist[-1], rotation_only, corr_fn)
        hist.append(nxt)
        if err < epsilon or k > max_iters:
            return hist, err
        if prev_err is not None and np.abs(prev_err - err) < stopping_thresh:
            return hist, err
        prev_err = err
        k += 1


def icp_batch(pairs, **kw):
    """Serial loop over (pc1, pc2, init) triples; returns (final T (B,3,3),
    err (B,), iterations (B,))."""
    tf, err, its = [], [], []
    for pc1, pc2, init in pairs:
        h, e = icp(pc1, pc2, init_transform=np.array(init, dtype=np.float64), **kw)
        tf.append(h[-1])
        err.append(e)
        its.append(len(h) - 1)
    return np.stack(tf), np.array(err), np.array(its)
