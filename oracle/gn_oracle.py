"""CPU oracle for the pose-graph Gauss-Newton solve — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module.

The reference has NO Gauss-Newton: its optimiser is the
SGD relaxation.  The build's GN is defined as the standard SE(2) least-squares
problem over the graph exactly as the reference EXPORTS it to g2o
(``/root/reference/src/pose_graph.py:61-73``): every edge (a -> b, tf) is a
relative-pose measurement z = (tf[0,2], tf[1,2], atan2(tf[1,0], tf[0,0]))
with information 2 I when |b - a| == 1 and 5 I otherwise; node 0 is held
fixed (gauge).  Residual and Jacobians follow the usual g2o EDGE_SE2 form:

    e_t = Rz^T (Ri^T (tj - ti) - tz),   e_th = wrap(thj - thi - thz)
    A = de/dxi = [[-Rz^T Ri^T, Rz^T dRi^T/dthi (tj - ti)], [0, 0, -1]]
    B = de/dxj = [[ Rz^T Ri^T, 0], [0, 0, 1]]

One iteration solves (J^T W J) dx = -J^T W e with a sparse direct solver
(SciPy SuperLU) and applies x <- x + dx (headings wrapped to [-pi, pi)).
"Parity unpinned" against the reference (there is nothing to pin to); the
GPU path is checked against this float64 restatement.
"""
import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

ODOM_INFO = 2.0
LOOP_INFO = 5.0


def wrap(a):
    return a - 2 * np.pi * np.floor((a + np.pi) / (2 * np.pi))


def edge_measurements(tf):
    tf = np.asarray(tf, dtype=np.float64).reshape(-1, 3, 3)
    return np.stack([tf[:, 0, 2], tf[:, 1, 2], np.arctan2(tf[:, 1, 0], tf[:, 0, 0])], axis=1)


def information(ea, eb, odom=ODOM_INFO, loop=LOOP_INFO):
    return np.where(np.abs(np.asarray(eb) - np.asarray(ea)) == 1, odom, loop).astype(np.float64)


def linearize(poses, ea, eb, z, w):
    """Per-edge residuals e (E,3) and Jacobians A, B (E,3,3)."""
    xi, xj = poses[ea], poses[eb]
    ci, si = np.cos(xi[:, 2]), np.sin(xi[:, 2])
    cz, sz = np.cos(z[:, 2]), np.sin(z[:, 2])
    dx, dy = xj[:, 0] - xi[:, 0], xj[:, 1] - xi[:, 1]
    # Ri^T (tj - ti)
    ux, uy = ci * dx + si * dy, -si * dx + ci * dy
    vx, vy = ux - z[:, 0], uy - z[:, 1]
    e = np.stack([cz * vx + sz * vy, -sz * vx + cz * vy, wrap(xj[:, 2] - xi[:, 2] - z[:, 2])], axis=1)
    # M = Rz^T Ri^T
    m00, m01 = cz * ci - sz * si, cz * si + sz * ci
    m10, m11 = -sz * ci - cz * si, -sz * si + cz * ci
    # d(Ri^T)/dthi (tj - ti) = [-si dx + ci dy, -ci dx - si dy]
    gx, gy = -si * dx + ci * dy, -ci * dx - si * dy
    E = len(ea)
    A = np.zeros((E, 3, 3))
    B = np.zeros((E, 3, 3))
    A[:, 0, 0], A[:, 0, 1], A[:, 1, 0], A[:, 1, 1] = -m00, -m01, -m10, -m11
    A[:, 0, 2] = cz * gx + sz * gy
    A[:, 1, 2] = -sz * gx + cz * gy
    A[:, 2, 2] = -1.0
    B[:, 0, 0], B[:, 0, 1], B[:, 1, 0], B[:, 1, 1] = m00, m01, m10, m11
    B[:, 2, 2] = 1.0
    return e, A, B


def build_system(poses, ea, eb, z, w, fixed=0):
    """Sparse H (3(N-1) square) and b for the free nodes (node `fixed` removed)."""
    N = len(poses)
    e, A, B = linearize(poses, ea, eb, z, w)
    col = np.full(N, -1)
    free = [n for n in range(N) if n != fixed]
    col[free] = 3 * np.arange(len(free))
    rows, cols, vals = [], [], []
    b = np.zeros(3 * len(free))

    def put(ni, nj, blk):
        ci, cj = col[ni], col[nj]
        m = (ci >= 0) & (cj >= 0)
        for r in range(3):
            for c in range(3):
                rows.append(ci[m] + r)
                cols.append(cj[m] + c)
                vals.append(blk[m, r, c])

    At, Bt = np.transpose(A, (0, 2, 1)), np.transpose(B, (0, 2, 1))
    wv = w[:, None, None]
    put(ea, ea, wv * At @ A)
    put(ea, eb, wv * At @ B)
    put(eb, ea, wv * Bt @ A)
    put(eb, eb, wv * Bt @ B)
    gi = (w[:, None] * np.einsum("eij,ej->ei", At, e))
    gj = (w[:, None] * np.einsum("eij,ej->ei", Bt, e))
    for r in range(3):
        mi, mj = col[ea] >= 0, col[eb] >= 0
        np.add.at(b, col[ea][mi] + r, gi[mi, r])
        np.add.at(b, col[eb][mj] + r, gj[mj, r])
    n = 3 * len(free)
    H = sp.csc_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(n, n))
    chi2 = float(np.sum(w * np.sum(e * e, axis=1)))
    return H, b, col, chi2


def gn_iteration(poses, ea, eb, tf, w=None, fixed=0):
    """One Gauss-Newton step; returns (new poses, chi2 before the step, |dx|_inf)."""
    ea = np.asarray(ea, dtype=np.int64)
    eb = np.asarray(eb, dtype=np.int64)
    z = edge_measurements(tf)
    if w is None:
        w = information(ea, eb)
    H, b, col, chi2 = build_system(poses, ea, eb, z, w, fixed)
    dx = spla.spsolve(H, -b)
    out = poses.copy()
    m = col >= 0
    for r in range(3):
        out[m, r] += dx[col[m] + r]
    out[:, 2] = wrap(out[:, 2])
    return out, chi2, float(np.max(np.abs(dx))) if len(dx) else 0.0


def optimize(poses, ea, eb, tf, iterations=10, w=None, fixed=0):
    p = np.array(poses, dtype=np.float64)
    chis = []
    for _ in range(iterations):
        p, chi2, _ = gn_iteration(p, ea, eb, tf, w, fixed)
        chis.append(chi2)
    return p, chis
