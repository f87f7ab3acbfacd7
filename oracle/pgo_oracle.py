"""CPU oracle for the pose-graph hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module; the product (``slamhip`` and the drop-in ``src``
package) never does.

Restates, in NumPy with the reference's rounding:

* ``sgd_step``  — ``pose_graph_optimization_step_sgd``
  (``/root/reference/src/pose_graph_optimization.py:7-49``): pass 1 builds
  M[i] = sum of diag(inv(R sigma R^T)) over loop edges covering i (edge order)
  and gamma = the first minimum-norm diag; pass 2 walks loop edges in
  networkx order, r = mat_to_pose(pose_to_mat(P_a) @ tf) - P_b with
  r[2] %= 2 pi, d = 2 inv(R^T sigma R) r, beta = clamp((b - a) d_j lr /
  gamma_j, |r_j|), and spreads beta over (a, b] in proportion to 1/M (the
  reference's left-to-right running sum == ``np.cumsum``), tail i > b by the
  full sum.  Bit-identical to the reference on the generating host
  (tests/test_oracle_golden.py::test_sgd_restatement).
* ``orient_from_positions`` / ``recompute_orientation`` —
  ``recompute_pose_graph_orientation`` (``:51-74``).
* ``FlatGraph`` — the networkx DiGraph semantics ``src/pose_graph.py:21-51``
  relies on (edge iteration order, overwrite-in-place, ``flip``), without
  networkx.
"""
import numpy as np

TWO_PI = 2 * np.pi


def wrap(a):
    return (np.asarray(a) + np.pi) % TWO_PI - np.pi


def _rot(theta):
    c, s = np.cos(theta), np.sin(theta)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def _pose_mat(p):
    return np.array([[np.cos(p[2]), -np.sin(p[2]), p[0]], [np.sin(p[2]), np.cos(p[2]), p[1]], [0, 0, 1]])


def _mat_pose(m):
    return np.array([m[0, 2], m[1, 2], np.arctan2(m[1, 0], m[0, 0])])


def sgd_step(poses, ea, eb, tf, learning_rate=1, loop_closure_uncertainty=0.1):
    """In place on ``poses`` (N, 3); edges in networkx iteration order."""
    N = len(poses)
    sigma = np.eye(3) * loop_closure_uncertainty
    loops = [e for e in range(len(ea)) if abs(int(ea[e]) - int(eb[e])) != 1]
    M = np.zeros((N, 3))
    gamma = np.full(3, np.inf)
    for e in loops:
        a, b = int(ea[e]), int(eb[e])
        R = _rot(poses[a][2])
        dW = np.diag(np.linalg.inv(R @ sigma @ R.T))
        if b >= a + 1:
            M[a + 1:b + 1] = M[a + 1:b + 1] + dW
            if np.dot(gamma, gamma) > np.dot(dW, dW):
                gamma = dW
    for e in loops:
        a, b = int(ea[e]), int(eb[e])
        R = _rot(poses[a][2])
        r = _mat_pose(_pose_mat(poses[a]) @ tf[e]) - poses[b]
        r[2] = r[2] % TWO_PI
        d = 2 * np.linalg.inv(R.T @ sigma @ R) @ r.reshape(-1, 1)
        if b < a + 1:
            continue   # empty (a, b]: the reference adds zeros
        for j in range(3):
            alpha = 1 / gamma[j]
            alpha *= learning_rate
            tw = np.sum(1 / M[a + 1:b + 1, j])
            beta = (b - a) * d[j, 0] * alpha
            if np.abs(beta) > np.abs(r[j]):
                beta = r[j]
            ramp = np.cumsum(beta / M[a + 1:b + 1, j] / tw)
            poses[a + 1:b + 1, j] = poses[a + 1:b + 1, j] + ramp
            poses[b + 1:, j] = poses[b + 1:, j] + ramp[-1]
    return poses


def orient_from_positions(poses):
    for i in range(1, len(poses) - 1):
        v = poses[i + 1][0:2] - poses[i][0:2]
        n = np.linalg.norm(v)
        if n > 0:
            v = v / n
            poses[i][2] = np.arctan2(v[1], v[0])
    return poses


def recompute_orientation(poses, scans, icp_max_iters, icp_epsilon, icp_recompute=False, icp_fn=None):
    orient_from_positions(poses)
    if icp_recompute:
        tfs = []
        for i in range(1, len(poses)):
            pc1 = np.c_[scans[i], np.ones(len(scans[i]))]
            pc2 = np.c_[scans[i - 1], np.ones(len(scans[i - 1]))]
            h, _ = icp_fn(pc1, pc2, _pose_mat(poses[i] - poses[i - 1]), icp_epsilon, icp_max_iters, 0.0001, True)
            tfs.append(h[-1])
        for i in range(len(poses) - 1, 0, -1):
            t = tfs[i - 1]
            poses[i][2] = poses[i - 1][2] + np.arctan2(t[1][0], t[0][0])
    return poses


class FlatGraph:
    """Edge list with networkx DiGraph ordering semantics.

    ``edges()`` of a DiGraph iterates nodes in first-insertion order and each
    node's successors in insertion order; re-adding an existing edge keeps its
    position and replaces its data.
    """

    def __init__(self, poses, ea=None, eb=None, tf=None, nodes=None):
        # PoseGraph.__init__ inserts nodes 0..N-1 through its successive edges
        self.poses = poses
        self.adj = {int(i): {} for i in (range(len(poses)) if nodes is None else nodes)}
        if ea is not None:
            for a, b, t in zip(ea, eb, tf):
                self.add(int(a), int(b), t)

    def add(self, a, b, t):
        self.adj.setdefault(a, {})
        self.adj.setdefault(b, {})
        self.adj[a][b] = np.asarray(t, dtype=np.float64)

    def edges(self):
        for a, succ in self.adj.items():
            for b, t in succ.items():
                yield a, b, t

    @property
    def ea(self):
        return np.array([a for a, _, _ in self.edges()], dtype=np.int64)

    @property
    def eb(self):
        return np.array([b for _, b, _ in self.edges()], dtype=np.int64)

    @property
    def tf(self):
        return np.stack([t for _, _, t in self.edges()])

    def flip(self):
        self.poses = self.poses[::-1]
        self.poses[:, 2] = (self.poses[:, 2] + np.pi) % TWO_PI
        n = len(self.poses) - 1
        old = list(self.edges())
        self.adj = {}
        for a, b, t in old:
            self.add(n - b, n - a, t)
