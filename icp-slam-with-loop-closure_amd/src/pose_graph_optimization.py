"""Drop-in ``src/pose_graph_optimization.py`` on MI355X.

Keeps the reference's functions (``/root/reference/src/pose_graph_optimization.py``)
with their signatures and in-place semantics:

* ``pose_graph_optimization_step_sgd(pose_graph, learning_rate=1,
  loop_closure_uncertainty=0.1)`` — runs in ``slam_pgo_sgd_step_f64``; the
  updated poses are written back INTO ``pose_graph.poses`` (same array object,
  so views such as the one ``PoseGraph.flip`` leaves behave as before);
* ``recompute_pose_graph_orientation(...)`` — ``slam_pgo_orient_f64``, and
  with ``icp_recompute`` one batched rotation-only ICP launch over all
  consecutive pairs (instead of the joblib fan-out at :59-68) followed by
  ``slam_pgo_orient_from_tf_f64``; ``n_jobs`` is accepted and ignored;
* ``construct_R(pose_graph, idx)`` — host helper, unchanged.

New: ``optimize_pose_graph`` — the Gauss-Newton solve (J^T J assembly +
Cholesky on the GPU) named by this build's north star; see slamhip.gn.
"""
import warnings

import numpy as np

from slamhip import icp as _icp
from slamhip import pgo as _pgo
from slamhip.se2 import pose_to_mat


def pose_graph_optimization_step_sgd(pose_graph, learning_rate=1, loop_closure_uncertainty=0.1):
    """Reference :7-49.  The flattened edges (``PoseGraph.edge_arrays``, cached
    until the graph changes) and their device copy plus the step's scratch are
    kept on the graph object between calls (scripts/main.py:325-326 runs 50
    steps on one graph): a call uploads the poses, runs the step and writes
    them back in place."""
    flat = pose_graph.edge_arrays() if hasattr(pose_graph, "edge_arrays") else _edges(pose_graph)
    cache = getattr(pose_graph, "_sgd_solver", None)
    N = len(pose_graph.poses)
    if cache is None or cache[0] is not flat or cache[1].N != N:
        cache = (flat, _pgo.SgdSolver(pose_graph.poses, *flat))
        try:
            pose_graph._sgd_solver = cache
        except AttributeError:   # a graph type without attribute storage: no cache
            pass
    else:
        cache[1].set_poses(pose_graph.poses)
    s = cache[1]
    s.step(learning_rate, loop_closure_uncertainty)
    pose_graph.poses[...] = s.host_poses()


def recompute_pose_graph_orientation(pose_graph, lidar_points, icp_max_iters, icp_epsilon, n_jobs,
                                     icp_recompute=False):
    pose_graph.poses[...] = _pgo.orient(pose_graph.poses)
    if icp_recompute:
        poses = pose_graph.poses
        N = len(poses)
        inits = np.stack([pose_to_mat(poses[i] - poses[i - 1]) for i in range(1, N)])
        res = _icp.icp_batch(list(lidar_points), np.arange(1, N), np.arange(0, N - 1), inits,
                             epsilon=icp_epsilon, max_iters=icp_max_iters, rotation_only=True)
        pose_graph.poses[...] = _pgo.orient_from_tf(poses, res.tf)


def construct_R(pose_graph, idx):
    theta = pose_graph.poses[idx][2]
    c, s = np.cos(theta), np.sin(theta)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def optimize_pose_graph(pose_graph, iterations=10, odom_information=2.0, loop_information=5.0,
                        tol=None, return_history=False, odometry_edges="global_delta", loop_edges="icp"):
    """Gauss-Newton on the SE(2) graph (relative-pose residuals, information
    2 I for odometry edges and 5 I for loop edges as ``PoseGraph.export_g2o``
    writes them); node 0 is held fixed.  Updates ``pose_graph.poses`` in place.

    GN measures every edge a -> b as z with X_b = X_a z.  The graph as
    scripts/main.py builds it holds two other conventions, converted here
    (``gn_measurements``): the constructor's odometry edges (b = a + 1) are
    GLOBAL-frame deltas P[a+1] - P[a] (reference src/pose_graph.py:32-36) and
    are re-expressed in node a's frame (``odometry_edges="global_delta"``;
    ``"relative"`` keeps them); loop edges are ICP results T of
    icp(pc_a, pc_b), i.e. X_a = X_b T (scripts/main.py:305), so z = T^-1
    (``loop_edges="icp"``; ``"relative"`` keeps them).  ``tol`` stops early
    once chi2 changes by less than tol (relative) between iterations."""
    from slamhip import gn as _gn
    ea, eb, tf = gn_measurements(pose_graph, odometry_edges, loop_edges)
    solver = _gn.GaussNewton(pose_graph.poses, ea, eb, tf, odom_information, loop_information)
    hist = solver.run(iterations, tol=tol)
    pose_graph.poses[...] = solver.host_poses()
    return hist if return_history else None


def gn_measurements(pose_graph, odometry_edges="global_delta", loop_edges="icp"):
    """(ea, eb, z (E, 3, 3)) in networkx edge order with X_b = X_a z for every edge.

    Each edge is classified by what ``PoseGraph`` recorded when it was added
    (``PoseGraph.edge_kinds``):

    * a constructor edge (a, a+1) holds odom_change_to_mat(P[a+1] - P[a]):
      rotation by the heading change and the GLOBAL translation delta; its
      relative measurement is R(theta_a)^T delta with theta_a the heading the
      delta was taken at (the edge's ``heading``) — ``odometry_edges=
      "relative"`` keeps such edges as they are;
    * a constraint added with ``convention="icp"`` (X_a = X_b T: icp(pc_a,
      pc_b), the manual / image loop closures) is inverted; one added with
      ``convention="relative"`` (icp(pc_b, pc_a), ``detect_proximity``) is kept;
    * a constraint without a recorded convention follows ``loop_edges``.

    An edge with no annotation at all (built by the reference's own
    PoseGraph, loaded from a reference pickle, or flipped) is classified by
    its shape, PER EDGE: (a, a+1) is a constructor delta at the current pose's
    heading, any other edge follows ``loop_edges``.  So an unannotated pickle
    that later gets closures added with a convention keeps its odometry
    edges as deltas.  The shape rule applies only while NO edge carries a
    heading: in a graph whose constructor edges are annotated, a bare
    (a, a+1) edge is a constraint saved without its convention (an older
    pickle of this build) and follows ``loop_edges``, with a warning."""
    if odometry_edges not in ("global_delta", "relative") or loop_edges not in ("icp", "relative"):
        raise ValueError("odometry_edges in {global_delta, relative}, loop_edges in {icp, relative}")
    ea, eb, tf = pose_graph.edge_arrays() if hasattr(pose_graph, "edge_arrays") else _edges(pose_graph)
    z = np.array(tf, dtype=np.float64).reshape(-1, 3, 3)
    if hasattr(pose_graph, "edge_kinds"):
        head, conv, added = pose_graph.edge_kinds()
    else:
        head, conv, added = np.full(len(ea), np.nan), np.zeros(len(ea), np.int8), np.zeros(len(ea), bool)
    delta = ~np.isnan(head)
    bare = ~delta & ~added & (conv == 0) & (eb.astype(np.int64) == ea.astype(np.int64) + 1)
    if bare.any() and not delta.any():
        # a graph with no heading annotation anywhere (the reference's own
        # PoseGraph or pickle): unannotated (a, a+1) edges are constructor
        # deltas, at the current heading (the shape rule)
        head = np.where(bare, np.asarray(pose_graph.poses, dtype=np.float64)[ea, 2], head)
        delta = delta | bare
    elif bare.any():
        # a mixed graph: its constructor edges carry headings, so a bare
        # (a, a+1) edge is a constraint whose convention was not recorded (an
        # older pickle of this build); it follows loop_edges, as it did there
        warnings.warn(f"{int(bare.sum())} unannotated (a, a+1) edge(s) in a graph whose odometry edges carry "
                      f"headings: treated as loop constraints (loop_edges={loop_edges!r})", stacklevel=2)
    if odometry_edges == "global_delta" and delta.any():
        th = head[delta]
        c, s = np.cos(th), np.sin(th)
        dx, dy = z[delta, 0, 2].copy(), z[delta, 1, 2].copy()
        z[delta, 0, 2] = c * dx + s * dy
        z[delta, 1, 2] = -s * dx + c * dy
    invert = ~delta & ((conv == 1) | ((conv == 0) & (loop_edges == "icp")))
    if invert.any():
        r = z[invert]
        inv = np.zeros_like(r)
        inv[:, :2, :2] = np.transpose(r[:, :2, :2], (0, 2, 1))        # R^T
        inv[:, :2, 2] = -np.einsum("eij,ej->ei", inv[:, :2, :2], r[:, :2, 2])
        inv[:, 2, 2] = 1.0
        z[invert] = inv
    return ea, eb, z


def _edges(pose_graph):
    ea, eb, tf = [], [], []
    for a, b, t in pose_graph.graph.edges(data="object"):
        ea.append(a)
        eb.append(b)
        tf.append(t)
    return np.asarray(ea, np.int32), np.asarray(eb, np.int32), np.asarray(tf, np.float64).reshape(-1, 3, 3)
