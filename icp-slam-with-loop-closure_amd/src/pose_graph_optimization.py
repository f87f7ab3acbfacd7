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
import numpy as np

from slamhip import icp as _icp
from slamhip import pgo as _pgo
from slamhip.se2 import pose_to_mat


def pose_graph_optimization_step_sgd(pose_graph, learning_rate=1, loop_closure_uncertainty=0.1):
    ea, eb, tf = pose_graph.edge_arrays() if hasattr(pose_graph, "edge_arrays") else _edges(pose_graph)
    out = _pgo.sgd_step(pose_graph.poses, ea, eb, tf, learning_rate, loop_closure_uncertainty)
    pose_graph.poses[...] = out


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
                        tol=1e-9, return_history=False):
    """Gauss-Newton on the SE(2) graph (relative-pose residuals, information
    2 I for odometry edges and 5 I for loop edges as ``PoseGraph.export_g2o``
    writes them); node 0 is held fixed.  Updates ``pose_graph.poses`` in place."""
    from slamhip import gn as _gn
    ea, eb, tf = pose_graph.edge_arrays() if hasattr(pose_graph, "edge_arrays") else _edges(pose_graph)
    solver = _gn.GaussNewton(pose_graph.poses, ea, eb, tf, odom_information, loop_information)
    hist = solver.run(iterations, tol)
    pose_graph.poses[...] = solver.host_poses()
    return hist if return_history else None


def _edges(pose_graph):
    ea, eb, tf = [], [], []
    for a, b, t in pose_graph.graph.edges(data="object"):
        ea.append(a)
        eb.append(b)
        tf.append(t)
    return np.asarray(ea, np.int32), np.asarray(eb, np.int32), np.asarray(tf, np.float64).reshape(-1, 3, 3)
