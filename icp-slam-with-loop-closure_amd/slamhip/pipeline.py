"""Batched SLAM driver: the GPU flow of ``scripts/main.py`` stages 1-3.

The reference runs its hot path from ``scripts/main.py``:

* stage 1, scan matching (``scripts/main.py:236-263``): ``icp.icp`` on every
  consecutive pair (i, i-1) with init ``pose_to_mat(odom_i - odom_{i-1})``,
  fanned out over a joblib pool, then the serial odometry chain
  ``P_i = mat_to_pose(pose_to_mat(P_{i-1}) @ T_i)`` and a ``PoseGraph``;
* stage 2, manual loop closures (``scripts/main.py:298-307``): ``icp.icp``
  with an identity init for every annotated (i, j); the constraint is added
  when the returned error is below 30 (image-based detection needs OpenCV and
  stays out of scope);
* stage 3, optimisation (``scripts/main.py:322-334``): ``optimization_max_iters``
  SGD steps with learning rate 1/(k+1), then the orientation recompute.

Here each ICP stage is ONE batched kernel launch (``slamhip.icp.IcpBatch``),
the SGD steps run on a device-resident ``SgdSolver`` (poses stay in HBM for
all steps), and the Gauss-Newton solve (``slamhip.gn``) is available as an
alternative optimiser.  Results equal the reference flow's: the per-pair ICP
results are the reference's (tests/test_icp_gpu.py), the chain is composed on
the host with the reference's own arithmetic, and the SGD/orientation kernels
match ``oracle/pgo_oracle.py`` (tests/test_pipeline_gpu.py).
"""
from dataclasses import dataclass

import numpy as np

from . import se2

LOOP_CLOSURE_ICP_ERROR = 30.0   # scripts/main.py:306 (manual path; --loop-closure-icp-error for detection)


@dataclass
class ScanMatchResult:
    poses: np.ndarray      # (S, 3) corrected poses (odometry chain of the ICP edges)
    tf: np.ndarray         # (S-1, 3, 3) transforms[-1] of every pair (i, i-1)
    err: np.ndarray        # (S-1,) ICP errors
    iters: np.ndarray      # (S-1,) ICP iterations


def scan_matching(odometry, lidar_points, icp_max_iters=100, icp_epsilon=0.05, scanset=None):
    """Stage 1 (``scripts/main.py:236-256``) as one batched ICP launch."""
    from . import icp as _icp
    odometry = np.asarray(odometry, dtype=np.float64)
    S = len(odometry)
    if len(lidar_points) != S:
        raise ValueError(f"{len(lidar_points)} scans for {S} odometry poses")
    if S < 2:
        return ScanMatchResult(odometry.copy(), np.zeros((0, 3, 3)), np.zeros(0), np.zeros(0, np.int64))
    # per pair, like the reference (scalar np.cos/np.sin: no SIMD-path rounding differences)
    inits = np.stack([se2.pose_to_mat(odometry[i] - odometry[i - 1]) for i in range(1, S)])
    ss = scanset if scanset is not None else _icp.ScanSet(lidar_points)
    batch = _icp.IcpBatch(ss, np.arange(1, S), np.arange(0, S - 1), inits,
                          epsilon=icp_epsilon, max_iters=icp_max_iters)
    batch.launch()
    r = batch.result()
    poses = se2.compose_chain(odometry[0], r.tf)
    return ScanMatchResult(poses, r.tf, r.err, r.iters)


def read_manual_loop_closures(fname):
    """``np.loadtxt(fname, dtype=int)`` rows (i, j) as ``scripts/main.py:300``
    reads them (a single row is accepted too)."""
    m = np.loadtxt(fname, dtype=int)
    return np.atleast_2d(m).reshape(-1, 2)


def manual_loop_closures(pg, lidar_points, matches, max_iters=100, epsilon=0.05,
                         err_thresh=LOOP_CLOSURE_ICP_ERROR, scanset=None):
    """Stage 2, manual path (``scripts/main.py:298-307``): ICP(pc_i, pc_j,
    init = I) for every annotated pair in ONE launch; constraints are added
    in file order (``add_constraint`` overwrites a repeated (i, j) in place,
    networkx semantics), exactly as the reference's serial loop does.
    Returns the boolean mask of accepted matches."""
    from . import icp as _icp
    matches = np.asarray(matches, dtype=np.int64).reshape(-1, 2)
    if len(matches) == 0:
        return np.zeros(0, dtype=bool)
    ss = scanset if scanset is not None else _icp.ScanSet(lidar_points)
    inits = np.broadcast_to(np.eye(3), (len(matches), 3, 3))
    batch = _icp.IcpBatch(ss, matches[:, 0], matches[:, 1], inits, epsilon=epsilon, max_iters=max_iters)
    batch.launch()
    r = batch.result()
    ok = r.err < err_thresh
    for (i, j), t, good in zip(matches, r.tf, ok):
        if good:
            add_loop_constraint(pg, int(i), int(j), t.copy(), "icp")   # icp(pc_i, pc_j): X_i = X_j T
    return ok


def add_loop_constraint(pg, i, j, T, convention):
    """``pg.add_constraint(i, j, T)`` recording the measurement convention
    (src/pose_graph.py) when the graph type supports it — the reference's
    own PoseGraph (or any duck-typed graph) gets the plain call."""
    try:
        pg.add_constraint(i, j, T, convention=convention)
    except TypeError:
        pg.add_constraint(i, j, T)


def optimize(pg, lidar_points, optimization_max_iters=50, icp_max_iters=100, icp_epsilon=0.05,
             icp_recompute=False, method="sgd", gn_iterations=10):
    """Stage 3 (``scripts/main.py:322-334``): SGD steps with learning rate
    1/(k+1) on device-resident poses, then the orientation recompute; or, with
    ``method="gn"``, the Gauss-Newton solve followed by the same recompute.
    Updates ``pg.poses`` in place."""
    import src.pose_graph_optimization as pgo_drop_in
    if method == "sgd":
        from . import pgo as _pgo
        ea, eb, tf = pg.edge_arrays()
        solver = _pgo.SgdSolver(pg.poses, ea, eb, tf)
        for k in range(optimization_max_iters):
            solver.step(1.0 / float(k + 1))
        pg.poses[...] = solver.host_poses()
    elif method == "gn":
        pgo_drop_in.optimize_pose_graph(pg, iterations=gn_iterations)
    else:
        raise ValueError(f"unknown optimiser {method!r} (sgd | gn)")
    pgo_drop_in.recompute_pose_graph_orientation(pg, lidar_points, icp_max_iters, icp_epsilon, -1,
                                                 icp_recompute=icp_recompute)
    return pg
