"""Pose-graph optimisation on the GPU (SGD relaxation + orientation recompute).

Device side of the drop-in ``src/pose_graph_optimization.py``:

* ``SgdSolver`` keeps poses, edges and scratch resident in HBM and runs
  ``slam_pgo_sgd_step_f64`` (reference ``src/pose_graph_optimization.py:7-49``)
  for any number of steps without host round trips;
* ``orient`` / ``orient_from_tf`` run the two halves of
  ``recompute_pose_graph_orientation`` (``:51-74``).
"""
import numpy as np

from . import _abi
from . import device as dv


class SgdSolver:
    def __init__(self, poses, ea, eb, tf, device=None):
        poses = np.ascontiguousarray(poses, dtype=np.float64)
        self.N = len(poses)
        self.E = len(ea)
        self.poses = dv.to_dev(poses, np.float64, device)
        dev = self.poses.device
        self.ea = dv.to_dev(np.asarray(ea, dtype=np.int32), np.int32, dev)
        self.eb = dv.to_dev(np.asarray(eb, dtype=np.int32), np.int32, dev)
        self.tf = dv.to_dev(np.asarray(tf, dtype=np.float64).reshape(-1, 9), np.float64, dev)
        n = int(_abi.lib().slam_pgo_sgd_work_size(self.N, self.E))
        self.work = dv.empty((max(n, 1),), np.float64, dev)

    def step(self, learning_rate=1.0, loop_closure_uncertainty=0.1, stream=None):
        _abi.check(_abi.lib().slam_pgo_sgd_step_f64(
            dv.ptr(self.poses), self.N, dv.ptr(self.ea), dv.ptr(self.eb), dv.ptr(self.tf), self.E,
            float(learning_rate), float(loop_closure_uncertainty), dv.ptr(self.work),
            dv.stream_handle(stream)), "slam_pgo_sgd_step_f64")

    def set_poses(self, poses):
        """Upload new (N, 3) poses into the resident buffer (same graph)."""
        p = np.ascontiguousarray(poses, dtype=np.float64).reshape(self.poses.shape)
        self.poses.copy_(dv.torch().from_numpy(p.copy() if not p.flags.writeable else p))

    def orient(self, stream=None):
        _abi.check(_abi.lib().slam_pgo_orient_f64(dv.ptr(self.poses), self.N, dv.stream_handle(stream)),
                   "slam_pgo_orient_f64")

    def host_poses(self):
        return self.poses.cpu().numpy().reshape(self.N, 3)


def sgd_step(poses, ea, eb, tf, learning_rate=1.0, loop_closure_uncertainty=0.1):
    """One step; returns the updated (N, 3) array (a new host array)."""
    s = SgdSolver(poses, ea, eb, tf)
    s.step(learning_rate, loop_closure_uncertainty)
    return s.host_poses()


def orient(poses):
    s = dv.to_dev(np.ascontiguousarray(poses, dtype=np.float64), np.float64)
    _abi.check(_abi.lib().slam_pgo_orient_f64(dv.ptr(s), len(poses), dv.stream_handle()), "slam_pgo_orient_f64")
    return s.cpu().numpy().reshape(-1, 3)


def orient_from_tf(poses, tfs):
    """theta_i = theta_{i-1}(old) + atan2(T_i[1,0], T_i[0,0]) for i = 1..N-1."""
    N = len(poses)
    p = dv.to_dev(np.ascontiguousarray(poses, dtype=np.float64), np.float64)
    t = dv.to_dev(np.asarray(tfs, dtype=np.float64).reshape(-1, 9), np.float64, p.device)
    w = dv.empty((max(N, 1),), np.float64, p.device)
    _abi.check(_abi.lib().slam_pgo_orient_from_tf_f64(dv.ptr(p), N, dv.ptr(t), dv.ptr(w), dv.stream_handle()),
               "slam_pgo_orient_from_tf_f64")
    return p.cpu().numpy().reshape(-1, 3)
