"""Occupancy-grid mapping on the GPU (device side of the drop-in
``src/produce_occupancy_grid.py``; kernels in csrc/grid_kernels.hip).

``OccupancyMapper`` packs the scans once, computes the global points on the
device (``construct_global_points``, reference :75-87) and applies every beam's
Bresenham miss/hit updates (``bresenham_update``, :89-121) in ONE launch over
all beams; the int8 grid semantics are the reference's (see the kernel file
for the order-free per-cell rule).  Host work is O(scans): np.cos / np.sin of
each pose (the reference's own values) and the grid geometry arithmetic of
``produce_occupancy_grid`` (:31-53) on four scalars.
"""
import numpy as np

from . import _abi
from . import device as dv


def pose4(poses):
    """(S, 4): cos theta, sin theta, x, y — np.cos/np.sin per pose as
    src/utils.py:odom_change_to_mat evaluates them."""
    poses = np.asarray(poses, dtype=np.float64)
    out = np.empty((len(poses), 4))
    for i, p in enumerate(poses):
        out[i] = (np.cos(p[2]), np.sin(p[2]), p[0], p[1])
    return out


class OccupancyMapper:
    def __init__(self, poses, lidar_points, device=None):
        pts = [np.asarray(s, dtype=np.float64).reshape(-1, 2) for s in lidar_points]
        if len(pts) != len(poses):
            raise ValueError(f"{len(pts)} scans for {len(poses)} poses")
        if len(pts) == 0:
            raise ValueError("no scans")
        self.S = len(pts)
        self.lens = np.array([len(p) for p in pts], dtype=np.int64)
        off = np.zeros(self.S + 1, dtype=np.int64)
        off[1:] = np.cumsum(self.lens)
        self.P = int(off[-1])
        host = np.concatenate(pts, axis=0) if self.P else np.zeros((0, 2))
        if not np.all(np.isfinite(host)):
            raise ValueError("non-finite scan points")
        self.pts = dv.to_dev(host if self.P else np.zeros((1, 2)), np.float64, device)
        dev = self.pts.device
        self.off = dv.to_dev(off, np.int64, dev)
        self.pose4 = dv.to_dev(pose4(poses), np.float64, dev)
        self.gpts = dv.empty((max(self.P, 1), 2), np.float64, dev)
        self.bounds = dv.empty((4,), np.float64, dev)
        self._work = None
        self._work_cells = -1
        self._points_done = False

    def _ensure_work(self, H, W):
        n = int(_abi.lib().slam_grid_work_size(self.S, H, W))
        if self._work is None or self._work.numel() < n:
            self._work = dv.empty((n,), np.uint8, self.pts.device)

    def global_points(self):
        """construct_global_points on the device; returns (gpts (P, 2) device, bounds host (4,))."""
        if not self._points_done:
            self._ensure_work(1, 1)
            _abi.check(_abi.lib().slam_grid_global_points_f64(
                dv.ptr(self.pts), dv.ptr(self.off), self.S, dv.ptr(self.pose4), dv.ptr(self.gpts),
                dv.ptr(self.bounds), dv.ptr(self._work), dv.stream_handle()), "slam_grid_global_points_f64")
            self._points_done = True
        return self.gpts, self.bounds.cpu().numpy()

    def update(self, grid, cell_width, min_x, min_y, k_hit=3, k_miss=1):
        """update_occupancy_grid: ``grid`` (H, W) int8 host array, updated in place."""
        grid = np.asarray(grid)
        if grid.dtype != np.int8 or grid.ndim != 2:
            raise ValueError("occupancy grid must be a 2-D np.int8 array")
        H, W = grid.shape
        self.global_points()
        self._ensure_work(H, W)
        g = dv.to_dev(np.ascontiguousarray(grid), np.int8, self.pts.device)
        _abi.check(_abi.lib().slam_grid_update_i8(
            dv.ptr(self.gpts), dv.ptr(self.off), self.S, dv.ptr(self.pose4), self.P, float(min_x), float(min_y),
            float(cell_width), H, W, int(k_hit), int(k_miss), dv.ptr(g), dv.ptr(self._work),
            dv.stream_handle()), "slam_grid_update_i8")
        grid[...] = g.cpu().numpy().reshape(H, W)
        return grid
