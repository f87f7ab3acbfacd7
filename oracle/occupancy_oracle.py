"""CPU oracle for the occupancy-grid mapper — TEST INFRASTRUCTURE ONLY.

Imported only by tests/ (never by the product path).  A plain restatement of
the reference's src/produce_occupancy_grid.py (cohnt/ICP-SLAM-with-Loop-
Closure), one beam at a time in the reference's loop order:

* global points (``construct_global_points``, :75-87): every point through
  ``odom_change_to_mat(pose) @ [x, y, 1]^T`` (src/utils.py:3-19), one 3x3 @ 3x1
  product per point as the reference does;
* grid geometry (``produce_occupancy_grid``, :12-57): min/max of all global
  points widened by half a cell, optional minimum extents, ``ceil`` cell counts;
* per beam (``bresenham_update``, :89-121): integer Bresenham from the robot's
  cell to the point's cell, a "miss" on every cell the loop visits (the
  endpoint included, before its "hit"), then a "hit" where the loop stopped.
  The odds arithmetic is int8 as in the reference: ``-128 - g`` and
  ``127 - g`` are evaluated on np.int8 scalars, so they wrap (a miss on a
  positive cell sets it to -128, a hit on a negative cell to 127) — the
  restatement uses the same expressions, hence the same wrap-around.

Parity: PINNED to the reference itself.  src/produce_occupancy_grid.py
imports cv2 at module level (only ``save_image`` uses it) and OpenCV is absent
here, so the module is not imported; tests/golden/gen_grid.py instead executes
the reference's own grid function definitions (extracted from its source with
``ast``: produce / update / construct_global_points / bresenham_update /
global_position_to_grid_cell, :12-138) and stores inputs and outputs in
tests/golden/grid_ref.npz.  tests/test_occupancy.py checks this file against
those fixtures bit for bit (grids, origins, global points), besides
hand-derived rays.
"""
import numpy as np


def odom_change_to_mat(delta):
    """src/utils.py:3-19."""
    dx, dy, dtheta = delta
    c, s = np.cos(dtheta), np.sin(dtheta)
    m = np.eye(3)
    m[0, 0], m[0, 1], m[1, 0], m[1, 1] = c, -s, s, c
    m[0, 2], m[1, 2] = dx, dy
    return m


def global_points(poses, scans):
    """construct_global_points (:75-87): list of (m_i, 2) float64."""
    out = []
    for pose, pts in zip(poses, scans):
        T = odom_change_to_mat(pose)
        g = np.zeros(pts.shape)
        for j in range(len(pts)):
            g[j] = (T @ np.array([[pts[j, 0]], [pts[j, 1]], [1.0]])).flatten()[:2]
        out.append(g)
    return out


def cell_of(pos, min_x, min_y, w):
    """global_position_to_grid_cell (:123-128): (row, column)."""
    col = np.floor((pos[0] - min_x) / w).astype(int)
    row = np.floor((pos[1] - min_y) / w).astype(int)
    return row, col


def ray_update(grid, pose_xy, point, min_x, min_y, w, k_hit, k_miss):
    """bresenham_update (:89-121) on an int8 grid, in place."""
    y0, x0 = cell_of(pose_xy, min_x, min_y, w)
    y1, x1 = cell_of(point, min_x, min_y, w)
    dx = np.abs(x1 - x0).astype(int)
    dy = -np.abs(y1 - y0).astype(int)
    sx = 1 if x1 > x0 else -1
    sy = 1 if y1 > y0 else -1
    err = dx + dy
    H, W = grid.shape
    with np.errstate(over="ignore"):
        while 0 <= x0 < W and 0 <= y0 < H:
            g = grid[y0, x0]
            grid[y0, x0] = g - k_miss if (-128 - g) < -k_miss else -128
            e2 = err * 2
            if e2 >= dy:
                if x0 == x1:
                    break
                err = err + dy
                x0 += sx
            if e2 <= dx:
                if y0 == y1:
                    break
                err = err + dx
                y0 += sy
        if 0 <= x0 < W and 0 <= y0 < H:
            g = grid[y0, x0]
            grid[y0, x0] = g + k_hit if (127 - g) > k_hit else 127


def geometry(gpts, cell_width, min_width=0, min_height=0):
    """Grid origin and size of produce_occupancy_grid (:31-53)."""
    allp = np.concatenate(gpts)
    min_x = np.min(allp[:, 0]) - (cell_width / 2)
    max_x = np.max(allp[:, 0]) + (cell_width / 2)
    min_y = np.min(allp[:, 1]) - (cell_width / 2)
    max_y = np.max(allp[:, 1]) + (cell_width / 2)
    wd, hd = max_x - min_x, max_y - min_y
    if wd < min_width:
        off = (min_width - wd) / 2
        min_x -= off
        wd = min_width
    if hd < min_height:
        off = (min_height - hd) / 2
        min_y -= off
        hd = min_height
    return min_x, min_y, int(np.ceil(wd / cell_width)), int(np.ceil(hd / cell_width))


def update(grid, poses, scans, cell_width, min_x, min_y, k_hit=3, k_miss=1, gpts=None):
    """update_occupancy_grid (:59-73), in place; returns grid."""
    gpts = global_points(poses, scans) if gpts is None else gpts
    for i in range(len(poses)):
        for j in range(len(scans[i])):
            ray_update(grid, poses[i, :2], gpts[i][j], min_x, min_y, cell_width, k_hit, k_miss)
    return grid


def produce(poses, scans, cell_width, min_width=0, min_height=0, k_hit=3, k_miss=1):
    """produce_occupancy_grid (:12-57): (grid int8 (H, W), (min_x, min_y))."""
    gpts = global_points(poses, scans)
    min_x, min_y, W, H = geometry(gpts, cell_width, min_width, min_height)
    grid = np.zeros((H, W), dtype=np.int8)
    update(grid, poses, scans, cell_width, min_x, min_y, k_hit, k_miss, gpts=gpts)
    return grid, (min_x, min_y)
