"""Drop-in ``src/produce_occupancy_grid.py`` on MI355X.

Same functions and return types as the reference
(``/root/reference/src/produce_occupancy_grid.py``):

* ``produce_occupancy_grid(poses, lidar_points, cell_width, min_width=0,
  min_height=0, kHitOdds=3, kMissOdds=1)`` -> (int8 grid (H, W), (min_x, min_y))
  (:12-57) — global points, bounds and every beam's update on the GPU
  (slamhip.grid, csrc/grid_kernels.hip); the grid geometry is computed on the
  host from the device bounds with the reference's own arithmetic;
* ``update_occupancy_grid(occupancy_grid, poses, lidar_points, cell_width,
  min_x, min_y, kHitOdds=3, kMissOdds=1)`` (:59-73) — updates the int8 grid in
  place and returns it;
* ``construct_global_points``, ``global_position_to_grid_cell``, ``grid_mle``,
  ``save_grid`` as the reference (``bresenham_update``, the reference's
  per-beam helper, is the body of the device kernel and has no host twin).
* ``save_image`` writes an 8-bit grayscale PNG with the standard library (the
  reference uses cv2.imwrite, and OpenCV is not part of this build).

Deviation (checked): kHitOdds and kMissOdds must be integers in [1, 127].
Global points are rounded as the reference's per-point 3x3 @ 3x1 NumPy product
rounds them on the build host (fma(a0, x0, a1 x1) + a2 x2), so grids and origins
match the reference's own functions bit for bit (tests/golden/grid_ref.npz).
"""
import struct
import zlib

import numpy as np

from slamhip import grid as _grid


def produce_occupancy_grid(poses, lidar_points, cell_width, min_width=0, min_height=0, kHitOdds=3, kMissOdds=1):
    poses = np.asarray(poses, dtype=np.float64)
    m = _grid.OccupancyMapper(poses, lidar_points)
    _, b = m.global_points()
    min_x = b[0] - (cell_width / 2)
    max_x = b[1] + (cell_width / 2)
    min_y = b[2] - (cell_width / 2)
    max_y = b[3] + (cell_width / 2)
    width_dist = max_x - min_x
    height_dist = max_y - min_y
    if width_dist < min_width:
        offset = (min_width - width_dist) / 2
        min_x -= offset
        width_dist = min_width
    if height_dist < min_height:
        offset = (min_height - height_dist) / 2
        min_y -= offset
        height_dist = min_height
    W = int(np.ceil(width_dist / cell_width))
    H = int(np.ceil(height_dist / cell_width))
    grid = np.zeros((H, W), dtype=np.int8)
    m.update(grid, cell_width, min_x, min_y, kHitOdds, kMissOdds)
    return grid, (min_x, min_y)


def update_occupancy_grid(occupancy_grid, poses, lidar_points, cell_width, min_x, min_y, kHitOdds=3, kMissOdds=1):
    m = _grid.OccupancyMapper(np.asarray(poses, dtype=np.float64), lidar_points)
    return m.update(occupancy_grid, cell_width, min_x, min_y, kHitOdds, kMissOdds)


def construct_global_points(poses, lidar_points):
    m = _grid.OccupancyMapper(np.asarray(poses, dtype=np.float64), lidar_points)
    g, _ = m.global_points()
    g = g.cpu().numpy()[:m.P]
    out, o = [], 0
    for n in m.lens:
        out.append(g[o:o + n].copy())
        o += n
    return out


def global_position_to_grid_cell(pos, min_x, min_y, cell_width):
    horizontal = np.floor((pos[0] - min_x) / cell_width).astype(int)
    vertical = np.floor((pos[1] - min_y) / cell_width).astype(int)
    return (vertical, horizontal)


def grid_mle(grid, unknown_empty=True):
    grid = grid.copy()
    grid[grid > 0] = 127
    grid[grid < 0] = -128
    return grid


def save_grid(grid, fname, cell_width):
    """EECS 467 .map text format: header, then rows top (max y) to bottom."""
    with open(fname, "w") as f:
        f.write("%d %d %d %d %f\n" % (0, 0, grid.shape[1], grid.shape[0], cell_width))
        for i in range(grid.shape[0] - 1, -1, -1):
            f.write("".join("%d " % v for v in grid[i]) + "\n")


def save_image(grid, fname):
    """127 - grid as uint8, rows flipped (top = max y), 8-bit grayscale PNG."""
    img = np.asarray(127 - grid.astype(np.int16), dtype=np.uint8)[::-1, :]
    h, w = img.shape
    raw = b"".join(b"\x00" + img[r].tobytes() for r in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)
    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 0, 0, 0, 0)) + \
        chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b"")
    with open(fname, "wb") as f:
        f.write(png)
