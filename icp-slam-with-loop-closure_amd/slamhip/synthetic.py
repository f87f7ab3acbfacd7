"""Deterministic synthetic 2-D lidar worlds.

The reference's datasets (``data/EECS_*``, fetched by ``scripts/download_data.py``)
are not available offline, so every benchmark and parity case runs on scans
produced here.  The generator mirrors the reference sensor model:

* an RPLidar-style scan, converted to points as ``src/dataloader.py:47-55``
  does (``x = r cos a``, ``y = r sin a``) and dropping returns with
  ``r <= 0.05`` (``src/dataloader.py:50``);
* 1081 beams over 270 degrees (the "1081-pt scans" of BASELINE.json);
* a closed rectangular room with square obstacles, ray-cast exactly;
* a random-walk trajectory and noisy odometry, so that
  ``scripts/main.py:241-247``'s initialisation
  ``pose_to_mat(odom_i - odom_{i-1})`` is a realistic ICP start.

Everything is float64 NumPy and seeded with ``numpy.random.default_rng``; the
arrays are the inputs of both the CPU oracle and the HIP path, so parity tests
compare like with like.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

N_BEAMS = 1081
FOV = 1.5 * np.pi          # 270 degrees
MIN_RANGE = 0.05           # src/dataloader.py:50 keeps r > 0.05


@dataclass
class World:
    width: float
    height: float
    obstacles: np.ndarray  # (k, 3): cx, cy, half-width (axis-aligned squares)


def make_world(rng: np.random.Generator, width=10.0, height=8.0, n_obstacles=4) -> World:
    obs = []
    while len(obs) < n_obstacles:
        h = rng.uniform(0.3, 0.5)
        cx = rng.uniform(1.5, width - 1.5)
        cy = rng.uniform(1.5, height - 1.5)
        if all(max(abs(cx - o[0]), abs(cy - o[1])) > h + o[2] + 0.8 for o in obs):
            obs.append((cx, cy, h))
    return World(width, height, np.asarray(obs, dtype=np.float64))


def beam_angles(n_beams: int = N_BEAMS) -> np.ndarray:
    k = np.arange(n_beams, dtype=np.float64)
    return -0.75 * np.pi + k * (FOV / (n_beams - 1))


def _clearance(world: World, x: float, y: float) -> float:
    c = min(x, y, world.width - x, world.height - y)
    for cx, cy, h in world.obstacles:
        c = min(c, max(abs(x - cx), abs(y - cy)) - h)
    return c


def raycast(world: World, poses: np.ndarray, angles: np.ndarray) -> np.ndarray:
    """Exact ranges for every (pose, beam): (S, n_beams) float64."""
    x = poses[:, 0:1]
    y = poses[:, 1:2]
    a = poses[:, 2:3] + angles[None, :]
    dx = np.cos(a)
    dy = np.sin(a)
    with np.errstate(divide="ignore", invalid="ignore"):
        tx = np.where(dx > 0, (world.width - x) / dx, np.where(dx < 0, (0.0 - x) / dx, np.inf))
        ty = np.where(dy > 0, (world.height - y) / dy, np.where(dy < 0, (0.0 - y) / dy, np.inf))
        r = np.minimum(tx, ty)
        for cx, cy, h in world.obstacles:
            t1x = (cx - h - x) / dx
            t2x = (cx + h - x) / dx
            t1y = (cy - h - y) / dy
            t2y = (cy + h - y) / dy
            tmin = np.maximum(np.minimum(t1x, t2x), np.minimum(t1y, t2y))
            tmax = np.minimum(np.maximum(t1x, t2x), np.maximum(t1y, t2y))
            hit = (tmax >= tmin) & (tmin > 0)
            r = np.where(hit & (tmin < r), tmin, r)
    return r


def random_walk(world: World, rng: np.random.Generator, n: int, step=0.05,
                heading_noise=0.03, margin=0.35) -> np.ndarray:
    poses = np.empty((n, 3), dtype=np.float64)
    x, y, th = world.width * 0.5, world.height * 0.2, 0.0
    while _clearance(world, x, y) < margin:
        x += 0.1
    for i in range(n):
        poses[i] = (x, y, th)
        th = th + rng.normal(0.0, heading_noise)
        for _ in range(64):
            nx_, ny_ = x + step * np.cos(th), y + step * np.sin(th)
            if _clearance(world, nx_, ny_) >= margin:
                break
            th += rng.uniform(0.4, 1.2)
        x, y = nx_, ny_
        th = float(np.arctan2(np.sin(th), np.cos(th)))
    return poses


def scans_from_poses(world: World, poses: np.ndarray, rng: np.random.Generator,
                     range_noise=0.01, n_beams=N_BEAMS, chunk=2048) -> list:
    """Ray-cast + noise + ``r > 0.05`` filter; returns list of (m_i, 2) float64."""
    angles = beam_angles(n_beams)
    out = []
    for s in range(0, len(poses), chunk):
        p = poses[s:s + chunk]
        r = raycast(world, p, angles)
        r = r + rng.normal(0.0, range_noise, size=r.shape)
        for i in range(len(p)):
            keep = r[i] > MIN_RANGE
            ri, ai = r[i][keep], angles[keep]
            out.append(np.stack([ri * np.cos(ai), ri * np.sin(ai)], axis=1))
    return out


@dataclass
class Sequence:
    world: World
    truth: np.ndarray       # (S, 3)
    odometry: np.ndarray    # (S, 3)
    scans: list             # S x (m_i, 2)


def make_sequence(n_scans: int, seed: int, n_beams=N_BEAMS, dropout=0.0) -> Sequence:
    """A scan stream like the reference's LCM logs (src/dataloader.py:106-125).

    dropout > 0: ragged scans — every scan loses a fraction U(0, dropout) of
    its beams at random positions, as returns with range <= 0.05 m that
    src/dataloader.py:47-55 filters out (dropout 0.35: 700-1081 points of
    1081).  Drawn from a separate generator: the stream itself (world, path,
    odometry, noise) is the same as without dropout."""
    rng = np.random.default_rng(seed)
    world = make_world(rng)
    truth = random_walk(world, rng, n_scans)
    odom = truth.copy()
    odom[:, 0:2] += rng.normal(0.0, 0.01, size=(n_scans, 2))
    odom[:, 2] += rng.normal(0.0, 0.005, size=n_scans)
    scans = scans_from_poses(world, truth, rng, n_beams=n_beams)
    if dropout > 0.0:
        drng = np.random.default_rng([seed, 0x5ca7])
        for i, sc in enumerate(scans):
            keep = drng.random(len(sc)) >= drng.uniform(0.0, dropout)
            keep[drng.integers(len(sc))] = True   # never empty
            scans[i] = sc[keep]
    return Sequence(world, truth, odom, scans)


def homogeneous(scan: np.ndarray) -> np.ndarray:
    """``np.c_[points, ones]`` exactly as ``scripts/main.py:242-243``."""
    return np.c_[scan, np.ones(len(scan))]


def sequence_pairs(seq: Sequence):
    """Pair list of ``scripts/main.py:241-247``: (pc_i, pc_{i-1}, init_i)."""
    from . import se2
    pairs = []
    for i in range(1, len(seq.scans)):
        init = se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1])
        pairs.append((i, i - 1, init))
    return pairs


def lap_pose_graph(side_len=3.0, poses_per_side=30, num_loops=4, seed=0,
                   pos_noise=0.01, theta_noise=0.025, num_constraints=100):
    """Seeded version of ``scripts/test_pose_graph_optimization.py:20-68``.

    Returns (poses (N,3), loop_edges list[(a, b)]) where every loop edge
    carries the identity transform, as the reference script adds.
    """
    rng = np.random.default_rng(seed)
    poses = []
    cur = [0.0, 0.0, 0.0]
    for _ in range(num_loops):
        for _ in range(4):
            for _ in range(poses_per_side):
                poses.append(cur.copy())
                cur[0] += (side_len / poses_per_side) * np.cos(cur[2])
                cur[1] += (side_len / poses_per_side) * np.sin(cur[2])
                cur[0] += rng.normal(0, pos_noise)
                cur[1] += rng.normal(0, pos_noise)
                cur[2] += rng.normal(0, theta_noise)
                cur[2] %= 2 * np.pi
            cur[2] += np.pi / 2
            cur[2] %= 2 * np.pi
    poses = np.array(poses)
    per_lap = poses_per_side * 4
    idx = rng.choice(per_lap, num_constraints, replace=True)
    laps = [rng.choice(num_loops, 2, replace=False) for _ in idx]
    edges = [(int(i + per_lap * l[0]), int(i + per_lap * l[1])) for i, l in zip(idx, laps)]
    edges.append((0, per_lap))
    edges.append((len(poses) - 1, len(poses) - 1 - per_lap))
    return poses, edges


def _wrap(a):
    return a - 2 * np.pi * np.floor((a + np.pi) / (2 * np.pi))


def lap_graph_c4(seed=0, poses_per_side=125, num_loops=10, side_len=3.0, n_loops=15001,
                 odo_xy=0.01, odo_th=0.01):
    """Config C4: 5,000-node / 20,000-edge SE(2) graph.

    Lap trajectory (side 3 m, 125 poses per side, 10 laps), 4,999 odometry
    edges with RELATIVE noisy measurements, 15,001 distinct loop edges between
    the same lap position on distinct laps (exact relative measurement), initial
    guess = dead reckoning of the odometry.  Returns (guess, ea, eb, tf, truth).
    """
    rng = np.random.default_rng(seed)
    per_lap = 4 * poses_per_side
    N = per_lap * num_loops
    step = side_len / poses_per_side
    truth = np.zeros((N, 3))
    for i in range(1, N):
        th = truth[i - 1, 2]
        truth[i, 0] = truth[i - 1, 0] + step * np.cos(th)
        truth[i, 1] = truth[i - 1, 1] + step * np.sin(th)
        truth[i, 2] = th + (np.pi / 2 if i % poses_per_side == 0 else 0.0)
    truth[:, 2] = _wrap(truth[:, 2])

    def rel(a, b):
        c, s = np.cos(a[2]), np.sin(a[2])
        d = b[:2] - a[:2]
        return np.array([c * d[0] + s * d[1], -s * d[0] + c * d[1], _wrap(b[2] - a[2])])

    def mat(p):
        c, s = np.cos(p[2]), np.sin(p[2])
        return np.array([[c, -s, p[0]], [s, c, p[1]], [0, 0, 1.0]])

    ea, eb, tf = [], [], []
    guess = np.zeros((N, 3))
    for i in range(N - 1):
        m = rel(truth[i], truth[i + 1]) + np.array([rng.normal(0, odo_xy), rng.normal(0, odo_xy),
                                                     rng.normal(0, odo_th)])
        ea.append(i)
        eb.append(i + 1)
        tf.append(mat(m))
        c, s = np.cos(guess[i, 2]), np.sin(guess[i, 2])
        guess[i + 1] = [guess[i, 0] + c * m[0] - s * m[1], guess[i, 1] + s * m[0] + c * m[1], _wrap(guess[i, 2] + m[2])]
    pairs = set()
    while len(pairs) < n_loops:
        pos = int(rng.integers(per_lap))
        l1, l2 = sorted(rng.choice(num_loops, 2, replace=False))
        pairs.add((pos + per_lap * int(l1), pos + per_lap * int(l2)))
    for a, b in sorted(pairs):
        ea.append(a)
        eb.append(b)
        tf.append(mat(rel(truth[a], truth[b])))
    return guess, np.array(ea), np.array(eb), np.stack(tf), truth


@dataclass
class LoopSequence(Sequence):
    per_lap: int = 0
    loop_pairs: np.ndarray = None   # (L, 2) ground-truth (earlier, later) scan pairs at the same lap position


def make_loop_sequence(n_scans: int, seed: int, n_beams=N_BEAMS, step=0.05, loop_every=10,
                       inset=1.2, lap_jitter=0.04) -> LoopSequence:
    """Config C5 stand-in: an indoor loop — the robot drives
    laps of a rectangle inset ``inset`` m from the walls of the same 10 x 8 m
    room (obstacles kept in the middle, off the path), each lap shifted by a
    small random lateral offset.  Scans at the same lap position on successive
    laps form the ground-truth loop pairs (every ``loop_every``-th position),
    which the manual loop-closure path (scripts/main.py:298-307) consumes
    instead of the OpenCV image matcher."""
    rng = np.random.default_rng(seed)
    width, height = 10.0, 8.0
    obs = []
    while len(obs) < 3:   # obstacles in the central region, clear of the loop
        h = rng.uniform(0.3, 0.5)
        cx = rng.uniform(inset + 1.5, width - inset - 1.5)
        cy = rng.uniform(inset + 1.3, height - inset - 1.3)
        if all(max(abs(cx - o[0]), abs(cy - o[1])) > h + o[2] + 0.5 for o in obs):
            obs.append((cx, cy, h))
    world = World(width, height, np.asarray(obs, dtype=np.float64))
    lx, ly = width - 2 * inset, height - 2 * inset
    perim = 2 * (lx + ly)
    per_lap = int(round(perim / step))
    s = np.arange(n_scans, dtype=np.float64) * step
    lap = (s // perim).astype(np.int64)
    u = np.mod(s, perim)
    n_laps = int(lap.max()) + 1
    off = rng.normal(0.0, lap_jitter, size=n_laps)[lap]          # per-lap lateral offset
    x = np.empty(n_scans)
    y = np.empty(n_scans)
    th = np.empty(n_scans)
    e1, e2, e3 = lx, lx + ly, 2 * lx + ly
    seg = np.select([u < e1, u < e2, u < e3], [0, 1, 2], 3)
    # counter-clockwise: bottom (+x), right (+y), top (-x), left (-y); offset pushes inward
    x = np.where(seg == 0, inset + u, np.where(seg == 1, width - inset - off,
                 np.where(seg == 2, width - inset - (u - e2), inset + off)))
    y = np.where(seg == 0, inset + off, np.where(seg == 1, inset + (u - e1),
                 np.where(seg == 2, height - inset - off, height - inset - (u - e3))))
    th = np.select([seg == 0, seg == 1, seg == 2], [0.0, 0.5 * np.pi, np.pi], -0.5 * np.pi)
    th = th + rng.normal(0.0, 0.01, size=n_scans)
    th = np.arctan2(np.sin(th), np.cos(th))
    truth = np.stack([x, y, th], axis=1)
    odom = truth.copy()
    odom[:, 0:2] += rng.normal(0.0, 0.01, size=(n_scans, 2))
    odom[:, 2] += rng.normal(0.0, 0.005, size=n_scans)
    scans = scans_from_poses(world, truth, rng, n_beams=n_beams)
    later = np.arange(per_lap, n_scans, loop_every)
    pairs = np.stack([later - per_lap, later], axis=1) if len(later) else np.zeros((0, 2), np.int64)
    return LoopSequence(world, truth, odom, scans, per_lap=per_lap, loop_pairs=pairs.astype(np.int64))
