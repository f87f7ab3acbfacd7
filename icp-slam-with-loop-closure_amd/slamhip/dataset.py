"""Scan-stream datasets for the batched driver.

The reference reads LCM logs (``src/dataloader.py:47-125``, needs the ``lcm``
package and the EECS_x logs, both unavailable here).  The driver takes the
same content — odometry poses (S, 3) and S ragged 2-D scans — from

* an ``.npz`` written by :func:`save` (``odometry``, ``scan_off``, ``scan_pts``
  and optionally ``loop_pairs``), or
* a generator spec ``synthetic:<walk|loop>:<n_scans>[:<seed>]`` (SURVEY.md
  §8(d) generator; ``loop`` also yields ground-truth loop pairs), or
* a reference dataset FOLDER holding an LCM ``*.log`` (ODOMETRY / LIDAR
  channels), read like src/dataloader.py's parse_lcm_log(load_images=False).
"""
import os

import numpy as np


def save(fname, odometry, scans, loop_pairs=None):
    scans = [np.asarray(s, dtype=np.float64)[:, :2] for s in scans]
    off = np.zeros(len(scans) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(s) for s in scans])
    extra = {} if loop_pairs is None else {"loop_pairs": np.asarray(loop_pairs, dtype=np.int64)}
    np.savez(fname, odometry=np.asarray(odometry, dtype=np.float64), scan_off=off,
             scan_pts=np.concatenate(scans, axis=0) if scans else np.zeros((0, 2)), **extra)


def load(spec):
    """-> (odometry (S, 3), scans list of (m_i, 2), loop_pairs (L, 2) or None)."""
    if spec.startswith("synthetic:"):
        from . import synthetic
        parts = spec.split(":")
        kind, n = parts[1], int(parts[2])
        seed = int(parts[3]) if len(parts) > 3 else 0
        if kind == "walk":
            seq = synthetic.make_sequence(n, seed=seed)
            return seq.odometry, seq.scans, None
        if kind == "loop":
            seq = synthetic.make_loop_sequence(n, seed=seed)
            return seq.odometry, seq.scans, seq.loop_pairs
        raise ValueError(f"unknown synthetic kind {kind!r} (walk | loop)")
    if os.path.isdir(spec):
        import src.dataloader as dl
        odometry, clouds = dl.parse_lcm_log(spec, load_images=False)
        return odometry, clouds, None
    with np.load(spec, allow_pickle=False) as z:
        off = z["scan_off"]
        pts = z["scan_pts"]
        scans = [pts[off[i]:off[i + 1]] for i in range(len(off) - 1)]
        pairs = z["loop_pairs"] if "loop_pairs" in z.files else None
        return z["odometry"], scans, pairs
