"""Drop-in src/loop_closure_detection.py (reference src/loop_closure_detection.py):

* CPU: the module imports without OpenCV (the reference imports cv2 at module
  level, so scripts/main.py:19 fails without it); the proximity candidates
  follow the reference's path-length / distance rule (restated here);
* GPU: detect_proximity — candidates ICP'd in one batched launch, the greedy
  pass replayed — adds the same constraints, in the same order, as the
  reference's per-candidate loop run with the CPU oracle's icp().
"""
import sys

import numpy as np
import pytest
import scipy.spatial

from conftest import homog


def _ref_candidates(poses, min_dist_along_path, max_dist):
    # restatement of /root/reference/src/loop_closure_detection.py:12-25
    d = scipy.spatial.distance.cdist(poses[:, :2], poses[:, :2])
    walked = np.append([0], np.cumsum(np.diag(d, k=1)))
    m = []
    for i in range(len(poses)):
        s = np.searchsorted(walked, walked[i] + min_dist_along_path, side="right")
        if s >= len(poses):
            break
        c = s + np.argmin(d[i, s:])
        if d[i, c] <= max_dist:
            m.append((i, int(c)))
    m.reverse()
    return m


def test_imports_without_opencv(monkeypatch):
    import importlib
    monkeypatch.setitem(sys.modules, "cv2", None)   # "import cv2" raises ImportError
    import src.loop_closure_detection as lcd
    lcd = importlib.reload(lcd)
    assert callable(lcd.detect_proximity) and callable(lcd.detect_images_direct_similarity)
    with pytest.raises(ImportError, match="OpenCV"):
        lcd.find_keypoints(np.zeros((8, 8), np.uint8))


def test_proximity_candidates_rule():
    import src.loop_closure_detection as lcd
    from slamhip import synthetic
    seq = synthetic.make_loop_sequence(700, seed=3, n_beams=61)
    for mdp, md in ((2, 1), (5, 0.3), (1, 2.5)):
        assert lcd.proximity_candidates(seq.odometry, mdp, md) == _ref_candidates(seq.odometry, mdp, md)


class _Graph:
    def __init__(self, poses):
        self.poses = poses
        self.added = []

    def add_constraint(self, i, j, tf):
        self.added.append((i, j, np.array(tf)))


@pytest.mark.gpu
def test_detect_proximity_vs_reference_flow():
    import src.loop_closure_detection as lcd
    from slamhip import synthetic
    import icp_oracle
    seq = synthetic.make_loop_sequence(700, seed=5, n_beams=361)
    g = _Graph(seq.odometry.copy())
    lcd.detect_proximity(g, seq.scans, min_dist_along_path=2, max_dist=1, err_thresh=110)
    # the reference's loop (:27-39) with the CPU oracle's icp()
    want, used = [], set()
    for i, j in _ref_candidates(seq.odometry, 2, 1):
        if i in used or j in used:
            continue
        tfs, err = icp_oracle.icp(homog(seq.scans[j]), homog(seq.scans[i]), np.eye(3), 0.05, 100)
        if err < 110:
            want.append((i, j, tfs[-1]))
            used.update((i, j))
    assert len(want) > 3
    assert [(i, j) for i, j, _ in g.added] == [(i, j) for i, j, _ in want]
    for (_, _, a), (_, _, b) in zip(g.added, want):
        assert np.abs(a - b).max() <= 1e-9
