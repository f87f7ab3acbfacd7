"""Host logic of the batched driver (no GPU): command line, dataset files,
manual loop-closure files, the loop generator's ground truth."""
import os
import sys

import numpy as np
import pytest

from conftest import PKG

sys.path.insert(0, os.path.join(PKG, "scripts"))


def test_cli_stage_validation():
    import main_batched as mb
    a = mb.parse(["synthetic:walk:5"])
    assert (a.program_start, a.program_end, a.icp_max_iters, a.icp_epsilon, a.optimization_max_iters) == \
        ("scan_matching", "optimization", 100, 0.05, 50)
    with pytest.raises(SystemExit):
        mb.parse(["x.npz", "--program-start", "optimization", "--program-end", "scan_matching",
                  "--pose-graph", "g.pickle"])
    with pytest.raises(SystemExit):
        mb.parse(["x.npz", "--program-start", "loop_closure"])          # needs --pose-graph
    # reference flags that do not apply are still accepted
    mb.parse(["x.npz", "--figure-dpi", "50", "--skip-occupancy-grid", "--image-downsample", "2"])


def test_dataset_roundtrip(tmp_path):
    from slamhip import dataset
    rng = np.random.default_rng(0)
    scans = [rng.normal(size=(n, 2)) for n in (5, 9, 1)]
    odo = rng.normal(size=(3, 3))
    f = str(tmp_path / "d.npz")
    dataset.save(f, odo, scans, loop_pairs=[[0, 2]])
    o2, s2, lp = dataset.load(f)
    assert np.array_equal(o2, odo) and all(np.array_equal(a, b) for a, b in zip(s2, scans))
    assert lp.tolist() == [[0, 2]]
    dataset.save(f, odo, scans)
    assert dataset.load(f)[2] is None


def test_manual_loop_closure_file(tmp_path):
    from slamhip import pipeline
    f = tmp_path / "m.txt"
    f.write_text("3 10\n")
    assert pipeline.read_manual_loop_closures(str(f)).tolist() == [[3, 10]]
    f.write_text("3 10\n4 11\n")
    assert pipeline.read_manual_loop_closures(str(f)).tolist() == [[3, 10], [4, 11]]


def test_loop_sequence_ground_truth():
    from slamhip import synthetic
    s = synthetic.make_loop_sequence(1200, seed=5)
    assert len(s.scans) == 1200 and s.per_lap > 0
    a, b = s.loop_pairs[:, 0], s.loop_pairs[:, 1]
    assert np.all(b - a == s.per_lap) and np.all(a < b)
    # the same lap position: within the per-lap jitter, heading noise only
    assert np.linalg.norm(s.truth[a, :2] - s.truth[b, :2], axis=1).max() < 0.3
