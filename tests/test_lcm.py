"""LCM log input (§8(f4), reference src/dataloader.py + src/lcmtypes): the
build's vectorised decoder against the reference's own LCM type code (the
fixture's messages were encoded and decoded by it, tests/golden/gen_lcm.py),
and the point-cloud conversion / odometry alignment restated from
src/dataloader.py:47-55, :83-107 (that module imports cv2 and lcm, absent)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _ref_point_cloud(ranges, thetas):
    """src/dataloader.py:47-55, restated."""
    r = np.array(ranges).reshape((-1, 1))
    th = -np.array(thetas).reshape((-1, 1))
    keep = 0.05 < r
    r, th = r[keep], th[keep]
    return np.hstack(((r * np.cos(th)).reshape((-1, 1)), (r * np.sin(th)).reshape((-1, 1))))


def test_codecs_match_reference_fixture():
    from slamhip import lcmlog
    e = np.load(os.path.join(GOLDEN, "lcm_expected.npz"))
    odo, lid = [], []
    for _, _, ch, data in lcmlog.read_events(os.path.join(GOLDEN, "lcm_run", "run.log")):
        if ch == "ODOMETRY":
            odo.append(lcmlog.decode_odometry(data))
        elif ch == "LIDAR":
            lid.append(lcmlog.decode_lidar(data))
    assert [o[0] for o in odo] == e["odo_t"].tolist()
    assert np.array_equal(np.array([o[1:] for o in odo]), e["odo"])
    off = e["off"]
    for k, (ut, r, th) in enumerate(lid):
        assert ut == e["lid_t"][k]
        assert np.array_equal(r, e["ranges"][off[k]:off[k + 1]])
        assert np.array_equal(th, e["thetas"][off[k]:off[k + 1]])
    # round trip through the build's encoders
    ut, r, th = lid[0]
    assert lcmlog.decode_lidar(lcmlog.encode_lidar(ut, r, th))[0] == ut


def test_parse_lcm_log_vs_restated_reference():
    import src.dataloader as dl
    e = np.load(os.path.join(GOLDEN, "lcm_expected.npz"))
    odometry, clouds = dl.parse_lcm_log(os.path.join(GOLDEN, "lcm_run"), load_images=False)
    off = e["off"]
    assert len(clouds) == len(off) - 1
    for k, c in enumerate(clouds):
        ref = _ref_point_cloud(e["ranges"][off[k]:off[k + 1]], e["thetas"][off[k]:off[k + 1]])
        assert np.array_equal(c, ref)
    for k in range(len(clouds)):   # align_data, no-image branch
        i = np.searchsorted(e["odo_t"].astype(float), float(e["lid_t"][k]))
        assert np.array_equal(odometry[k], e["odo"][i if i < len(e["odo"]) else -1])
    with pytest.raises(NotImplementedError):
        dl.parse_lcm_log(os.path.join(GOLDEN, "lcm_run"), load_images=True)


def test_bad_log_raises(tmp_path):
    from slamhip import lcmlog
    f = tmp_path / "bad.log"
    f.write_bytes(b"\x00" * 40)
    with pytest.raises(ValueError):
        list(lcmlog.read_events(str(f)))
    with pytest.raises(ValueError):
        lcmlog.decode_lidar(b"\x00" * 30)


def test_dataset_loader_reads_lcm_folder():
    from slamhip import dataset
    odometry, scans, pairs = dataset.load(os.path.join(GOLDEN, "lcm_run"))
    assert pairs is None and len(scans) == len(odometry) and odometry.shape[1] == 3
