"""LCM log input (§8(f4), reference src/dataloader.py + src/lcmtypes): the
build's vectorised decoder against the reference's own LCM type code (the
fixture's messages were encoded and decoded by it, tests/golden/gen_lcm.py),
and the point-cloud conversion and both branches of the time alignment
against the reference's own ``get_point_cloud`` / ``align_data``
(tests/golden/dataloader_ref.npz, made by gen_dataloader.py, which runs those
two functions extracted from src/dataloader.py with ``ast``: the module
imports cv2 and lcm, absent here).  The event-log framing itself is the LCM
library's (absent): it is checked against the build's own writer only."""
import os

import numpy as np
import pytest

from conftest import GOLDEN


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


def _ref_clouds(d):
    off = d["cloud_off"]
    return [d["cloud_pts"][off[k]:off[k + 1]] for k in range(len(off) - 1)]


def test_point_cloud_vs_reference(golden):
    """get_point_cloud equals the reference's function bit for bit: the lidar
    scans of the fixture log and the 0.05 m cut (exactly 0.05 dropped)."""
    import src.dataloader as dl
    d = golden("dataloader_ref.npz")
    e = np.load(os.path.join(GOLDEN, "lcm_expected.npz"))
    off = e["off"]
    for k, ref in enumerate(_ref_clouds(d)):
        assert np.array_equal(dl.get_point_cloud(e["ranges"][off[k]:off[k + 1]].tolist(),
                                                 e["thetas"][off[k]:off[k + 1]].tolist()), ref), k
    got = dl.get_point_cloud(d["cut_ranges"], d["cut_thetas"])
    assert got.shape == (3, 2) and np.array_equal(got, d["cut_cloud"])


def test_parse_lcm_log_without_images_vs_reference(golden):
    """parse_lcm_log(load_images=False): the reference's align_data no-image
    branch (odometry at every scan time)."""
    import src.dataloader as dl
    d = golden("dataloader_ref.npz")
    odometry, clouds = dl.parse_lcm_log(os.path.join(GOLDEN, "lcm_run"), load_images=False)
    ref = _ref_clouds(d)
    assert len(clouds) == len(ref) and all(np.array_equal(c, r) for c, r in zip(clouds, ref))
    assert np.array_equal(odometry, d["noimg_odometry"])


def test_parse_lcm_log_with_images_vs_reference(golden):
    """parse_lcm_log(load_images=True), what scripts/main.py:226 calls: three
    values; odometry and scans sampled at the camera times of
    image_timestamps.txt exactly as the reference's align_data image branch
    does (times before, on, between and past the records); the frames are a
    lazy sequence (OpenCV only when pixels are read)."""
    import src.dataloader as dl
    d = golden("dataloader_ref.npz")
    folder = os.path.join(GOLDEN, "lcm_run")
    odometry, clouds, images = dl.parse_lcm_log(folder, load_images=True, image_stop=np.inf, n_jobs=-1)
    ref = _ref_clouds(d)
    assert np.array_equal(odometry, d["img_odometry"])
    assert len(clouds) == len(d["img_cloud_index"])
    for c, k in zip(clouds, d["img_cloud_index"]):
        assert np.array_equal(c, ref[k])
    assert len(images) == len(d["img_timestamps"]) == images.shape[0]
    _, ts = dl.get_images(folder, np.inf, -1)
    assert np.array_equal(ts, d["img_timestamps"])
    # image_stop (main.py passes --dataset-end): frames 0..image_stop
    o4, c4, im4 = dl.parse_lcm_log(folder, load_images=True, image_stop=3)
    assert len(im4) == 4 and np.array_equal(o4, d["img4_odometry"])
    assert all(np.array_equal(c, ref[k]) for c, k in zip(c4, d["img4_cloud_index"]))
    # image_stop == len(lines): the reference indexes past the file, and so does this
    with pytest.raises(IndexError):
        dl.get_images(folder, len(d["img_timestamps"]), -1)
    # main.py:228-230 slices all three by --dataset-start
    sub = images[2:]
    assert len(sub) == len(images) - 2 and sub.names == images.names[2:]


def test_align_data_with_an_image_array_vs_reference(golden):
    """align_data's image branch on an (n, h, w, 3) array shorter than the
    timestamps (it loops over images.shape[0]), returning the array itself."""
    import src.dataloader as dl
    d = golden("dataloader_ref.npz")
    e = np.load(os.path.join(GOLDEN, "lcm_expected.npz"))
    ref = _ref_clouds(d)
    ts = d["img_timestamps"]
    images = np.zeros((4, 2, 3, 3), dtype=np.uint8)
    o, c, im = dl.align_data(e["odo"].astype(float), e["odo_t"].astype(float), ref, e["lid_t"].astype(float),
                             images, ts)
    assert im is images and np.array_equal(o, d["img4_odometry"])
    assert all(p is ref[k] for p, k in zip(c, d["img4_cloud_index"]))


def test_image_sequence_is_lazy(tmp_path):
    """Frames: shape from the PNG header without decoding; reading pixels
    needs OpenCV, and says so when it is absent."""
    import src.dataloader as dl
    (tmp_path / "raw_images").mkdir()
    from PIL import Image
    Image.new("RGB", (7, 5)).save(tmp_path / "raw_images" / "image0.png")
    Image.new("RGB", (7, 5)).save(tmp_path / "raw_images" / "image1.png")
    (tmp_path / "image_timestamps.txt").write_text("0, 1.5\n1, 2.0\n")
    ims, ts = dl.get_images(str(tmp_path), np.inf, -1)
    assert ims.shape == (2, 5, 7, 3) and ims.ndim == 4 and ts.tolist() == [1.5e6, 2.0e6]
    assert ims[1:].shape == (1, 5, 7, 3) and ims[[1, 0]].names == ["1", "0"]
    try:
        import cv2  # noqa: F401
    except ImportError:
        with pytest.raises(ImportError, match="OpenCV"):
            ims[0]


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
