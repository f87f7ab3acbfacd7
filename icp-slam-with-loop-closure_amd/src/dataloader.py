"""Drop-in ``src/dataloader.py`` without ``lcm`` (and ``cv2`` until pixels are read).

Reference: ``/root/reference/src/dataloader.py``.

* ``get_point_cloud(ranges, thetas)`` (:47-55): ranges > 0.05 kept, angles
  NEGATED, x = r cos(-theta), y = r sin(-theta) — same NumPy expressions;
* ``get_all_lcm_data(data_folder_name)`` (:58-80): the ``*.log`` in the folder
  (the last one listed, as the reference's loop leaves it), ODOMETRY and LIDAR
  events decoded by slamhip.lcmlog (vectorised; identical values);
* ``get_images(data_folder_name, image_stop, n_jobs)`` (:25-44): the camera
  timestamps of ``image_timestamps.txt`` ("n, seconds" per line, times 1e6),
  the same ``image_stop`` clamp (``> len(lines)`` -> ``len(lines) - 1``) and
  frame count; the frames are returned as an ``ImageSequence`` that reads
  ``raw_images/image{n}.png`` with OpenCV only when its pixels are touched
  (the reference decodes every frame up front with a joblib pool);
* ``align_data`` (:83-107): both branches — with images, odometry and scans
  sampled at every image time by ``np.searchsorted`` (the last one past the
  end); without, the odometry at every scan time;
* ``parse_lcm_log(data_folder_name, ..., load_images=True, image_stop, n_jobs)``
  (:110-129): returns (odometry, point clouds, images) with images and
  (odometry, point clouds) without, as the reference does, so
  scripts/main.py:226 runs unchanged.
"""
import os

import numpy as np

from slamhip import lcmlog


def get_point_cloud(ranges, thetas):
    np_ranges = np.array(ranges).reshape((-1, 1))
    np_thetas = -np.array(thetas).reshape((-1, 1))
    valid = 0.05 < np_ranges
    np_ranges = np_ranges[valid]
    np_thetas = np_thetas[valid]
    x = np_ranges * np.cos(np_thetas)
    y = np_ranges * np.sin(np_thetas)
    return np.hstack((x.reshape((-1, 1)), y.reshape((-1, 1))))


def _log_file(folder):
    name = ""
    for f in os.listdir(folder):
        if f.endswith(".log"):
            name = os.path.join(folder, f)
    if not name:
        raise FileNotFoundError(f"no .log file in {folder}")
    return name


def get_all_lcm_data(data_folder_name):
    odo, odo_t, clouds, cloud_t = [], [], [], []
    for _, _, channel, data in lcmlog.read_events(_log_file(data_folder_name)):
        if channel == "ODOMETRY":
            utime, x, y, th = lcmlog.decode_odometry(data)
            odo.append((x, y, th))
            odo_t.append(utime)
        if channel == "LIDAR":
            utime, r, th = lcmlog.decode_lidar(data)
            clouds.append(get_point_cloud(r, th))
            cloud_t.append(utime)
    odometry = np.array(odo, dtype=float).reshape(-1, 3)
    return odometry, np.array(odo_t, dtype=float), clouds, np.array(cloud_t, dtype=float)


class ImageSequence:
    """The camera frames of ``get_images``: a sequence of ``len(names)`` frames
    ``raw_images/image{n}.png`` decoded on access by the reference's
    ``read_img`` (``cv2.imread(path, cv2.COLOR_BGR2RGB)``, :16-18).

    ``shape`` is (n, h, w, c) from the first frame's PNG header (no decoding;
    (n,) when it cannot be read); ``len``, iteration and indexing behave as
    on the reference's (n, h, w, 3) array: an integer gives one decoded frame,
    a slice or index array another ImageSequence, ``np.asarray`` every frame."""

    def __init__(self, folder, names):
        self.folder = folder
        self.names = list(names)

    def path(self, k):
        return f"{self.folder}/raw_images/image{self.names[k]}.png"

    def __len__(self):
        return len(self.names)

    @property
    def shape(self):
        n = len(self.names)
        hdr = _png_shape(self.path(0)) if n else None
        return (n,) + hdr if hdr else (n,)

    @property
    def ndim(self):
        return len(self.shape)

    def __getitem__(self, k):
        if isinstance(k, (int, np.integer)):
            return read_img(self.path(range(len(self.names))[int(k)]))
        if isinstance(k, slice):
            return ImageSequence(self.folder, self.names[k])
        idx = np.arange(len(self.names))[np.asarray(k)]
        return ImageSequence(self.folder, [self.names[i] for i in np.atleast_1d(idx)])

    def __iter__(self):
        return (self[i] for i in range(len(self.names)))

    def __array__(self, dtype=None, copy=None):
        a = np.asarray([self[i] for i in range(len(self.names))])
        return a.astype(dtype) if dtype is not None else a


def _png_shape(path):
    """(h, w[, channels]) from a PNG's IHDR chunk, or None."""
    try:
        with open(path, "rb") as f:
            head = f.read(26)
    except OSError:
        return None
    if len(head) < 26 or head[:8] != b"\x89PNG\r\n\x1a\n" or head[12:16] != b"IHDR":
        return None
    w, h = int.from_bytes(head[16:20], "big"), int.from_bytes(head[20:24], "big")
    # cv2.imread's flag 4 (the reference passes cv2.COLOR_BGR2RGB == IMREAD_ANYCOLOR):
    # grey frames stay 2-D, colour frames come back with 3 channels
    return (h, w) if head[25] in (0, 4) else (h, w, 3)


def read_img(path):
    """Reference :16-18 (needs OpenCV, imported on first use)."""
    try:
        import cv2
    except ImportError as e:
        raise ImportError("decoding the camera frames needs OpenCV (cv2); the timestamps, odometry and "
                          "scans of parse_lcm_log(load_images=True) do not") from e
    return cv2.imread(path, cv2.COLOR_BGR2RGB)


def get_image(data_folder_name, line):
    """Reference :20-23."""
    n, _ = line.split(", ")
    return read_img(f'{data_folder_name}/raw_images/image{n}.png')


def get_images(data_folder_name, image_stop, n_jobs):
    """Reference :25-44: (frames, timestamps in microseconds).  The frames
    are an ImageSequence (decoded on access); n_jobs is accepted and unused."""
    with open(f'{data_folder_name}/image_timestamps.txt', 'r') as f:
        lines = f.readlines()
    if image_stop > len(lines):
        image_stop = len(lines) - 1
    n = int(image_stop) + 1
    if n > len(lines):   # the reference reads lines[image_stop] and fails there too
        raise IndexError("list index out of range")
    names, timestamps = [], np.zeros(n, dtype=float)
    for i in range(0, n):
        k, time = lines[i].split(", ")
        names.append(k)
        timestamps[i] = float(time)
    timestamps *= 1E6
    return ImageSequence(data_folder_name, names), timestamps


def align_data(odometry, odometry_timestamps, point_clouds, point_cloud_timestamps, images=None,
               image_timestamps=None):
    """Reference :83-107.  With images: per image time, the odometry and the
    scan at ``np.searchsorted`` of it (the last one past the end); returns
    (odometry, point clouds, images).  Without: the odometry at every scan
    time; returns (odometry, point clouds)."""
    if images is not None:
        t = np.asarray(image_timestamps, dtype=float)[:images.shape[0]]
        oi = np.searchsorted(odometry_timestamps, t)
        oi = np.where(oi < odometry.shape[0], oi, -1)
        pi = np.searchsorted(point_cloud_timestamps, t)
        pi = np.where(pi < len(point_clouds), pi, -1)
        final_odometry = odometry[oi].reshape(-1, 3) if len(t) else np.empty((0, 3))
        return final_odometry, [point_clouds[i] for i in pi], images
    idx = np.searchsorted(odometry_timestamps, point_cloud_timestamps)
    idx = np.where(idx < odometry.shape[0], idx, -1)
    final_odometry = odometry[idx].reshape(-1, 3) if len(point_clouds) else np.empty((0, 3))
    return final_odometry, point_clouds


def parse_lcm_log(data_folder_name, start_time=0, stop_time=np.inf, load_images=True, image_stop=np.inf, n_jobs=-1):
    """Reference :110-129 (start_time / stop_time are unused there too)."""
    odometry, odometry_t, clouds, clouds_t = get_all_lcm_data(data_folder_name)
    if load_images:
        images, image_timestamps = get_images(data_folder_name, image_stop=image_stop, n_jobs=n_jobs)
    else:
        images, image_timestamps = None, None
    return align_data(odometry, odometry_t, clouds, clouds_t, images, image_timestamps)


def create_results_file_structure():
    if not os.path.exists("results"):
        os.makedirs("results")
