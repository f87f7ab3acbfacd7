"""Drop-in ``src/dataloader.py`` (lidar + odometry part) without ``lcm``/``cv2``.

Reference: ``/root/reference/src/dataloader.py``.

* ``get_point_cloud(ranges, thetas)`` (:47-55): ranges > 0.05 kept, angles
  NEGATED, x = r cos(-theta), y = r sin(-theta) — same NumPy expressions;
* ``get_all_lcm_data(data_folder_name)`` (:58-80): the ``*.log`` in the folder
  (the last one listed, as the reference's loop leaves it), ODOMETRY and LIDAR
  events decoded by slamhip.lcmlog (vectorised; identical values);
* ``align_data(..., images=None, ...)`` (:83-107, the no-image branch): each
  scan takes the odometry at ``np.searchsorted(odometry_timestamps, t)``
  (the last one past the end);
* ``parse_lcm_log(data_folder_name, ..., load_images=False)`` (:110-129).
  Images need OpenCV (absent): ``load_images=True`` raises.
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


def align_data(odometry, odometry_timestamps, point_clouds, point_cloud_timestamps, images=None,
               image_timestamps=None):
    if images is not None:
        raise NotImplementedError("image alignment needs the camera images (OpenCV), not part of this build")
    idx = np.searchsorted(odometry_timestamps, point_cloud_timestamps)
    idx = np.where(idx < odometry.shape[0], idx, -1)
    final_odometry = odometry[idx].reshape(-1, 3) if len(point_clouds) else np.empty((0, 3))
    return final_odometry, point_clouds


def parse_lcm_log(data_folder_name, start_time=0, stop_time=np.inf, load_images=True, image_stop=np.inf, n_jobs=-1):
    if load_images:
        raise NotImplementedError("load_images=True needs OpenCV (camera frames); use load_images=False")
    odometry, odometry_t, clouds, clouds_t = get_all_lcm_data(data_folder_name)
    return align_data(odometry, odometry_t, clouds, clouds_t)


def create_results_file_structure():
    if not os.path.exists("results"):
        os.makedirs("results")
