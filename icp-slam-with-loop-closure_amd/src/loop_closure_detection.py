"""Drop-in ``src/loop_closure_detection.py``: loop-closure search with the ICP
alignments batched on MI355X.

Same functions and arguments as the reference module
(``/root/reference/src/loop_closure_detection.py``), which ``scripts/main.py``
imports at start-up (``scripts/main.py:19``).  The reference imports OpenCV at
module level; here only the image path needs it and imports it when called,
so the module (and ``scripts/main.py``) imports on a host without cv2.

* ``detect_proximity`` (reference :11-39): candidate pairs from the pose
  geometry (same cdist / path-length rule), then ONE batched ICP launch over
  every candidate (init identity, eps 0.05, max_iters 100) instead of one
  ``icp.icp`` call per accepted candidate; the reference's greedy pass (reverse
  order, each node used once, ``error < err_thresh``) is replayed on the batch
  results.  A pair's ICP result does not depend on the others, so the
  constraints added are the reference's; candidates the greedy pass skips are
  computed and discarded.
* ``detect_images_direct_similarity`` (reference :81-175): ORB keypoints and
  descriptor matching stay OpenCV's (ImportError without it); the ICP
  alignment of the accepted image matches (reference :136-142, a joblib
  fan-out) is one batched launch.
"""
import numpy as np
import scipy.spatial

from slamhip import icp as _k
from slamhip.pipeline import add_loop_constraint


def _cv2():
    try:
        import cv2
    except ImportError as e:   # image loop closures need OpenCV, like the reference
        raise ImportError("image-based loop closure detection needs OpenCV (cv2); "
                          "detect_proximity does not") from e
    return cv2


def _homog(p):
    p = np.asarray(p, dtype=np.float64)
    return np.c_[p[:, :2], np.ones(len(p))]


def _path_geometry(poses):
    d = scipy.spatial.distance.cdist(poses[:, :2], poses[:, :2])
    walked = np.append([0], np.cumsum(np.diag(d, k=1)))
    return d, walked


def proximity_candidates(poses, min_dist_along_path=2, max_dist=1):
    """(i, j) pairs of reference :12-24, in the order the greedy pass visits them."""
    d, walked = _path_geometry(poses)
    out = []
    for i in range(len(poses)):
        s = np.searchsorted(walked, walked[i] + min_dist_along_path, side="right")
        if s >= len(poses):
            break
        j = s + int(np.argmin(d[i, s:]))
        if d[i, j] <= max_dist:
            out.append((i, j))
    out.reverse()
    return out


def detect_proximity(pose_graph, lidar_points, min_dist_along_path=2, max_dist=1, err_thresh=110):
    cand = proximity_candidates(pose_graph.poses, min_dist_along_path, max_dist)
    if not cand:
        return
    # icp(pc_j, pc_i) for every candidate, one launch (reference :33-35)
    res = _k.icp_pairs([_homog(lidar_points[j]) for _, j in cand], [_homog(lidar_points[i]) for i, _ in cand],
                       np.stack([np.eye(3)] * len(cand)), epsilon=0.05, max_iters=100)
    used = set()
    for b, (i, j) in enumerate(cand):
        if i in used or j in used:
            continue
        error = float(res.err[b])
        if error < err_thresh:
            print("%d %d %f" % (i, j, error))
            # icp(pc_j, pc_i): X_j = X_i T, the "relative" convention (src/pose_graph.py)
            add_loop_constraint(pose_graph, i, j, res.tf[b].copy(), "relative")
            used.update((i, j))


def serialize_keypoints(kp, des):
    return [(p.pt, p.size, p.angle, p.response, p.octave, p.class_id, d) for p, d in zip(kp, des)]


def deserialize_keypoints(serialized_keypoints):
    cv2 = _cv2()
    kp = [cv2.KeyPoint(x=s[0][0], y=s[0][1], size=s[1], angle=s[2], response=s[3], octave=s[4], class_id=s[5])
          for s in serialized_keypoints]
    return kp, np.array([s[6] for s in serialized_keypoints])


def serialize_matches(matches):
    return [(m.queryIdx, m.trainIdx, m.distance) for m in matches]


def deserialize_matches(serialized_matches):
    cv2 = _cv2()
    return [cv2.DMatch(s[0], s[1], s[2]) for s in serialized_matches]


def find_keypoints(img):
    kp, des = _cv2().ORB_create().detectAndCompute(img, None)
    return serialize_keypoints(kp, des)


def matchify(desc1, desc2, i, j, n_matches, approximate_match):
    cv2 = _cv2()
    if approximate_match:
        flann = cv2.FlannBasedMatcher(dict(algorithm=0, trees=5), dict(checks=50))
        matches = flann.match(np.asarray(desc1, np.float32), np.asarray(desc2, np.float32))
    else:
        matches = cv2.BFMatcher(cv2.NORM_HAMMING, crossCheck=True).match(desc1, desc2)
    matches = sorted(matches, key=lambda m: m.distance)
    if len(matches) < n_matches:
        return np.inf
    best = matches[:n_matches]
    return np.sum([m.distance for m in best]), serialize_matches(best), (i, j)


def detect_images_direct_similarity(pose_graph, lidar_points, images, image_rate=1, min_dist_along_path=5,
                                    image_err_thresh=125, n_matches=10, icp_err_thresh=30, save_dists=False,
                                    save_matches=False, n_jobs=-1, approximate_match=True):
    cv2 = _cv2()
    from joblib import Parallel, delayed
    d, walked = _path_geometry(pose_graph.poses)
    start = np.array([np.searchsorted(walked, w + min_dist_along_path, side="right") for w in walked])
    start[start == len(start)] = start[start == len(start)] * image_rate
    start = np.floor(start[::image_rate] / image_rate).astype(int)

    greys = [cv2.cvtColor(np.asarray(im, dtype=np.uint8), cv2.COLOR_RGB2GRAY) for im in images]
    par = Parallel(n_jobs=n_jobs, verbose=0, backend="loky")
    kps = par(delayed(find_keypoints)(greys[i]) for i in range(0, len(greys), image_rate))
    keypoints, descriptors = zip(*[deserialize_keypoints(s) for s in kps])
    scored = par(delayed(matchify)(descriptors[i], descriptors[j], i, j, n_matches, approximate_match)
                 for i in range(len(descriptors)) for j in range(start[i], len(descriptors)))
    dist_mat = np.full((len(descriptors), len(descriptors)), np.inf)
    matched = {}
    for r in scored:
        if np.isscalar(r):   # fewer than n_matches matches
            continue
        dist, ser, (i, j) = r
        dist_mat[i, j] = dist
        matched[(i, j)] = deserialize_matches(ser)
    print("Closest images keypoint match error %f" % np.min(dist_mat))
    if save_dists:
        import matplotlib.pyplot as plt
        for img, name in ((dist_mat, "dist_mat"), (dist_mat < image_err_thresh, "dist_mat_threshed")):
            fig, ax = plt.subplots()
            ax.imshow(img)
            plt.savefig("results/%s.png" % name)
            plt.close(fig)
    good = []
    for j in range(dist_mat.shape[1]):
        i = int(np.argmin(dist_mat[:, j]))
        if dist_mat[i, j] < image_err_thresh:
            good.append((i, j))
    if not good:
        return
    # reference :136-142: icp(pc_i, pc_j, init eye, max_iters 100, eps 0.05) per match -> one launch
    res = _k.icp_pairs([_homog(lidar_points[i * image_rate]) for i, _ in good],
                       [_homog(lidar_points[j * image_rate]) for _, j in good],
                       np.stack([np.eye(3)] * len(good)), epsilon=0.05, max_iters=100)
    for b, (i0, j0) in enumerate(good):
        i, j = i0 * image_rate, j0 * image_rate
        if float(res.err[b]) < icp_err_thresh:
            add_loop_constraint(pose_graph, i, j, res.tf[b].copy(), "icp")   # icp(pc_i, pc_j): X_i = X_j T
            if save_matches:
                img = cv2.drawMatches(greys[i], keypoints[i0], greys[j], keypoints[j0], matched.get((i0, j0), []), None,
                                      flags=cv2.DrawMatchesFlags_NOT_DRAW_SINGLE_POINTS)
                cv2.imwrite("results/match_%d_%d_%f.png" % (i, j, dist_mat[i0, j0]), img)
