"""SE(2) helpers with the reference's exact conventions (``src/utils.py:3-36``).

These are host-side conversions at the boundary (pose vectors <-> 3x3
homogeneous matrices).  The device kernels inline the same formulas.
"""
import numpy as np


def odom_change_to_mat(delta):
    """``src/utils.py:3-19``: matrix [[c,-s,dx],[s,c,dy],[0,0,1]] of a delta."""
    dx, dy, dtheta = delta
    c = np.cos(dtheta)
    s = np.sin(dtheta)
    mat = np.eye(3)
    mat[0, 0] = c
    mat[0, 1] = -s
    mat[1, 0] = s
    mat[1, 1] = c
    mat[0, 2] = dx
    mat[1, 2] = dy
    return mat


def pose_to_mat(pose):
    """``src/utils.py:28-33``."""
    c, s = np.cos(pose[2]), np.sin(pose[2])
    return np.array([[c, -s, pose[0]], [s, c, pose[1]], [0, 0, 1]])


def mat_to_pose(mat):
    """``src/utils.py:35-36``: (m02, m12, atan2(m10, m00))."""
    return np.array([mat[0, 2], mat[1, 2], np.arctan2(mat[1, 0], mat[0, 0])])


def poses_to_mats(poses):
    """Vectorised ``pose_to_mat`` over (N,3) -> (N,3,3)."""
    poses = np.asarray(poses, dtype=np.float64)
    c, s = np.cos(poses[:, 2]), np.sin(poses[:, 2])
    m = np.zeros((len(poses), 3, 3))
    m[:, 0, 0] = c
    m[:, 0, 1] = -s
    m[:, 1, 0] = s
    m[:, 1, 1] = c
    m[:, 0, 2] = poses[:, 0]
    m[:, 1, 2] = poses[:, 1]
    m[:, 2, 2] = 1.0
    return m


def compose_chain(first_pose, tfs):
    """Odometry chain of ``scripts/main.py:249-256``.

    P_0 = first_pose; P_i = mat_to_pose(pose_to_mat(P_{i-1}) @ T_i).
    Serial by construction (each step re-derives the matrix from the pose
    vector, exactly as the reference does).
    """
    tfs = np.asarray(tfs, dtype=np.float64)
    out = np.zeros((len(tfs) + 1, 3))
    out[0] = first_pose
    for i in range(1, len(tfs) + 1):
        out[i] = mat_to_pose(pose_to_mat(out[i - 1]) @ tfs[i - 1])
    return out
