"""Drop-in ``src/pose_graph.py``: the pose-graph container (reference
``src/pose_graph.py:21-73``).

Same data model as the reference: ``poses`` is an (N, 3) float64 array and
``graph`` a networkx DiGraph whose edges carry ``object=`` 3x3 SE(2)
transforms (T takes node a's frame to node b's).  Iteration order of
``graph.edges(data="object")`` is the networkx order the SGD pass relies on;
``edge_arrays()`` flattens it for the device (new).
"""
import pickle

import networkx as nx
import numpy as np

from slamhip.se2 import odom_change_to_mat

ODOM_INFORMATION = 2.0    # src/pose_graph.py:65 (information 2 I)
LOOP_INFORMATION = 5.0    # src/pose_graph.py:66 (information 5 I)


class PoseGraph():
    def __init__(self, poses):
        """``poses`` (N, 3) or None (when the graph will be ``load``-ed).

        Successive poses are linked by ``odom_change_to_mat(poses[i+1] -
        poses[i])`` — a global-frame difference, exactly as the reference.
        """
        self.poses = poses
        self.graph = nx.DiGraph()
        # new (not pickled): node a's heading when the constructor wrote the
        # global-frame delta of edge (a, a+1) — what optimize_pose_graph needs
        # to re-express that edge in node a's frame for Gauss-Newton
        self.odometry_headings = {}
        if poses is None:
            return
        deltas = np.diff(poses, axis=0)
        self.graph.add_edges_from((i, i + 1, {"object": odom_change_to_mat(d)}) for i, d in enumerate(deltas))
        self.odometry_headings = {i: float(poses[i, 2]) for i in range(len(deltas))}

    def add_constraint(self, i, j, transformation):
        """Adds (or overwrites, keeping its position) the edge i -> j."""
        self.graph.add_edge(i, j, object=transformation)
        if j == i + 1:
            self.odometry_headings.pop(i, None)   # no longer the constructor's global delta

    def flip(self):
        """Reverse node order (theta + pi) and remap every edge a->b to
        (n-b)->(n-a); the pose array is reversed as a view, as in the reference."""
        self.poses = self.poses[::-1]
        self.poses[:, 2] = (self.poses[:, 2] + np.pi) % (2 * np.pi)
        last = len(self.poses) - 1
        self.odometry_headings = {}   # flipped edges are no longer constructor deltas
        flipped = nx.DiGraph()
        flipped.add_edges_from((last - b, last - a, {"object": t}) for a, b, t in self.graph.edges(data="object"))
        self.graph = flipped

    def save(self, fname):
        with open(fname, "wb") as f:
            pickle.dump((self.poses, self.graph), f)

    def load(self, fname):
        # Only for pose graphs this pipeline wrote itself (pickle executes code).
        with open(fname, "rb") as f:
            self.poses, self.graph = pickle.load(f)
        self.odometry_headings = {}   # unknown after a load: see optimize_pose_graph

    def export_g2o(self, fname):
        rows = ["VERTEX_SE2 %d %f %f %f" % (i, p[0], p[1], p[2]) for i, p in enumerate(self.poses)]
        for a, b, t in self.graph.edges(data="object"):
            w = ODOM_INFORMATION if abs(b - a) == 1 else LOOP_INFORMATION
            rows.append("EDGE_SE2 %d %d %f %f %f %f %f %f %f %f %f" % (
                a, b, t[0, 2], t[1, 2], np.arctan2(t[1, 0], t[0, 0]), w, 0.0, 0.0, w, 0.0, w))
        with open(fname, "w") as f:
            f.write("".join(r + "\n" for r in rows))

    # ---- new: flattened views for the device kernels -------------------------
    def edge_arrays(self):
        """(ea int32, eb int32, tf (E, 3, 3) float64) in networkx edge order."""
        ea, eb, tf = [], [], []
        for a, b, t in self.graph.edges(data="object"):
            ea.append(a)
            eb.append(b)
            tf.append(t)
        if not ea:
            return np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros((0, 3, 3))
        return (np.asarray(ea, dtype=np.int32), np.asarray(eb, dtype=np.int32),
                np.asarray(tf, dtype=np.float64).reshape(-1, 3, 3))
