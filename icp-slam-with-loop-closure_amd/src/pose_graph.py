"""Drop-in ``src/pose_graph.py``: the pose-graph container (reference
``src/pose_graph.py:21-73``).

Same data model as the reference: ``poses`` is an (N, 3) float64 array and
``graph`` a networkx DiGraph whose edges carry ``object=`` 3x3 SE(2)
transforms.  Iteration order of ``graph.edges(data="object")`` is the
networkx order the SGD pass relies on; ``edge_arrays()`` flattens it for the
device (new, cached until the graph changes).

New edge attributes (extra keys of the same nx edge dict, so they survive the
reference's ``(poses, DiGraph)`` pickle and are ignored by every
``edges(data="object")`` reader) record what each measurement means, for
Gauss-Newton (``optimize_pose_graph``), which needs X_b = X_a z for every edge:

* ``heading`` — set by the constructor on (i, i+1): the edge holds the
  GLOBAL-frame delta ``odom_change_to_mat(P[i+1] - P[i])`` taken at heading
  ``poses[i, 2]`` (reference :32-36);
* ``convention`` — set by ``add_constraint(..., convention=...)``:
  ``"icp"`` for the result T of ``icp(pc_i, pc_j)`` (X_i = X_j T: the manual
  and image loop closures, reference scripts/main.py:305,
  src/loop_closure_detection.py:141) or ``"relative"`` for X_j = X_i T (the
  proximity closures, which run ``icp(pc_j, pc_i)``, reference
  src/loop_closure_detection.py:34);
* ``constraint`` — set by every ``add_constraint`` call: the edge is a
  measurement added after construction (so an (i, i+1) edge carrying it is
  not a constructor delta, even without a convention).

An edge with none of these keys (a graph built by the reference's own
PoseGraph, a reference pickle, or a flipped graph) is classified per edge by
its shape: (i, i+1) is a constructor delta at the current heading.
"""
import pickle

import networkx as nx
import numpy as np

from slamhip.se2 import odom_change_to_mat

ODOM_INFORMATION = 2.0    # src/pose_graph.py:65 (information 2 I)
LOOP_INFORMATION = 5.0    # src/pose_graph.py:66 (information 5 I)
CONVENTIONS = ("icp", "relative")


class PoseGraph():
    def __init__(self, poses):
        """``poses`` (N, 3) or None (when the graph will be ``load``-ed).

        Successive poses are linked by ``odom_change_to_mat(poses[i+1] -
        poses[i])`` — a global-frame difference, exactly as the reference.
        """
        self.poses = poses
        self.graph = nx.DiGraph()
        self._flat = None
        if poses is None:
            return
        deltas = np.diff(poses, axis=0)
        self.graph.add_edges_from((i, i + 1, {"object": odom_change_to_mat(d), "heading": float(poses[i, 2])})
                                  for i, d in enumerate(deltas))

    def add_constraint(self, i, j, transformation, convention=None):
        """Adds (or overwrites, keeping its position) the edge i -> j.

        ``convention`` (new, optional): ``"icp"`` (X_i = X_j T) or
        ``"relative"`` (X_j = X_i T); see the module docstring.  An overwritten
        constructor edge is no longer a global delta."""
        if convention is not None and convention not in CONVENTIONS:
            raise ValueError(f"convention must be one of {CONVENTIONS} or None")
        self.graph.add_edge(i, j, object=transformation)
        attrs = self.graph.edges[i, j]
        attrs.pop("heading", None)
        attrs["constraint"] = True
        if convention is None:
            attrs.pop("convention", None)
        else:
            attrs["convention"] = convention
        self._flat = None

    def flip(self):
        """Reverse node order (theta + pi) and remap every edge a->b to
        (n-b)->(n-a); the pose array is reversed as a view, as in the reference.
        The flipped edges keep the reference's transforms unchanged, which no
        longer carry a known convention."""
        self.poses = self.poses[::-1]
        self.poses[:, 2] = (self.poses[:, 2] + np.pi) % (2 * np.pi)
        last = len(self.poses) - 1
        flipped = nx.DiGraph()
        flipped.add_edges_from((last - b, last - a, {"object": t}) for a, b, t in self.graph.edges(data="object"))
        self.graph = flipped
        self._flat = None

    def save(self, fname):
        with open(fname, "wb") as f:
            pickle.dump((self.poses, self.graph), f)

    def load(self, fname):
        # Only for pose graphs this pipeline wrote itself (pickle executes code).
        with open(fname, "rb") as f:
            self.poses, self.graph = pickle.load(f)
        self._flat = None

    def export_g2o(self, fname):
        rows = ["VERTEX_SE2 %d %f %f %f" % (i, p[0], p[1], p[2]) for i, p in enumerate(self.poses)]
        for a, b, t in self.graph.edges(data="object"):
            w = ODOM_INFORMATION if abs(b - a) == 1 else LOOP_INFORMATION
            rows.append("EDGE_SE2 %d %d %f %f %f %f %f %f %f %f %f" % (
                a, b, t[0, 2], t[1, 2], np.arctan2(t[1, 0], t[0, 0]), w, 0.0, 0.0, w, 0.0, w))
        with open(fname, "w") as f:
            f.write("".join(r + "\n" for r in rows))

    # ---- new: flattened views for the device kernels -------------------------
    @property
    def odometry_headings(self):
        """{a: heading} of the constructor's global-delta edges (a, a+1)."""
        return {a: h for a, b, h in self.graph.edges(data="heading") if h is not None}

    def edge_arrays(self):
        """(ea int32, eb int32, tf (E, 3, 3) float64) in networkx edge order.

        Cached: ``add_constraint`` / ``flip`` / ``load`` drop the cache, and
        a graph object or edge count changed behind the class's back does too
        (scripts/main.py:325-326 runs the SGD step 50 times on one graph).
        Edits that keep the edge count — ``graph.add_edge`` on an existing
        edge, ``graph[a][b]["object"] = T``, or mutating a stored transform in
        place — are NOT seen: make them through ``add_constraint`` or call
        ``invalidate()`` afterwards (checking every edge's contents per call
        would cost as much as the flattening the cache saves)."""
        n_edges = self.graph.number_of_edges()
        if self._flat is not None and self._flat[0] is self.graph and self._flat[1] == n_edges:
            return self._flat[2]
        ea, eb, tf = [], [], []
        for a, b, t in self.graph.edges(data="object"):
            ea.append(a)
            eb.append(b)
            tf.append(t)
        if not ea:
            out = np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros((0, 3, 3))
        else:
            out = (np.asarray(ea, dtype=np.int32), np.asarray(eb, dtype=np.int32),
                   np.asarray(tf, dtype=np.float64).reshape(-1, 3, 3))
        for a in out:
            a.flags.writeable = False   # shared by every caller of the cache
        self._flat = (self.graph, n_edges, out)
        return out

    def invalidate(self):
        """Drop the flattened-edge cache (and the drop-in SGD solver keyed on
        it) after editing ``graph`` directly."""
        self._flat = None
        self.__dict__.pop("_sgd_solver", None)

    def edge_kinds(self):
        """Per edge in nx order: (heading or NaN, convention code, added by
        ``add_constraint``) where the code is 0 unknown, 1 "icp", 2
        "relative"."""
        codes = {None: 0, "icp": 1, "relative": 2}
        head, conv, added = [], [], []
        for _, _, d in self.graph.edges(data=True):
            head.append(d.get("heading", np.nan))
            conv.append(codes.get(d.get("convention"), 0))
            added.append(bool(d.get("constraint", False)) or "convention" in d)
        return (np.asarray(head, dtype=np.float64), np.asarray(conv, dtype=np.int8),
                np.asarray(added, dtype=bool))
