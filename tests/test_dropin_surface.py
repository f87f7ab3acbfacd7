"""The drop-in surface scripts/main.py and src/visualization.py bind (CPU).

Every attribute the reference's ``scripts/main.py`` (and ``src/visualization.py``
:85-98, which main.py calls through ``gen_and_save_map``) uses on the build's
``src`` modules resolves, and every call as written there binds to the
build's ``inspect.signature`` (same positional order, same keyword names).
The call shapes are transcribed from the reference with their file:line;
nothing here reads /root/reference at run time."""
import inspect

import numpy as np
import pytest

X = object()   # any argument value: only the binding is checked

# (module, attribute, positional args, keyword names) as the reference calls them
CALLS = [
    # scripts/main.py
    ("dataloader", "create_results_file_structure", 0, ()),                              # :30
    ("dataloader", "parse_lcm_log", 1, ("load_images", "image_stop", "n_jobs")),         # :226
    ("icp", "icp", 2, ("init_transform", "max_iters", "epsilon")),                       # :242-247, :303
    ("utils", "pose_to_mat", 1, ()),                                                     # :245, :252
    ("utils", "mat_to_pose", 1, ()),                                                     # :254
    ("pose_graph", "PoseGraph", 1, ()),                                                  # :277, :290
    ("loop_closure_detection", "detect_images_direct_similarity", 3,
     ("min_dist_along_path", "save_dists", "save_matches", "image_rate", "n_matches", "image_err_thresh",
      "icp_err_thresh")),                                                                # :294-296
    ("pose_graph_optimization", "pose_graph_optimization_step_sgd", 1, ("learning_rate",)),   # :326
    ("pose_graph_optimization", "recompute_pose_graph_orientation", 5, ("icp_recompute",)),  # :334
    # src/visualization.py (gen_and_save_map, draw_robot)
    ("produce_occupancy_grid", "produce_occupancy_grid", 3, ("kHitOdds", "kMissOdds")),  # :85
    ("produce_occupancy_grid", "grid_mle", 1, ("unknown_empty",)),                       # :87
    ("produce_occupancy_grid", "save_image", 2, ()),                                     # :96
    ("produce_occupancy_grid", "save_grid", 3, ()),                                      # :98
    ("utils", "pose_to_mat", 1, ()),                                                     # :25
    # src/loop_closure_detection.py / pose_graph_optimization.py (reference callers of the hot path)
    ("icp", "icp", 2, ("init_transform", "max_iters", "epsilon", "rotation_only")),      # p_g_o.py:61-68
    ("loop_closure_detection", "detect_proximity", 2, ()),                               # l_c_d.py:11
    ("utils", "odom_change_to_mat", 1, ()),                                              # p_o_g.py:89, pose_graph.py:36
]

# PoseGraph methods main.py uses (:278-279, :286-287, :291, :305, :308-309, :337-338)
PG_CALLS = [("save", 1), ("export_g2o", 1), ("load", 1), ("add_constraint", 3)]


@pytest.mark.parametrize("mod,attr,npos,kws", CALLS, ids=[f"{m}.{a}" for m, a, _, _ in CALLS])
def test_main_py_call_binds(mod, attr, npos, kws):
    import importlib
    m = importlib.import_module(f"src.{mod}")
    fn = getattr(m, attr)
    inspect.signature(fn).bind(*([X] * npos), **{k: X for k in kws})


def test_pose_graph_surface(tmp_path):
    """PoseGraph(None) + load, save, export_g2o, add_constraint, and the
    attributes visualization.py reads (poses, graph.edges)."""
    import src.pose_graph as pgm
    for name, npos in PG_CALLS:
        inspect.signature(getattr(pgm.PoseGraph, name)).bind(X, *([X] * npos))
    pg = pgm.PoseGraph(np.array([[0.0, 0.0, 0.0], [1.0, 0.0, 0.1], [2.0, 0.5, 0.2]]))
    pg.add_constraint(0, 2, np.eye(3))
    f = str(tmp_path / "g.pickle")
    pg.save(f)
    q = pgm.PoseGraph(None)
    q.load(f)
    assert np.array_equal(q.poses, pg.poses)
    assert sorted(tuple(e) for e in q.graph.edges) == [(0, 1), (0, 2), (1, 2)]
    q.export_g2o(str(tmp_path / "g.g2o"))
    assert q.poses[[0, 2], 0].tolist() == [0.0, 2.0]   # visualization.py:40 indexes poses by an edge


def test_main_py_load_unpacks_three_values():
    """scripts/main.py:226-230: three values, each sliceable by --dataset-start."""
    import os

    import src.dataloader as dl
    from conftest import GOLDEN
    odometry, lidar_points, images = dl.parse_lcm_log(os.path.join(GOLDEN, "lcm_run"), load_images=True,
                                                      image_stop=np.inf, n_jobs=-1)
    odometry, lidar_points, images = odometry[1:], lidar_points[1:], images[1:]
    assert len(odometry) == len(lidar_points) == len(images)
    assert odometry.shape[1] == 3 and all(p.shape[1] == 2 for p in lidar_points)
    raw = odometry[1:] - odometry[:-1]   # :238
    assert raw.shape == (len(odometry) - 1, 3)
