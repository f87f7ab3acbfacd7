#!/usr/bin/env python3
"""Batched GPU driver with the command line of the reference's scripts/main.py.

Runs the reference's program flow (``scripts/main.py:66-181`` flags,
``:230-339`` stages) with every ICP stage as one batched MI355X launch:

  scan_matching  ->  loop_closure (manual annotations)  ->  optimization

and writes the same artefacts under ``--results-dir``:
``icp_pose_graph.{pickle,g2o}`` (or ``odometry_pose_graph.*`` with
``--skip-icp``), ``loop_closure_pose_graph.*``, ``optim.*``, and the occupancy
grids of src/visualization.py:74-98 (``<name>_og.png``, ``<name>.map`` with
``--save-map-files``; names odometry / icp / final) built on the GPU.

Inputs: ``dataset`` is an ``.npz`` scan stream (slamhip.dataset.save) or a
generator spec ``synthetic:<walk|loop>:<n_scans>[:<seed>]``; for ``loop``
datasets ``--manual-loop-closures auto`` uses the generator's ground-truth
loop pairs.  Out of scope here (flags accepted, ignored): image-based loop
closure detection (OpenCV) and the matplotlib figures.

    python icp-slam-with-loop-closure_amd/scripts/main_batched.py synthetic:loop:2000:3 \\
        --manual-loop-closures auto --results-dir /tmp/results
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402

STAGES = ["scan_matching", "loop_closure", "optimization"]


def parse(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("dataset")
    p.add_argument("--program-start", default="scan_matching", choices=STAGES)
    p.add_argument("--program-end", default="optimization", choices=STAGES)
    p.add_argument("--skip-icp", action="store_true")
    p.add_argument("--icp-max-iters", default=100, type=int)
    p.add_argument("--icp-epsilon", default=0.05, type=float)
    p.add_argument("--pose-graph")
    p.add_argument("--n-jobs", default=-1, type=int, help="accepted; the GPU path needs no host pool")
    p.add_argument("--dataset-start", default=0, type=int)
    p.add_argument("--dataset-end", type=int)
    p.add_argument("--optimization-max-iters", default=50, type=int)
    p.add_argument("--manual-loop-closures",
                   help="text file of (i, j) rows, or 'auto' for a synthetic loop dataset's ground truth")
    p.add_argument("--loop-closure-icp-error", default=30, type=float,
                   help="accepted for compatibility; the manual path uses the reference's fixed 30")
    p.add_argument("--icp-recompute", action="store_true")
    p.add_argument("--optimizer", default="sgd", choices=["sgd", "gn"],
                   help="sgd = the reference's relaxation (default); gn = Gauss-Newton")
    p.add_argument("--gn-iterations", default=10, type=int)
    p.add_argument("--results-dir", default="results")
    p.add_argument("--cell-width", default=0.1, type=float)
    p.add_argument("--hit-odds", default=5, type=int)
    p.add_argument("--miss-odds", default=2, type=int)
    for f in ("--produce-odometry-map", "--skip-occupancy-grid", "--save-map-files", "--occupancy-grid-mle"):
        p.add_argument(f, action="store_true")
    # reference flags for figures / image matching: accepted, not used here
    for f, kw in (("--figure-dpi", dict(type=int)), ("--figure-width", dict(type=float)),
                  ("--figure-height", dict(type=float)), ("--image-downsample", dict(type=int)),
                  ("--image-match-error", dict(type=float)), ("--keypoint-n-matches", dict(type=int)),
                  ("--image-pointcloud-downsample", dict(type=int)), ("--min-dist-along-path", dict(type=int))):
        p.add_argument(f, **kw)
    for f in ("--save-icp-images", "--no-save-matches", "--no-save-dist-mat"):
        p.add_argument(f, action="store_true")
    a = p.parse_args(argv)
    if STAGES.index(a.program_end) < STAGES.index(a.program_start):
        p.error("--program-end precedes --program-start")
    if a.program_start != "scan_matching" and not a.pose_graph:
        p.error("starting after scan matching needs --pose-graph")
    return a


def save_map(a, poses, scans, name, report):
    """src/visualization.py:83-98 without the figures: the occupancy grid of
    `poses` (GPU), optionally its MLE, saved as <name>_og.png (+ <name>.map)."""
    if a.skip_occupancy_grid:
        return
    import src.produce_occupancy_grid as pog
    t0 = time.perf_counter()
    og, (min_x, min_y) = pog.produce_occupancy_grid(np.asarray(poses), scans, a.cell_width, kHitOdds=a.hit_odds,
                                                    kMissOdds=a.miss_odds)
    if a.occupancy_grid_mle:
        og = pog.grid_mle(og, unknown_empty=True)
    pog.save_image(og, os.path.join(a.results_dir, "%s_og.png" % name))
    if a.save_map_files:
        pog.save_grid(og, os.path.join(a.results_dir, "%s.map" % name), a.cell_width)
    report["map_" + name] = {"cells": list(og.shape), "origin": [float(min_x), float(min_y)],
                             "s": round(time.perf_counter() - t0, 3)}


def run(a):
    from slamhip import dataset, pipeline
    import src.pose_graph as pose_graph

    os.makedirs(a.results_dir, exist_ok=True)
    out = lambda name: os.path.join(a.results_dir, name)   # noqa: E731
    report = {"dataset": a.dataset}
    odometry, scans, gt_pairs = dataset.load(a.dataset)
    end = a.dataset_end if a.dataset_end is not None else len(odometry)
    odometry = np.asarray(odometry)[a.dataset_start:end]
    scans = list(scans)[a.dataset_start:end]
    report["scans"] = len(scans)
    if a.produce_odometry_map:
        save_map(a, odometry, scans, "odometry", report)

    pg = None
    if a.program_start == "scan_matching":
        t0 = time.perf_counter()
        if a.skip_icp:
            pg = pose_graph.PoseGraph(odometry.copy())
            stem = "odometry_pose_graph"
        else:
            r = pipeline.scan_matching(odometry, scans, a.icp_max_iters, a.icp_epsilon)
            pg = pose_graph.PoseGraph(r.poses)
            stem = "icp_pose_graph"
            report["icp_mean_iters"] = float(np.mean(r.iters)) if len(r.iters) else 0.0
        report["scan_matching_s"] = round(time.perf_counter() - t0, 3)
        if not a.skip_icp:
            save_map(a, pg.poses, scans, "icp", report)
        pg.save(out(stem + ".pickle"))
        pg.export_g2o(out(stem + ".g2o"))
    if a.program_end == "scan_matching":
        return report

    if pg is None:
        pg = pose_graph.PoseGraph(None)
        pg.load(a.pose_graph)
    if a.program_start in ("scan_matching", "loop_closure"):
        if a.manual_loop_closures is None:
            print("image-based loop closure detection needs OpenCV (out of scope); no loop closures added",
                  file=sys.stderr)
        else:
            if a.manual_loop_closures == "auto":
                if gt_pairs is None:
                    raise SystemExit("--manual-loop-closures auto needs a synthetic:loop dataset")
                matches = gt_pairs - a.dataset_start
                matches = matches[(matches >= 0).all(1) & (matches < len(scans)).all(1)]
            else:
                matches = pipeline.read_manual_loop_closures(a.manual_loop_closures)
            t0 = time.perf_counter()
            ok = pipeline.manual_loop_closures(pg, scans, matches)
            report["loop_closures"] = {"annotated": int(len(matches)), "accepted": int(ok.sum()),
                                       "s": round(time.perf_counter() - t0, 3)}
        pg.save(out("loop_closure_pose_graph.pickle"))
        pg.export_g2o(out("loop_closure_pose_graph.g2o"))
    if a.program_end == "loop_closure":
        return report

    t0 = time.perf_counter()
    pipeline.optimize(pg, scans, a.optimization_max_iters, a.icp_max_iters, a.icp_epsilon,
                      icp_recompute=a.icp_recompute, method=a.optimizer, gn_iterations=a.gn_iterations)
    report["optimization_s"] = round(time.perf_counter() - t0, 3)
    save_map(a, pg.poses, scans, "final", report)
    pg.save(out("optim.pickle"))
    pg.export_g2o(out("optim.g2o"))
    return report


def main(argv=None):
    rep = run(parse(argv))
    print(json.dumps(rep))


if __name__ == "__main__":
    main()
