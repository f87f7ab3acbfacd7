"""Max |GPU - oracle| of the SGD step on the C4-size and >6,144-node graphs (tolerance study).  GPU only."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import pgo_oracle as po  # noqa: E402
import src.pose_graph as pgm  # noqa: E402
from slamhip import pgo, synthetic  # noqa: E402

for pps, laps, ncons, steps in ((125, 10, 15000, 1), (125, 10, 15000, 5), (150, 15, 3000, 3)):
    poses, loops = synthetic.lap_pose_graph(side_len=3.0, poses_per_side=pps, num_loops=laps, seed=0,
                                            num_constraints=ncons)
    pg = pgm.PoseGraph(poses.copy())
    for a, b in loops:
        pg.add_constraint(a, b, np.eye(3))
    ea, eb, tf = pg.edge_arrays()
    ref = poses.copy()
    s = pgo.SgdSolver(poses, ea, eb, tf)
    for k in range(steps):
        po.sgd_step(ref, ea, eb, tf, learning_rate=1.0 / (k + 1))
        s.step(1.0 / (k + 1))
    got = s.host_poses()
    dp = np.abs(got[:, :2] - ref[:, :2]).max()
    dth = np.abs(got[:, 2] - ref[:, 2]).max()
    print(f"N {len(poses)} E {len(ea)} steps {steps}: max|dpos| {dp:.3e} (max|pos| {np.abs(ref[:, :2]).max():.2f}), "
          f"max|dtheta| {dth:.3e} (max|theta| {np.abs(ref[:, 2]).max():.1f})", flush=True)
