"""C4-size SGD steps and GN iterations for rocprofv3 kernel tracing. GPU only."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
import torch  # noqa: E402
from slamhip import gn, pgo, synthetic  # noqa: E402
import src.pose_graph as pgm  # noqa: E402

poses, loops = synthetic.lap_pose_graph(side_len=3.0, poses_per_side=125, num_loops=10, seed=0, num_constraints=15000)
pg = pgm.PoseGraph(poses.copy())
for a, b in loops:
    pg.add_constraint(a, b, np.eye(3))
ea, eb, tf = pg.edge_arrays()
s = pgo.SgdSolver(poses, ea, eb, tf)
for i in range(3):
    s.step(1.0 / (i + 1))
torch.cuda.synchronize()
guess, ea, eb, tf, _ = synthetic.lap_graph_c4()
g = gn.GaussNewton(guess, ea, eb, tf)
t0 = time.perf_counter()
print("gn chi2", g.run(5), "s", time.perf_counter() - t0)
