"""Per-call time of the drop-in pose_graph_optimization_step_sgd (networkx
graph in, poses written back) at the C4 size, against the device-resident
SgdSolver step.  GPU only."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
import torch  # noqa: E402
import src.pose_graph as pgm  # noqa: E402
import src.pose_graph_optimization as pgo  # noqa: E402
from slamhip import pgo as dpgo, synthetic  # noqa: E402

poses, loops = synthetic.lap_pose_graph(side_len=3.0, poses_per_side=125, num_loops=10, seed=0, num_constraints=15000)
pg = pgm.PoseGraph(poses.copy())
for a, b in loops:
    pg.add_constraint(a, b, np.eye(3))
pgo.pose_graph_optimization_step_sgd(pg)
ts = []
for k in range(5):
    t0 = time.perf_counter()
    pgo.pose_graph_optimization_step_sgd(pg, learning_rate=1.0 / (k + 2))
    ts.append(time.perf_counter() - t0)
t0 = time.perf_counter()
ea, eb, tf = pg.edge_arrays()
t_flat = time.perf_counter() - t0
s = dpgo.SgdSolver(pg.poses, ea, eb, tf)
s.step(1.0)
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(5):
    s.step(1.0 / (k + 2))
torch.cuda.synchronize()
print(f"drop-in step {np.median(ts) * 1e3:.1f} ms (edge_arrays {t_flat * 1e3:.1f} ms); device-resident step "
      f"{(time.perf_counter() - t0) / 5 * 1e3:.1f} ms; graph {len(poses)} nodes / {len(ea)} edges")
