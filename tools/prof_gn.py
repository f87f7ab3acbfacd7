"""C4 Gauss-Newton iterations for rocprofv3 kernel-trace collection.  GPU only.
    python tools/prof_gn.py [iterations] [solver: 0 auto | 1 band | 2 bcr] [plan: default | noborder | nowrap]
nowrap: C4 without its 9 lap-wrap odometry edges (the band the border plan leaves; timing only)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
from slamhip import _abi, gn, synthetic  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
_abi.lib().slam_gn_set_solver(int(sys.argv[2]) if len(sys.argv) > 2 else 0)
guess, ea, eb, tf, _ = synthetic.lap_graph_c4()
mode = sys.argv[3] if len(sys.argv) > 3 else "default"
if mode == "nowrap":
    import numpy as np
    ea, eb, tf = np.asarray(ea), np.asarray(eb), np.asarray(tf)
    keep = ~((eb == ea + 1) & (eb % 500 == 0))
    ea, eb, tf = ea[keep], eb[keep], tf[keep]
plan = gn.GnPlan(len(guess), ea, eb, border=[] if mode == "noborder" else None)
s = gn.GaussNewton(guess, ea, eb, tf, plan=plan)
print(plan.ordering, s.run(iters))
