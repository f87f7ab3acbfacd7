"""C4 Gauss-Newton iterations for rocprofv3 kernel-trace collection.  GPU only.
    python tools/prof_gn.py [iterations] [solver: 0 auto | 1 band | 2 bcr] [plan: default | noborder]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
from slamhip import _abi, gn, synthetic  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
_abi.lib().slam_gn_set_solver(int(sys.argv[2]) if len(sys.argv) > 2 else 0)
guess, ea, eb, tf, _ = synthetic.lap_graph_c4()
plan = gn.GnPlan(len(guess), ea, eb, border=[] if len(sys.argv) > 3 and sys.argv[3] == "noborder" else None)
s = gn.GaussNewton(guess, ea, eb, tf, plan=plan)
print(plan.ordering, s.run(iters))
