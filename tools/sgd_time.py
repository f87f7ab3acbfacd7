"""SGD relaxation step time on the C4-size graph (A/B builds via SLAMHIP_LIB).  GPU only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
import bench  # noqa: E402

r = bench.pgo_bench()
print(os.environ.get("SLAMHIP_LIB", "cur"), "sgd_step_ms", r["sgd_step_ms"], "gn it/s", r.get("gn_iters_per_sec"))
