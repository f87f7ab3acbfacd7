"""GN iterations/s on C4 for A/B builds (SLAMHIP_LIB=...).  GPU only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
import torch  # noqa: E402,F401
from slamhip import gn  # noqa: E402

r = gn.bench_c4(iterations=10, reps=5)
print(os.environ.get("SLAMHIP_LIB", "cur"), r["gn_iters_per_sec"], r["gn_ms_per_iter"], r["gn_chi2_first_last"])
