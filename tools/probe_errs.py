"""Per-pair error after m = 1..8 ICP iterations and the final iteration count
on the C3 workload (GPU), for the cost-prediction study of the phased
scheduler.  Writes gpurun_out/c3_probe.npz."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
import torch  # noqa: E402,F401
from slamhip import se2, synthetic  # noqa: E402
from slamhip import icp as k  # noqa: E402

pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
seq = synthetic.make_sequence(pairs + 1, seed=2025)
inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, pairs + 1)])
ss = k.ScanSet(seq.scans)
src, dst = np.arange(1, pairs + 1), np.arange(0, pairs)
errs, its = [], []
MS = list(range(1, 9)) + [11, 12, 15, 16, 23, 24, 31, 32, 47, 48]
for m in MS:
    r = k.icp_batch(ss, src, dst, inits, epsilon=0.05, max_iters=m - 2)
    errs.append(r.err)
    its.append(r.iters)
full = k.icp_batch(ss, src, dst, inits, epsilon=0.05, max_iters=100)
np.savez("gpurun_out/c3_probe.npz", ms=np.array(MS), errs=np.array(errs), its=np.array(its), final_iters=full.iters,
         init=inits, tf=full.tf)
print("ok", full.iters.mean())
