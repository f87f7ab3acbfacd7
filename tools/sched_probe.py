"""How much of the C3 batch time is the long-tail of slow-converging pairs:
the same pairs launched in natural order, in descending order of their
(known) iteration counts, and ascending — as one launch (scheduler off) and
through the two-phase scheduler.  GPU only."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
import torch  # noqa: E402
from slamhip import se2, synthetic  # noqa: E402
from slamhip import icp as k  # noqa: E402

pairs = 10000
seq = synthetic.make_sequence(pairs + 1, seed=2025)
inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, pairs + 1)])
ss = k.ScanSet(seq.scans)
src, dst = np.arange(1, pairs + 1), np.arange(0, pairs)
r = k.icp_batch(ss, src, dst, inits, epsilon=0.05, max_iters=100)
from slamhip import _abi  # noqa: E402
lib = _abi.lib()
for name, perm, probe in (("natural", np.arange(pairs), 0), ("desc", np.argsort(-r.iters, kind="stable"), 0),
                          ("asc", np.argsort(r.iters, kind="stable"), 0), ("natural+scheduler", np.arange(pairs), 5),
                          ("desc+scheduler", np.argsort(-r.iters, kind="stable"), 5)):
    lib.slam_icp_set_schedule(probe, 2048)
    b = k.IcpBatch(ss, src[perm], dst[perm], inits[perm], epsilon=0.05, max_iters=100)
    b.launch()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.launch()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(name, "ms", round(float(np.median(ts)), 3))
