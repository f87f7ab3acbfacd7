"""Where the longest C3 pairs land in the scheduler's phase-2 order: run the
probe phase alone (slam_icp_set_schedule(probe, ...) with max_iters = probe
- 2 would stop them), so instead replay the scheduler's key on the host from
a probe-length run.  GPU only.

    python tools/sched_keys.py [pairs] [probe]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
import torch  # noqa: E402
from slamhip import _abi, se2, synthetic  # noqa: E402
from slamhip import icp as k  # noqa: E402

pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
probe = int(sys.argv[2]) if len(sys.argv) > 2 else 5
seq = synthetic.make_sequence(pairs + 1, seed=2025)
inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, pairs + 1)])
ss = k.ScanSet(seq.scans)
full = k.icp_batch(ss, np.arange(1, pairs + 1), np.arange(0, pairs), inits, epsilon=0.05, max_iters=100, history=True)
it = full.iters
# the phase-1 key: |E_probe - E_(probe-1)| from the error history is not returned; recompute
# it from the transform history with the oracle's error (host)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import icp_oracle  # noqa: E402
longest = np.argsort(it)[::-1][:12]
keys = np.full(pairs, np.inf)
cand = np.unique(np.r_[longest, np.random.default_rng(0).choice(pairs, 400, replace=False)])
for b in cand:
    if it[b] <= probe:
        continue
    pc1 = np.c_[seq.scans[b + 1], np.ones(len(seq.scans[b + 1]))]
    pc2 = np.c_[seq.scans[b], np.ones(len(seq.scans[b]))]
    e = []
    for t in (probe - 2, probe - 1):
        T = full.hist[b][t]
        q = (T @ pc1.T).T
        c = icp_oracle.correspondences(q, pc2)
        e.append(icp_oracle.sq_error(q, pc2[c]))
    keys[b] = abs(e[1] - e[0])
ks = keys[cand][np.isfinite(keys[cand])]
for b in longest:
    rank = float(np.mean(ks > keys[b]))   # fraction of sampled unfinished pairs with a larger key
    print(f"pair {b}: iters {it[b]}, key {keys[b]:.3g}, fraction of sampled pairs keyed slower {rank:.3f}")
print("iteration percentiles 50/90/99/99.9/max:", np.percentile(it, [50, 90, 99, 99.9]).tolist(), it.max())
