"""One warm C3 batched-ICP launch (10k pairs x 1081 pts by default) for
rocprofv3 kernel-trace / PMC collection.  GPU only."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
import torch  # noqa: E402
from slamhip import _abi, se2, synthetic  # noqa: E402
from slamhip import icp as k  # noqa: E402

pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
inst = int(os.environ.get("SLAMHIP_INSTANCE", "-1"))
lib = _abi.lib()
lib.slam_icp_force_instance(inst)
lib.slam_icp_set_screen(int(os.environ.get("SLAMHIP_SCREEN", "2")))
lib.slam_icp_set_xcd_map(int(os.environ.get("SLAMHIP_XCD_MAP", "-1")))
seq = synthetic.make_sequence(pairs + 1, seed=2025)
inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, pairs + 1)])
ss = k.ScanSet(seq.scans)
batch = k.IcpBatch(ss, np.arange(1, pairs + 1), np.arange(0, pairs), inits, epsilon=0.05, max_iters=100)
for _ in range(reps):
    batch.launch()
torch.cuda.synchronize()
r = batch.result()
print("pairs", pairs, "mean iters", r.iters.mean(), "evals", float(np.sum(r.iters * ss.lens[1:] * ss.lens[:-1])))
