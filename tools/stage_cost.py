"""Staging + first-iteration cost of the batched ICP kernel: the C3 batch as
ONE launch (scheduler off) with every pair stopped after 1 and after 2
iterations, for A/B builds (SLAMHIP_LIB=..., e.g. the SLAM_ABL_STAGE2X
timing-only build that stages every pair twice).  GPU only.

    python tools/stage_cost.py [P]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))


def main():
    import torch
    torch.cuda.set_device(0)
    from slamhip import _abi, se2, synthetic
    from slamhip import icp as k
    lib = _abi.lib()
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    seq = synthetic.make_sequence(P + 1, seed=2025)
    inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, P + 1)])
    ss = k.ScanSet(seq.scans)
    lib.slam_icp_set_schedule(0, 1024)
    out = []
    try:
        for m in (1, 2):
            b = k.IcpBatch(ss, np.arange(1, P + 1), np.arange(0, P), inits, epsilon=0.0, max_iters=m - 2,
                           stopping_thresh=-1.0)
            b.launch()
            torch.cuda.synchronize()
            ts = []
            for _ in range(7):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                b.launch()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            out.append(f"{m} it {np.median(ts):7.1f} us ({np.median(ts) * 256 / P:5.2f} CU-us/pair)")
    finally:
        lib.slam_icp_set_schedule(-1, 1024)
    print(os.environ.get("SLAMHIP_LIB", "cur"), "; ".join(out), flush=True)


if __name__ == "__main__":
    main()
