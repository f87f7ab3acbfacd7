"""Cost of the k-th ICP iteration: the C3 batch (first P pairs) as ONE launch
(scheduler off) with max_iters = m - 2, i.e. every pair runs at most m
iterations; the time differences between m and m + 1 give the cost of
iteration m + 1 over the pairs still running.  GPU only.

    python tools/iter_cost.py [P]
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
    seq = synthetic.make_sequence(10001, seed=2025)
    inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, P + 1)])
    ss = k.ScanSet(seq.scans[:P + 1])
    lib.slam_icp_set_schedule(0, 1024)
    prev = None
    try:
        for m in (1, 2, 3, 4, 5, 6, 8, 12, 16, 24, 103):
            b = k.IcpBatch(ss, np.arange(1, P + 1), np.arange(0, P), inits, epsilon=0.05, max_iters=m - 2)
            b.launch()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                b.launch()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            it = b.result().iters
            t = float(np.median(ts))
            pit = int(it.sum())
            line = f"max {m:3d} iterations: {t:8.1f} us, {pit} pair-iterations, {t * 256 / pit:6.2f} CU-us per pair-iteration"
            if prev:
                dt, dp = t - prev[0], pit - prev[1]
                line += f"; marginal {dt * 256 / max(dp, 1):6.2f} CU-us per pair-iteration ({dp} more)"
            print(line, flush=True)
            prev = (t, pit)
    finally:
        lib.slam_icp_set_schedule(-1, 1024)


if __name__ == "__main__":
    main()
