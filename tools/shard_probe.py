"""Where a strong-scaling shard's time goes: rank 0's shard of the C3 stream
(first P pairs) timed as is and with its k longest pairs left out (k = 1, 3,
8, 16), so the bound the remaining pairs set is visible.  GPU only.

    python tools/shard_probe.py [P ...]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))


def time_batch(k, ss, src, dst, inits, reps=10):
    import torch
    b = k.IcpBatch(ss, src, dst, inits, epsilon=0.05, max_iters=100)
    for _ in range(2):
        b.launch()
    torch.cuda.synchronize()
    ts = []
    s = torch.cuda.current_stream()
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        b.launch()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts)), float(np.min(ts)), b.result()


def main():
    import torch
    torch.cuda.set_device(0)
    from slamhip import icp as k
    from slamhip import se2, synthetic
    sizes = [int(x) for x in sys.argv[1:]] or [1250, 2500]
    n = max(sizes)
    seq = synthetic.make_sequence(10001, seed=2025)
    inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, n + 1)])
    ss = k.ScanSet(seq.scans[:n + 1])
    for P in sizes:
        src, dst = np.arange(1, P + 1), np.arange(0, P)
        med, best, res = time_batch(k, ss, src, dst, inits[:P])
        order = np.argsort(-res.iters, kind="stable")
        print(f"P {P}: {med:.3f} ms (best {best:.3f}); longest {res.iters[order[:6]].tolist()} at {order[:6].tolist()}",
              flush=True)
        for drop in (1, 3, 8, 16):
            keep = np.sort(order[drop:])
            med, best, _ = time_batch(k, ss, src[keep], dst[keep], inits[keep])
            print(f"   without the {drop} longest (next {res.iters[order[drop]]} iters): {med:.3f} ms "
                  f"(best {best:.3f})", flush=True)


if __name__ == "__main__":
    main()
