"""One-launch scheduling probe on the 10k C3 stream ("a single-phase launch
ordered by the a-priori key, with no pause"): the default two-phase scheduler against one launch
(slam_icp_set_schedule(0, ...)) with the pairs in stream order, ordered by the a-priori turn key
(|dtheta| of the initial transform, descending), and ordered by the true iteration count
(descending; the best any a-priori order could do).  HIP events, median of 7 launches.
GPU only.   python tools/single_phase_probe.py [seed ...]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))


def main():
    import torch
    torch.cuda.set_device(0)
    from slamhip import _abi, se2, synthetic
    from slamhip import dist as sd
    from slamhip import icp as k
    lib = _abi.lib()
    total = int(os.environ.get("SHARD_TOTAL", "10000"))
    for seed in [int(s) for s in sys.argv[1:]] or [2025, 7]:
        seq = synthetic.make_sequence(total + 1, seed=seed)
        inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, total + 1)])
        ss = k.ScanSet(seq.scans)
        idx = np.arange(total)
        base = k.IcpBatch(ss, idx + 1, idx, inits, epsilon=0.05, max_iters=100)

        def timed(b, reps=7):
            b.launch()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                b.launch()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            return float(np.median(ts)), float(np.min(ts))

        lib.slam_icp_set_schedule_auto(1)
        lib.slam_icp_set_schedule(-1, 1024)
        t_def = timed(base)
        ref = base.result()
        orders = {"stream": idx,
                  "turn_key": np.argsort(-sd.turn_keys(inits), kind="stable"),
                  "true_iters": np.argsort(-ref.iters, kind="stable")}
        line = [f"seed {seed}: two-phase (default) {t_def[0]:.3f} ms (min {t_def[1]:.3f})"]
        assert lib.slam_icp_set_schedule(0, 1024) == 0
        for name, o in orders.items():
            b = k.IcpBatch(ss, o + 1, o, inits[o], epsilon=0.05, max_iters=100)
            t = timed(b)
            r = b.result()
            same = np.array_equal(r.iters, ref.iters[o]) and np.array_equal(r.tf, ref.tf[o])
            line.append(f"one launch, {name} order {t[0]:.3f} ms (min {t[1]:.3f}){'' if same else ' MISMATCH'}")
        lib.slam_icp_set_schedule(-1, 1024)
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
