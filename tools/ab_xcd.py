"""Interleaved A/B of the XCD-aware pair map (slam_icp_set_xcd_map, runs of
XCD_RUNS consecutive pairs per XCD; 0 = identity) on the
10k C3 batch and the N = 8 / 4 shards of the same stream: HIP events, median
of 5 launches per setting per round, 4 rounds.  GPU only."""
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
    seq = synthetic.make_sequence(10001, seed=2025)
    inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, 10001)])
    ss = k.ScanSet(seq.scans)
    cases = {"10k": (0, 10000)}
    for nr, r in ((8, 0), (8, 5), (4, 2)):
        lo, hi, _ = sd.shard_range(10000, nr, r)
        cases[f"{nr}:{r}"] = (lo, hi)
    batches = {n: k.IcpBatch(ss, np.arange(lo + 1, hi + 1), np.arange(lo, hi), inits[lo:hi], epsilon=0.05,
                             max_iters=100) for n, (lo, hi) in cases.items()}
    runs = [int(x) for x in os.environ.get("XCD_RUNS", "16,0,4,64").split(",")]
    res = {(n, m): [] for n in cases for m in runs}
    ref = {}
    for rnd in range(4):
        for m in runs:
            lib.slam_icp_set_xcd_map(m)
            for n, b in batches.items():
                b.launch()
                torch.cuda.synchronize()
                ts = []
                for _ in range(5):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    b.launch()
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1))
                res[(n, m)].append(float(np.median(ts)))
                r = b.result()
                if n not in ref:
                    ref[n] = r
                assert np.array_equal(r.tf, ref[n].tf) and np.array_equal(r.iters, ref[n].iters), (n, m)
    lib.slam_icp_set_xcd_map(-1)
    for n in cases:
        print(f"{n:6s} " + " | ".join(f"run {m}: " + " ".join(f"{t:.3f}" for t in res[(n, m)]) for m in runs),
              flush=True)


if __name__ == "__main__":
    main()
