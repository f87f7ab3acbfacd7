"""Per-shard iteration statistics of a balanced / contiguous 8-rank split of a C3 stream: how many
long pairs each shard holds and whether the angle pre-tier (|dtheta| > 0.3 rad) sees them, plus
each shard's time with the automatic profile (median of 5).  GPU only (iterations from one
full-batch launch).   python tools/shard_stats.py [seed] [ranks]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))


def main():
    import torch
    torch.cuda.set_device(0)
    from slamhip import se2, synthetic
    from slamhip import dist as sd
    from slamhip import icp as k
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    nr = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    seq = synthetic.make_sequence(10001, seed=seed)
    inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, 10001)])
    keys = sd.turn_keys(inits)
    ss = k.ScanSet(seq.scans)
    full = k.IcpBatch(ss, np.arange(1, 10001), np.arange(0, 10000), inits, epsilon=0.05, max_iters=100)
    full.launch()
    it = full.result().iters
    np.savez(os.path.join(REPO, "gpurun_out", f"iters_seed{seed}.npz"), iters=it, inits=inits)
    turn = keys > 0.3
    print(f"seed {seed}: pairs >= 60 iterations {int((it >= 60).sum())} (turning {int((turn & (it >= 60)).sum())}); "
          f"non-turning max {int(it[~turn].max())}, turning iterations p50 {np.median(it[turn]):.0f}", flush=True)
    for mode in ("balanced", "contiguous"):
        shards = sd.balanced_shards(keys, nr) if mode == "balanced" else sd.contiguous_shards(10000, nr)
        for r, idx in enumerate(shards):
            b = k.IcpBatch(ss, idx + 1, idx, inits[idx], epsilon=0.05, max_iters=100)
            b.launch()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                b.launch()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            si, st = it[idx], turn[idx]
            top = np.argsort(-si)[:6]
            print(f"{mode:10s} rank {r}: {np.median(ts):.3f} ms; iterations sum {int(si.sum())}, >=60: {int((si >= 60).sum())}"
                  f" (turning {int((st & (si >= 60)).sum())}); turning pairs {int(st.sum())} with iteration sum"
                  f" {int(si[st].sum())}; longest non-turning {int(si[~st].max())}; top "
                  + " ".join(f"{int(si[j])}{'t' if st[j] else 'n'}" for j in top), flush=True)


if __name__ == "__main__":
    main()
