"""Per-pair timeline of one batched ICP launch (slam_icp_set_trace): for a
shard of the C3 stream (the 10k stream bench.py shards), when each pair's
workgroup started and ended in each scheduler phase, where (XCC / CU), and
what bounds the makespan.  GPU only.

    python tools/timeline.py [N:rank ...]     (default 8:0 4:0; a bare P: the first P pairs;
                                              bN:rank: rank's shard of slamhip.dist.balanced_shards)
Environment: SHARD_SEED (2025).
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
    from slamhip import dist as sd
    specs = sys.argv[1:] or ["8:0", "4:0"]
    seq = synthetic.make_sequence(10001, seed=int(os.environ.get("SHARD_SEED", "2025")))
    inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, 10001)])
    ss = k.ScanSet(seq.scans)
    full = k.IcpBatch(ss, np.arange(1, 10001), np.arange(0, 10000), inits, epsilon=0.05, max_iters=100)
    full.launch()
    it_all = full.result().iters
    np.save(os.path.join(REPO, "gpurun_out", "iters_10k.npy"), it_all)
    for nr in (2, 4, 8):
        mx = [int(it_all[sd.shard_range(10000, nr, r)[0]:sd.shard_range(10000, nr, r)[1]].max()) for r in range(nr)]
        print(f"N{nr}: longest pair per shard (iterations) {mx}", flush=True)
    keys = sd.turn_keys(inits)
    for spec in specs:
        if spec.startswith("b"):
            nr, r = (int(x) for x in spec[1:].split(":"))
            idx = sd.balanced_shards(keys, nr)[r]
        elif ":" in spec:
            nr, r = (int(x) for x in spec.split(":"))
            lo, hi, _ = sd.shard_range(10000, nr, r)
            idx = np.arange(lo, hi)
        else:
            idx = np.arange(0, int(spec))
        P = len(idx)
        print(f"shard {spec}: {P} pairs", flush=True)
        b = k.IcpBatch(ss, idx + 1, idx, inits[idx], epsilon=0.05, max_iters=100)
        for _ in range(3):
            b.launch()
        torch.cuda.synchronize()
        buf = torch.zeros(P * 8, dtype=torch.int64, device="cuda")
        lib.slam_icp_set_trace(buf.data_ptr())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.launch()
        e1.record()
        torch.cuda.synchronize()
        lib.slam_icp_set_trace(None)
        ms = e0.elapsed_time(e1)
        it = b.result().iters
        turn = keys[idx] > 0.3
        t = buf.cpu().numpy().reshape(P, 2, 4)
        st, en = t[:, :, 0].astype(np.float64), t[:, :, 1].astype(np.float64)
        ran = st > 0
        t0 = st[ran].min()
        us = lambda x: (x - t0) / 100.0   # 100 MHz ticks -> us
        end1 = np.where(ran[:, 0], us(en[:, 0]), np.nan)
        st2 = np.where(ran[:, 1], us(st[:, 1]), np.nan)
        end2 = np.where(ran[:, 1], us(en[:, 1]), np.nan)
        fin = np.where(np.isnan(end2), end1, end2)
        print(f"P {P}: event {ms * 1e3:.0f} us; phase 1 starts {np.nanmin(us(st[:, 0])):.0f}..{np.nanmax(us(st[:, 0])):.0f}"
              f" ends {np.nanmin(end1):.0f}..{np.nanmax(end1):.0f}; phase 2 starts {np.nanmin(st2):.0f}..{np.nanmax(st2):.0f};"
              f" last finish {np.nanmax(fin):.0f} us; pairs in phase 2: {int(ran[:, 1].sum())}", flush=True)
        # staging latency (start -> pc2 staged, constants ready) and per-iteration latency
        for ph in (0, 1):
            ok = ran[:, ph] & (t[:, ph, 3] > 0)
            stg = (t[ok, ph, 3].astype(np.float64) - st[ok, ph]) / 100.0
            print(f"   phase {ph + 1} staging latency us: p50 {np.median(stg):.1f} p90 {np.percentile(stg, 90):.1f}",
                  flush=True)
        # finish-time quantiles and the last finishers
        q = np.nanpercentile(fin, [50, 90, 99, 100])
        print(f"   finish p50 {q[0]:.0f} p90 {q[1]:.0f} p99 {q[2]:.0f} max {q[3]:.0f} us", flush=True)
        last = np.argsort(-np.nan_to_num(fin, nan=-1))[:16]
        for j in last:
            dur = (end2[j] - st2[j]) if not np.isnan(st2[j]) else np.nan
            rem = it[j] - 4
            print(f"   pair {j:5d}{'t' if turn[j] else ' '} iters {it[j]:3d} p1 {us(st[j, 0]):6.0f}-{end1[j]:6.0f} p2 {st2[j]:6.0f}-{end2[j]:6.0f}"
                  f" ({dur / max(rem, 1):5.1f} us/it) xcc {int(t[j, 0, 2]) >> 32}/{int(t[j, 1, 2]) >> 32}",
                  flush=True)
        # how many pairs are running over time (phase 2)
        grid = np.arange(0, np.nanmax(fin) + 50, 50)
        run = [int(np.sum((np.nan_to_num(st2, nan=1e18) <= g) & (np.nan_to_num(end2, nan=-1) > g))) for g in grid]
        print("   phase-2 pairs running every 50 us: " + " ".join(str(r) for r in run), flush=True)
        np.save(os.path.join(REPO, "gpurun_out", f"timeline_{spec.replace(':', '_')}.npy"), t)


if __name__ == "__main__":
    main()
