"""Strong-scaling projection on ONE GPU, done the way bench.py shards: every
rank's shard of ONE C3 stream over N ranks (N = 2, 4, 8) timed on its own
(HIP events, median of 5 launches), under each scheduler setting
"heads,gangs,parts,wide,share[,probe[,sort_one[,tier_limit[,xcd_map[,angle_max[,angle_centirad[,angle_kind[,mix,mix_share]]]]]]]]"
or "auto" (the library's automatic tier profile; "auto:P" with a phase-1 probe of P iterations).  The projected N-GPU time
is the slowest shard (bench.py takes the max over ranks).
(bench.py --pairs P builds ANOTHER stream of P pairs: synthetic.make_sequence
draws its noise after the whole trajectory, so a shorter stream is not a
prefix of the 10k one.)  GPU only.

    python tools/shard_sweep.py [setting ... | auto]

Environment: SHARD_TOTAL (10000 pairs), SHARD_N (2,4,8), SHARD_SEED (2025:
the C3 stream), SHARD_DROPOUT (0: 1081-point scans; 0.35: ragged 700-1081),
SHARD_MODE (contiguous | balanced | both: slamhip.dist.contiguous_shards /
balanced_shards), SHARD_WIDE_GROUPS (query groups per wide-tier workgroup),
SHARD_DRAIN (drain tier pairs: -1 the default, 0 off), SHARD_TIMING (b2b: 20 back-to-back launches
per shard as bench.py times them, instead of the median of single launches, which also counts
the host's enqueue of the scheduler's launches).
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
    from slamhip import dist as sd
    from slamhip import icp as k
    lib = _abi.lib()
    settings = sys.argv[1:] or ["auto"]
    if os.environ.get("SHARD_DRAIN"):   # drain tier pairs (-1 default, 0 off)
        assert lib.slam_icp_set_drain(int(os.environ["SHARD_DRAIN"])) == 0
    if os.environ.get("SHARD_WIDE_GROUPS"):   # query groups per wide-tier workgroup (1 or 2)
        assert lib.slam_icp_set_wide_groups(int(os.environ["SHARD_WIDE_GROUPS"])) == 0
    total = int(os.environ.get("SHARD_TOTAL", "10000"))
    seed = int(os.environ.get("SHARD_SEED", "2025"))
    dropout = float(os.environ.get("SHARD_DROPOUT", "0"))
    modes = {"both": ["contiguous", "balanced"]}.get(os.environ.get("SHARD_MODE", "both"),
                                                     [os.environ.get("SHARD_MODE", "both")])
    seq = synthetic.make_sequence(total + 1, seed=seed, dropout=dropout)
    lens = np.array([len(s) for s in seq.scans])
    print(f"stream seed {seed} dropout {dropout}: {total} pairs, scans of {lens.min()}-{lens.max()} points", flush=True)
    inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, total + 1)])
    keys = sd.turn_keys(inits)
    ss = k.ScanSet(seq.scans)
    ranks = [int(x) for x in os.environ.get("SHARD_N", "2,4,8").split(",")]
    batches = {}
    for mode in modes:
        for n in [1] + ranks:
            shards = sd.balanced_shards(keys, n) if mode == "balanced" else sd.contiguous_shards(total, n)
            for r, idx in enumerate(shards):
                batches[(mode, n, r)] = (idx, k.IcpBatch(ss, idx + 1, idx, inits[idx], epsilon=0.05, max_iters=100))
    ref = {}
    full = {}

    b2b = os.environ.get("SHARD_TIMING") == "b2b"

    def timed(b, reps=5):
        b.launch()
        torch.cuda.synchronize()
        if b2b:   # as bench.py times: 20 back-to-back launches between two events, per launch
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b.launch()
            e0.record()
            for _ in range(20):
                b.launch()
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1) / 20
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            b.launch()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts))
    try:
        for st in settings:
            if st.startswith("auto"):   # the library's automatic tier profile by batch size ("auto:P": phase-1 probe P)
                assert lib.slam_icp_set_schedule_auto(1) == 0
                v = [0, 0, 4, 0, 1] + ([int(st[5:])] if st.startswith("auto:") else [])
            else:
                v = [int(x) for x in st.split(",")]
            h, g, gp, w, ws = v[:5]
            if not st.startswith("auto"):
                assert lib.slam_icp_set_schedule_heads(h) == 0
                assert lib.slam_icp_set_schedule_gangs(g, gp) == 0
                assert lib.slam_icp_set_schedule_wide(w, ws) == 0
            assert lib.slam_icp_set_schedule(v[5] if len(v) > 5 else -1, 1024) == 0
            assert lib.slam_icp_set_sched_sort_one(v[6] if len(v) > 6 else 1) == 0
            assert lib.slam_icp_set_tier_limit(v[7] if len(v) > 7 else 0) == 0
            assert lib.slam_icp_set_xcd_map(v[8] if len(v) > 8 else -1) == 0
            if not st.startswith("auto"):
                assert lib.slam_icp_set_angle_tier(v[9] if len(v) > 9 else 0, (v[10] if len(v) > 10 else 30) / 100.0) == 0
                assert lib.slam_icp_set_angle_tier_kind(v[11] if len(v) > 11 else 0) == 0
                assert lib.slam_icp_set_angle_tier_mix(v[12] if len(v) > 12 else 0, v[13] if len(v) > 13 else 2) == 0
            for mode in modes:
                line = []
                t1 = None
                lib.slam_icp_gang_timeouts()   # clear
                for n in [1] + ranks:
                    ts = []
                    for r in range(n):
                        idx, b = batches[(mode, n, r)]
                        ts.append(timed(b, 3 if n == 1 else 5))
                        res = b.result()
                        if n == 1:
                            full.setdefault("tf", res.tf)
                            full.setdefault("iters", res.iters)
                        # every shard bit-identical to the full batch's rows
                        if not (np.array_equal(res.tf, full["tf"][idx]) and np.array_equal(res.iters, full["iters"][idx])):
                            line.append(f"MISMATCH n{n}r{r}")
                        key = (mode, n, r)
                        if key not in ref:
                            ref[key] = res
                    mx = max(ts)
                    if n == 1:
                        t1 = mx
                    its = [int(full["iters"][batches[(mode, n, r)][0]].max()) for r in range(n)]
                    line.append(f"N{n}: max {mx:.3f} ({t1 / mx:.2f}x) shards " + " ".join(f"{t:.3f}" for t in ts) +
                                (f" longest {its}" if n > 1 else ""))
                tmo = lib.slam_icp_gang_timeouts()
                print(f"{mode:10s} {st:16s} | " + " | ".join(line) + f" | timeouts {tmo}", flush=True)
    finally:
        lib.slam_icp_set_schedule_auto(1)
        lib.slam_icp_set_schedule(-1, 1024)
        lib.slam_icp_set_sched_sort_one(1)
        lib.slam_icp_set_tier_limit(0)
        lib.slam_icp_set_xcd_map(-1)
        lib.slam_icp_set_angle_tier(0, 0.3)
        lib.slam_icp_set_schedule_auto(1)


if __name__ == "__main__":
    main()
