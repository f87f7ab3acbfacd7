"""A/B of the phase-1 probe length on the 10k C3 batch, timed the way bench.py times it (K
back-to-back launches between two events, no sync between them), alternating settings on one
box.   python tools/ab_probe.py [probe ...]  (default 3 2)
Environment: AB_SHARD "N:r" times rank r's balanced shard of N ranks instead of the whole batch;
AB_KNOB=drain: the values are drain-tier settings (slam_icp_set_drain) instead of probe lengths;
AB_KNOB=wide: the values are phase-2 wide heads (0: the automatic profile; n: n slowest-keyed pairs
on wide workgroups of two query groups, every tier limit lifted)."""
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
    probes = [int(x) for x in sys.argv[1:]] or [3, 2]
    for seed in (2025, 7):
        seq = synthetic.make_sequence(10001, seed=seed)
        inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, 10001)])
        ss = k.ScanSet(seq.scans)
        idx = np.arange(10000)
        if os.environ.get("AB_SHARD"):
            from slamhip import dist as sd
            nr, rk = (int(x) for x in os.environ["AB_SHARD"].split(":"))
            idx = sd.balanced_shards(sd.turn_keys(inits), nr)[rk]
        b = k.IcpBatch(ss, idx + 1, idx, inits[idx], epsilon=0.05, max_iters=100)
        res = {p: [] for p in probes}
        ref = None
        for rep in range(4):
            for p in probes:
                if os.environ.get("AB_KNOB") == "drain":
                    assert lib.slam_icp_set_drain(p) == 0
                elif os.environ.get("AB_KNOB") == "wide":
                    if p == 0:
                        assert lib.slam_icp_set_schedule_auto(1) == 0
                        assert lib.slam_icp_set_tier_limit(0) == 0
                    else:
                        assert lib.slam_icp_set_wide_groups(2) == 0
                        assert lib.slam_icp_set_schedule_heads(p) == 0
                        assert lib.slam_icp_set_schedule_gangs(0, 4) == 0
                        assert lib.slam_icp_set_schedule_wide(p, 1) == 0
                        assert lib.slam_icp_set_angle_tier(0, 0.3) == 0
                        assert lib.slam_icp_set_tier_limit(100000) == 0
                else:
                    assert lib.slam_icp_set_schedule(p, 1024) == 0
                for _ in range(2):
                    b.launch()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    b.launch()
                e1.record()
                e1.synchronize()
                res[p].append(e0.elapsed_time(e1) / 20)
                r = b.result()
                if ref is None:
                    ref = r
                assert np.array_equal(r.iters, ref.iters) and np.array_equal(r.tf, ref.tf)
        lib.slam_icp_set_schedule(-1, 1024)
        lib.slam_icp_set_drain(-1)
        lib.slam_icp_set_tier_limit(0)
        lib.slam_icp_set_wide_groups(1)
        lib.slam_icp_set_schedule_auto(1)
        print(f"seed {seed} pairs {len(idx)}: " + " | ".join(f"{os.environ.get('AB_KNOB', 'probe')} {p}: " + " ".join(f"{t:.3f}" for t in res[p]) +
                                            f" (median {np.median(res[p]):.3f} ms)" for p in probes), flush=True)


if __name__ == "__main__":
    main()
