"""Latency of ONE C3 pair alone on the GPU run as a gang of K workgroups
(phase 1: 4 iterations on one workgroup, then phase 2 as a gang) against the
one-workgroup head instance and the default instance.  GPU only.

    python tools/gang_lone.py [pair ...]     (pairs of the 10k C3 stream)
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
import torch  # noqa: E402
from slamhip import _abi, se2, synthetic  # noqa: E402
from slamhip import icp as k  # noqa: E402

pairs = [int(a) for a in sys.argv[1:]] or [1118, 1018, 236, 0]
seq = synthetic.make_sequence(10001, seed=2025)
lib = _abi.lib()
ss = k.ScanSet(seq.scans[:max(pairs) + 2])


def timed(batch, reps=7):
    batch.launch()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        batch.launch()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    r = batch.result()
    return float(np.median(ts)) * 1e3, int(r.iters[0]), r


try:
    lib.slam_icp_set_schedule(4, 1)
    for p in pairs:
        init = se2.pose_to_mat(seq.odometry[p + 1] - seq.odometry[p])[None]
        batch = k.IcpBatch(ss, [p + 1], [p], init, epsilon=0.05, max_iters=100)
        line = []
        lib.slam_icp_set_schedule_heads(0)
        us, its, ref = timed(batch)
        line.append(f"default:{us / its:.1f}")
        lib.slam_icp_set_schedule_heads(64)
        lib.slam_icp_set_schedule_gangs(0, 2)
        us, its, _ = timed(batch)
        line.append(f"head512x3:{us / its:.1f}")
        for parts in (4, 0):
            lib.slam_icp_set_schedule_gangs(1, parts)
            us, its2, r = timed(batch)
            assert its2 == its and np.array_equal(r.tf, ref.tf), (p, parts)
            line.append(f"{'team' if parts == 0 else 'gang' + str(parts)}:{us / its:.1f}")
        lib.slam_icp_set_schedule_gangs(0, 4)
        for share in (1, 2, 4):
            lib.slam_icp_set_schedule_wide(1, share)
            us, its2, r = timed(batch)
            assert its2 == its and np.array_equal(r.tf, ref.tf), (p, "wide", share)
            line.append(f"wide/{share}:{us / its:.1f}")
        lib.slam_icp_set_schedule_wide(0, 1)
        print(f"pair {p} iters {its} us/iter (incl. 4 probe iterations on one workgroup) " + " ".join(line), flush=True)
finally:
    lib.slam_icp_set_schedule(-1, 1024)
    lib.slam_icp_set_schedule_heads(64)
    lib.slam_icp_set_schedule_gangs(24, 4)
    lib.slam_icp_set_schedule_wide(0, 1)
