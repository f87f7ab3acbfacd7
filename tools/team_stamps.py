"""Where a lone team-run (or, with --wide, wide-tier) pair's iteration goes:
per query group (workgroup), wave 0's s_memtime cycles per phase and
iteration.  Pairs of the 10k C3 stream.  GPU only.
    python tools/team_stamps.py [--wide | --wide2] [pair ...]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
import torch  # noqa: E402
from slamhip import _abi, se2, synthetic  # noqa: E402
from slamhip import icp as k  # noqa: E402

wide = "--wide" in sys.argv or "--wide2" in sys.argv
groups = 2 if "--wide2" in sys.argv else 1   # --wide2: two query groups per 16-wave workgroup
pairs = [int(a) for a in sys.argv[1:] if not a.startswith("--")] or [1118, 236]
seq = synthetic.make_sequence(10001, seed=2025)
lib = _abi.lib()
ss = k.ScanSet(seq.scans[:max(pairs) + 2])
names = (["scan", "bar1", "merge", "certify", "sums", "exchange", "kabsch", "bar2", "-", "-"] if wide else
         ["window", "merge1", "clear", "group", "bar2", "merge2", "certify", "sums", "exchange", "kabsch"])
try:
    lib.slam_icp_set_schedule(4, 1)
    lib.slam_icp_set_schedule_heads(64)
    if wide:
        lib.slam_icp_set_schedule_gangs(0, 4)
        lib.slam_icp_set_schedule_wide(1, 1)
        lib.slam_icp_set_wide_groups(groups)
    else:
        lib.slam_icp_set_schedule_gangs(1, 0)
    for p in pairs:
        init = se2.pose_to_mat(seq.odometry[p + 1] - seq.odometry[p])[None]
        batch = k.IcpBatch(ss, [p + 1], [p], init, epsilon=0.05, max_iters=100)
        batch.launch()
        torch.cuda.synchronize()
        buf = torch.zeros(256 + 16 * 64, dtype=torch.int64, device="cuda")
        lib.slam_icp_set_stamps(buf.data_ptr())
        batch.launch()
        torch.cuda.synchronize()
        lib.slam_icp_set_stamps(None)
        its = int(batch.result().iters[0]) - 4
        t = buf.cpu().numpy()[256:].reshape(64, 16)[:, :10].astype(float) / max(its, 1)
        parts = int((t.sum(1) > 0).sum())
        print(f"pair {p}: {its} {'wide' if wide else 'team'} iterations, {parts} groups; cycles per iteration (wave 0 of each group):", flush=True)
        print("   group " + " ".join(f"{n:>8}" for n in names) + "    total", flush=True)
        for g in range(parts):
            print(f"   {g:5d} " + " ".join(f"{v:8.0f}" for v in t[g]) + f" {t[g].sum():8.0f}", flush=True)
finally:
    lib.slam_icp_set_schedule(-1, 1024)
    lib.slam_icp_set_schedule_gangs(24, 4)
    lib.slam_icp_set_schedule_wide(0, 1)
    lib.slam_icp_set_wide_groups(1)
    lib.slam_icp_set_schedule_auto(1)
