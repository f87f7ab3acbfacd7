"""Where a lone pair's pruned search goes, per query-group iteration (diagnostics
build, workgroup 0): group iterations with active queries, their live and
visited sub-chunks, by the number of active lanes.  Pairs of the 10k C3 stream.

    python tools/group_hist.py [--inst=BxQ] [pair ...]
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
import torch  # noqa: E402
from slamhip import _abi, se2, synthetic  # noqa: E402
from slamhip import icp as k  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
inst = next((a.split("=")[1] for a in sys.argv[1:] if a.startswith("--inst=")), "512x3")
pairs = [int(a) for a in args] or [1118, 1018, 236, 0]
seq = synthetic.make_sequence(10001, seed=2025)
lib = _abi.lib()
ss = k.ScanSet(seq.scans[:max(pairs) + 2])
for i in range(lib.slam_icp_num_instances()):
    b, q = ctypes.c_int32(), ctypes.c_int32()
    lib.slam_icp_instance_shape(i, ctypes.byref(b), ctypes.byref(q))
    if f"{b.value}x{q.value}" == inst:
        lib.slam_icp_force_instance(i)
names = ["1", "2-4", "5-8", "9-16", "17-32", "33-64"]
for p in pairs:
    init = se2.pose_to_mat(seq.odometry[p + 1] - seq.odometry[p])[None]
    buf = torch.zeros(160, dtype=torch.int64, device="cuda")
    lib.slam_icp_set_stamps(buf.data_ptr())
    batch = k.IcpBatch(ss, [p + 1], [p], init, epsilon=0.05, max_iters=100)
    batch.launch()
    torch.cuda.synchronize()
    lib.slam_icp_set_stamps(None)
    its = int(batch.result().iters[0])
    t = buf.cpu().numpy().astype(float)
    g = t[96:102] / its
    live = t[104:110] / its
    vis = t[112:118] / its
    print(f"pair {p} iters {its} ({inst}) per iteration: group-iters {g.sum():.1f}, live {live.sum():.1f}, "
          f"visited {vis.sum():.1f}; wave-0 cycles scan {t[0] / its:.0f} cert {t[1] / its:.0f} red {t[3] / its:.0f}",
          flush=True)
    for j, nm in enumerate(names):
        print(f"    active {nm:>5}: group-iters {g[j]:5.2f} live {live[j]:6.1f} visited {vis[j]:5.1f}", flush=True)
lib.slam_icp_force_instance(-1)
