"""Latency of ONE ICP pair alone on the GPU (the strong-scaling tail), per
kernel instance, plus per-phase s_memtime stamps.  GPU only.

    python tools/lone_pair.py [pair ...]      (default: the longest C3 pairs)
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

pairs = [int(a) for a in sys.argv[1:] if not a.startswith("--")] or [1118, 7264, 0]
trunc = next((int(a.split("=")[1]) for a in sys.argv[1:] if a.startswith("--n1=")), 0)   # diagnostics: pc1 prefix
seq = synthetic.make_sequence(max(pairs) + 2, seed=2025)
lib = _abi.lib()
if trunc:
    seq.scans = [s[:trunc] if i - 1 in pairs else s for i, s in enumerate(seq.scans)]
shapes = {}
for i in range(lib.slam_icp_num_instances()):
    b, q = ctypes.c_int32(), ctypes.c_int32()
    lib.slam_icp_instance_shape(i, ctypes.byref(b), ctypes.byref(q))
    if b.value * q.value >= (trunc or 1081):
        shapes[i] = f"{b.value}x{q.value}"
ss = k.ScanSet(seq.scans)
for p in pairs:
    init = se2.pose_to_mat(seq.odometry[p + 1] - seq.odometry[p])[None]
    batch = k.IcpBatch(ss, [p + 1], [p], init, epsilon=0.05, max_iters=100)
    line = []
    for i, name in shapes.items():
        lib.slam_icp_force_instance(i)
        batch.launch()
        torch.cuda.synchronize()
        ts = []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            batch.launch()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        its = int(batch.result().iters[0])
        line.append(f"{name}:{np.median(ts) * 1e3 / its:.1f}")
        if "--stamps-all" in sys.argv:   # per-instance phase stamps (wave 0), cycles per iteration
            sb = torch.zeros(160, dtype=torch.int64, device="cuda")
            lib.slam_icp_set_stamps(sb.data_ptr())
            k.IcpBatch(ss, [p + 1], [p], init, epsilon=0.05, max_iters=100).launch()
            torch.cuda.synchronize()
            lib.slam_icp_set_stamps(None)
            t = sb.cpu().numpy().astype(float) / its
            line[-1] += f"[scan {t[0]:.0f} cert {t[1]:.0f} red {t[3]:.0f} win {t[5]:.0f} clr {t[6]:.0f} vis {t[7]:.0f} b {t[9]:.1f}]"
            if f"--waves={name}" in sys.argv:   # every wave's totals per iteration
                nw = int(name.split("x")[0]) // 64
                w8 = t[16:16 + 8 * nw].reshape(nw, 8)
                print(f"   {name} per wave: " + " | ".join(
                    f"w{w}: scan {r[0]:.0f} cert {r[1]:.0f} red {r[3]:.0f} vis {r[4]:.1f} fail {r[5]:.2f} live {r[6]:.1f} b {r[7]:.1f}"
                    for w, r in enumerate(w8)), flush=True)
    lib.slam_icp_force_instance(-1)
    print(f"pair {p} iters {its} us/iter " + " ".join(line), flush=True)
    buf = torch.zeros(160, dtype=torch.int64, device="cuda")
    lib.slam_icp_set_stamps(buf.data_ptr())
    batch2 = k.IcpBatch(ss, [p + 1], [p], init, epsilon=0.05, max_iters=100)
    batch2.launch()
    torch.cuda.synchronize()
    lib.slam_icp_set_stamps(None)
    t = buf.cpu().numpy().astype(float) / its
    print(f"   stamps/iter (wave 0): scan {t[0]:.0f} certify {t[1]:.0f} fallback {t[2]:.0f} reduce+kabsch {t[3]:.0f} "
          f"| window {t[5]:.0f} mask {t[6]:.0f} visits {t[7]:.0f} | visited sub-chunks/iter {t[4]:.1f} "
          f"live/iter {t[8]:.1f} batches/iter {t[9]:.1f}", flush=True)
    print(f"   group loop/iter: box reductions {t[10]:.0f} group mask {t[11]:.0f} tests+or {t[12]:.0f} scans {t[13]:.0f}",
          flush=True)
