"""Per-phase timing of workgroup 0 of the batched ICP kernel (s_memtime). GPU only."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
import torch  # noqa: E402
from slamhip import _abi, se2, synthetic  # noqa: E402
from slamhip import icp as k  # noqa: E402

pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
seq = synthetic.make_sequence(pairs + 1, seed=2025)
inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, pairs + 1)])
ss = k.ScanSet(seq.scans)
batch = k.IcpBatch(ss, np.arange(1, pairs + 1), np.arange(0, pairs), inits, epsilon=0.05, max_iters=100)
_abi.lib().slam_icp_set_screen(int(os.environ.get("SLAMHIP_SCREEN", "2")))
batch.launch()
buf = torch.zeros(160, dtype=torch.int64, device="cuda")
_abi.lib().slam_icp_set_stamps(buf.data_ptr())
batch.launch()
torch.cuda.synchronize()
_abi.lib().slam_icp_set_stamps(None)
r = batch.result()
t = buf.cpu().numpy().astype(float)
its = r.iters[0]
names = ["transform+fp32 scan", "certify+rescan", "fallback+sync", "reductions+kabsch"]
print("pair 0 iterations", its)
for n, v in zip(names, t[:4]):
    print(f"{n:22s} {v / its:10.1f} ticks/iter ({v / max(t[:4].sum(), 1) * 100:5.1f} %)")
nch = (int(ss.lens[0]) + 31) // 32
qpt = int(os.environ.get("QPT", "5"))
print(f"extra sub-chunks visited per query group per iteration (wave 0): {t[4] / its / qpt:.2f} of {nch * 4}")

for n, v in zip(["  window scan", "  group box+mask", "  visits"], t[5:8]):
    print(f"{n:22s} {v / its:10.1f} ticks/iter")
print(f"live sub-chunks per group per iteration: {t[8] / its / qpt:.2f}; test batches per group: {t[9] / its / qpt:.2f}")

# wall time of the same launch without stamps, per iteration of pair 0
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
batch.launch()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1)
print(f"launch {ms:.3f} ms for {pairs} pairs (max iters {int(r.iters.max())}); pair 0: {its} iterations; "
      f"stamp total {t[:4].sum() / its:.0f} ticks/iter; wall/iter of the longest pair {ms * 1e3 / r.iters.max():.1f} us")
