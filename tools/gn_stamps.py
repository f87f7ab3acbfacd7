"""Per-phase timing of the GN band-Cholesky kernel (s_memtime stamps). GPU only."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
import torch  # noqa: E402
from slamhip import _abi, gn, synthetic  # noqa: E402

guess, ea, eb, tf, _ = synthetic.lap_graph_c4()
g = gn.GaussNewton(guess, ea, eb, tf)
buf = torch.zeros(5, dtype=torch.int64, device="cuda")
g.run(1)
_abi.lib().slam_gn_set_stamps(buf.data_ptr())
g.run(1)
torch.cuda.synchronize()
_abi.lib().slam_gn_set_stamps(None)
t = buf.cpu().numpy().astype(float)
steps = (g.plan.nv + 15) // 16
names = ["prologue", "b:panel+sync", "c:lookahead(a)+update+enter+sync", "-", "-"]
print("W", g.plan.W, "steps", steps)
for n, v in zip(names, t):
    print(f"{n:16s} {v / steps:10.1f} ticks/step  ({v / t.sum() * 100:5.1f} %)")
