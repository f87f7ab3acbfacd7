"""Per-phase timing of the BCR odd-block kernel (workgroup (0, 1) of every
level, s_memtime ticks summed over levels).  GPU only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
import torch  # noqa: E402
from slamhip import _abi, gn, synthetic  # noqa: E402

guess, ea, eb, tf, _ = synthetic.lap_graph_c4()
g = gn.GaussNewton(guess, ea, eb, tf)
buf = torch.zeros(8, dtype=torch.int64, device="cuda")
g.run(1, graph=False)
_abi.lib().slam_gn_set_stamps(buf.data_ptr())
g.run(1, graph=False)
torch.cuda.synchronize()
_abi.lib().slam_gn_set_stamps(None)
t = buf.cpu().numpy().astype(float)
for n, v in zip(["load", "elimination", "(unused)", "store"], t[:4]):
    print(f"odd {n:10s} {v:12.0f} ticks over all levels ({v / 2.4e3:8.1f} us at 2.4 GHz)")
