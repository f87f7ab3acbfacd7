"""GN iterations/s at C4 under different node orderings (timing probe):
RCM (default), a folded place-major ring order, and position-major order on
C4 without its 9 lap-wrap odometry edges (a path of places: the band a
band + border ordering leaves)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "icp-slam-with-loop-closure_amd"))
from slamhip import _abi, gn, synthetic  # noqa: E402
from slamhip import device as dv  # noqa: E402


def timeit(guess, ea, eb, tf, order, label, border=None):
    t = dv.torch()
    plan = gn.GnPlan(len(guess), ea, eb, order=order, border=border)
    s = gn.GaussNewton(guess, ea, eb, tf, plan=plan)
    s.run(2)
    best = 1e9
    for _ in range(5):
        s.poses.copy_(dv.to_dev(guess, np.float64, s.poses.device))
        t.cuda.synchronize()
        t0 = time.perf_counter()
        chis = s.run(10)
        best = min(best, time.perf_counter() - t0)
    wb = _abi.lib().slam_gn_bcr_block_rows(plan.nv_band, plan.W)
    print(f"{label:28s} W {plan.W:3d} Wb {wb:3d} border {plan.nv - plan.nv_band:2d} {10 / best:8.1f} it/s "
          f"chi2 {chis[0]:.6g} -> {chis[-1]:.9g}", flush=True)


guess, ea, eb, tf, _ = synthetic.lap_graph_c4()
N = len(guess)
per_lap, laps = 500, 10
import scipy.sparse as sp  # noqa: E402
from scipy.sparse.csgraph import reverse_cuthill_mckee  # noqa: E402
adj = sp.coo_matrix((np.ones(2 * len(ea)), (np.r_[ea, eb], np.r_[eb, ea])), shape=(N, N)).tocsr()
timeit(guess, ea, eb, tf, None, "default plan")
timeit(guess, ea, eb, tf, reverse_cuthill_mckee(adj, symmetric_mode=True), "rcm")
place = np.arange(N) % per_lap
lap = np.arange(N) // per_lap
fold = np.where(place < per_lap // 2, 2 * place, 2 * (per_lap - 1 - place) + 1)
timeit(guess, ea, eb, tf, np.lexsort((lap, fold)), "folded place-major")
keep = ~((np.asarray(eb) == np.asarray(ea) + 1) & (np.asarray(eb) % per_lap == 0))
ea2, eb2, tf2 = np.asarray(ea)[keep], np.asarray(eb)[keep], np.asarray(tf)[keep]
timeit(guess, ea2, eb2, tf2, None, "no-wrap rcm")
timeit(guess, ea2, eb2, tf2, np.lexsort((lap, place)), "no-wrap position-major")
