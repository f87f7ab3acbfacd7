"""The unchanged scripts/main.py:240-247 fan-out of the drop-in src.icp.icp
over joblib loky workers, against one batched launch:
1,000 consecutive pairs of the C3 stream (seed 2025, pairs 0-999), main.py's
parameters.  Per n_jobs: wall time of the 1,000 calls (pool already warm),
the device memory every worker's HIP context and staging buffers take
(torch.cuda.mem_get_info of the device before the pool and while the warm
workers are alive, / n_jobs), and bit-identity with the batched results.
GPU only; at most 12 workers (the GPU box allows 16 processes on the card).

    python tools/loky_fanout.py [n_jobs ...]     (default 1 4 8 12)
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "icp-slam-with-loop-closure_amd")
sys.path.insert(0, PKG)


def main():
    import torch
    from joblib import Parallel, delayed
    torch.cuda.set_device(0)
    import src.icp as icp
    from slamhip import se2, synthetic
    jobs = [int(x) for x in sys.argv[1:]] or [1, 4, 8, 12]
    n = 1000
    seq = synthetic.make_sequence(10001, seed=2025)
    pc = [np.c_[s, np.ones(len(s))] for s in seq.scans[:n + 1]]
    inits = [se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, n + 1)]
    out = {"pairs": n, "workload": "C3 stream seed 2025, pairs 0-999, eps 0.05, max_iters 100"}
    icp.icp_batch(pc[1:], pc[:-1], inits, epsilon=0.05, max_iters=100)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    b_tf, b_err, b_it = icp.icp_batch(pc[1:], pc[:-1], inits, epsilon=0.05, max_iters=100)
    out["icp_batch_s"] = round(time.perf_counter() - t0, 4)
    out["mean_iterations"] = float(np.mean(b_it))
    os.environ["PYTHONPATH"] = PKG + (os.pathsep + os.environ["PYTHONPATH"] if os.environ.get("PYTHONPATH") else "")
    runs = []
    for nj in jobs:
        free0, total = torch.cuda.mem_get_info()
        if nj == 1:
            par = None
            icp.icp(pc[1], pc[0], init_transform=inits[0].copy(), max_iters=100, epsilon=0.05)
        else:
            par = Parallel(n_jobs=nj, verbose=0, backend="loky")
            # warm every worker (HIP context, pinned staging buffers)
            par(delayed(icp.icp)(pc[i + 1], pc[i], init_transform=inits[i].copy(), max_iters=100, epsilon=0.05)
                for i in range(4 * nj))
        free1, _ = torch.cuda.mem_get_info()
        t0 = time.perf_counter()
        if par is None:
            res = [icp.icp(pc[i + 1], pc[i], init_transform=inits[i].copy(), max_iters=100, epsilon=0.05)
                   for i in range(n)]
        else:
            res = par(delayed(icp.icp)(pc[i + 1], pc[i], init_transform=inits[i].copy(), max_iters=100, epsilon=0.05)
                      for i in range(n))
        dt = time.perf_counter() - t0
        tf = np.stack([r[0][-1] for r in res])
        it = np.array([len(r[0]) - 1 for r in res])
        err = np.array([r[1] for r in res])
        same = bool(np.array_equal(tf, b_tf) and np.array_equal(it, b_it) and np.array_equal(err, b_err))
        runs.append({"n_jobs": nj, "wall_s": round(dt, 3), "pairs_per_s": round(n / dt, 1),
                     "vs_icp_batch": round(dt / out["icp_batch_s"], 1),
                     "device_mem_per_worker_MiB": round((free0 - free1) / max(nj, 1) / 2**20, 1) if nj > 1 else None,
                     "bit_identical_to_icp_batch": same})
        print(json.dumps(runs[-1]), flush=True)
        if par is not None:
            from joblib.externals.loky import get_reusable_executor
            get_reusable_executor().shutdown(wait=True)
            time.sleep(2)
    out["fanout"] = runs
    out["device_total_GiB"] = round(total / 2**30, 1)
    out["host"] = {"os_cpu_count": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
