"""Config C2 stand-in (BASELINE.json configs[1]): sequential ICP odometry over a
full 1,000-scan synthetic sequence (scripts/main.py:236-256) on one MI355X,
pose match against the CPU reference flow (oracle ICP per pair + the serial
chain, joblib over the host cores).  GPU only.  Prints one JSON line.

    python tools/c2_sequence.py [n_scans] [workers]
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "icp-slam-with-loop-closure_amd"), os.path.join(REPO, "oracle")]


def cpu_pair(pc1, pc2, init):
    import icp_oracle
    h, _ = icp_oracle.icp(np.c_[pc1, np.ones(len(pc1))], np.c_[pc2, np.ones(len(pc2))], init, 0.05, 100)
    return h[-1]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    workers = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    import torch
    from joblib import Parallel, delayed
    from slamhip import pipeline, se2, synthetic
    seq = synthetic.make_sequence(n, seed=1)
    pipeline.scan_matching(seq.odometry[:3], seq.scans[:3])          # warm-up (library load, first launch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = pipeline.scan_matching(seq.odometry, seq.scans)
    t_gpu = time.perf_counter() - t0
    os.environ.update({"OMP_NUM_THREADS": "1", "OPENBLAS_NUM_THREADS": "1"})
    t0 = time.perf_counter()
    tfs = Parallel(n_jobs=workers, backend="loky")(
        delayed(cpu_pair)(seq.scans[i], seq.scans[i - 1], se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]))
        for i in range(1, n))
    t_cpu = time.perf_counter() - t0
    ref = se2.compose_chain(seq.odometry[0], np.stack(tfs))
    d = np.abs(r.poses - ref)
    out = {"config": "C2 stand-in: synthetic 1,000-scan sequence (seed 1), scripts/main.py stage 1",
           "scans": n, "gpu_s_end_to_end": round(t_gpu, 4),
           "gpu_note": "one batched launch + host chain, incl. host->device copy of the scans",
           "cpu_s": round(t_cpu, 2), "cpu_workers": workers,
           "cpu_note": "oracle/icp_oracle.py (vectorised NumPy, bit-exact with the reference) per pair, joblib loky",
           "max_abs_pose_diff": float(d.max()), "max_abs_xy_diff": float(d[:, :2].max()),
           "tolerance": 1e-5, "pass": bool(d.max() <= 1e-5),
           "mean_icp_iters": float(np.mean(r.iters))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
