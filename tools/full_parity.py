"""Parity of the benchmarked path over EVERY pair of the C3 stream: the GPU's
batched ICP (default scheduler; the full 10k batch and the shards ranks 0 get
at 2 / 4 / 8 GPUs, which run the CU-exclusive head pairs) against the CPU
oracle (oracle/icp_oracle.py, vectorised NumPy, bit-exact with src/icp.py),
run on the host cores with joblib.  GPU only; ~2 minutes on 16 cores.

    python tools/full_parity.py [pairs] [workers] > profiles/rNN_full_parity.json
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
os.environ.setdefault("OMP_NUM_THREADS", "1")
from slamhip import se2, synthetic  # noqa: E402
from slamhip import icp as k  # noqa: E402


def oracle_pair(pc1, pc2, init):
    import icp_oracle
    h, e = icp_oracle.icp(np.c_[pc1, np.ones(len(pc1))], np.c_[pc2, np.ones(len(pc2))], init, 0.05, 100)
    return h[-1], float(e), len(h) - 1


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    workers = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    seq = synthetic.make_sequence(n + 1, seed=2025)
    inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, n + 1)])
    ss = k.ScanSet(seq.scans)
    runs = {}
    for shard in (n, n // 2, n // 4, n // 8):
        res = k.icp_batch(ss, np.arange(1, shard + 1), np.arange(0, shard), inits[:shard], epsilon=0.05, max_iters=100)
        runs[shard] = res
    from joblib import Parallel, delayed
    t0 = time.perf_counter()
    ref = Parallel(n_jobs=workers, backend="loky", batch_size=16)(
        delayed(oracle_pair)(seq.scans[i + 1], seq.scans[i], inits[i].copy()) for i in range(n))
    dt = time.perf_counter() - t0
    rtf = np.stack([r[0] for r in ref])
    rerr = np.array([r[1] for r in ref])
    rit = np.array([r[2] for r in ref])
    out = {"workload": f"C3 stream seed 2025, {n} consecutive pairs of 1081-point scans, scripts/main.py parameters",
           "oracle": "oracle/icp_oracle.py (vectorised, bit-exact with the reference's src/icp.py)",
           "oracle_seconds": round(dt, 1), "oracle_workers": workers, "runs": {}}
    for shard, res in runs.items():
        dtf = np.abs(res.tf - rtf[:shard]).max(axis=(1, 2))
        derr = np.abs(res.err - rerr[:shard]) / np.maximum(1.0, np.abs(rerr[:shard]))
        out["runs"][f"first_{shard}_pairs"] = {
            "pairs": shard, "iters_equal": int(np.sum(res.iters == rit[:shard])),
            "max_abs_tf_diff": float(dtf.max()), "max_rel_err_diff": float(derr.max()),
            "pairs_over_1e-9": int(np.sum((dtf > 1e-9) | (derr > 1e-9) | (res.iters != rit[:shard]))),
            "longest_pair_iters": int(res.iters.max())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
