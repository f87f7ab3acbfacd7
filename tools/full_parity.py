"""Parity of the benchmarked path over EVERY pair of the C3 stream: the GPU's
batched ICP (default scheduler; the full 10k batch and EVERY rank's shard at
2 / 4 / 8 GPUs, contiguous and cost-balanced (slamhip.dist), which run the
angle pre-tier and the exchange / head tiers) against the
CPU oracle (oracle/icp_oracle.py, vectorised NumPy, bit-exact with
src/icp.py), run on the host cores with joblib.  GPU only; ~2 minutes on 16
cores.

Besides equality it records how close every stopping decision of the oracle
run comes to its threshold (src/icp.py:86-94): per iteration k the margins
|err_k - eps| and, from the second iteration, ||err_{k-1} - err_k| - thresh|;
per pair the smallest of them, against the GPU-vs-oracle difference of the
final error.  A margin below ~1e3 x that difference would mark a pair whose
iteration count rides on rounding.

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

EPS, MAX_ITERS, THRESH = 0.05, 100, 1e-4


def oracle_pair(pc1, pc2, init):
    """icp_oracle.icp's loop (src/icp.py:72-97) keeping every iteration's error."""
    import icp_oracle
    a, b = np.c_[pc1, np.ones(len(pc1))], np.c_[pc2, np.ones(len(pc2))]
    T, errs, it = init, [], 0
    while True:
        T, _, err = icp_oracle.icp_iteration(a, b, T)
        errs.append(float(err))
        if err < EPS or it > MAX_ITERS:
            break
        if len(errs) > 1 and abs(errs[-2] - err) < THRESH:
            break
        it += 1
    e = np.array(errs)
    m_eps = np.abs(e - EPS).min()
    m_d = np.abs(np.abs(np.diff(e)) - THRESH).min() if len(e) > 1 else np.inf
    return T, errs[-1], len(errs), float(m_eps), float(m_d)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    workers = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    seq = synthetic.make_sequence(n + 1, seed=2025)
    inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, n + 1)])
    ss = k.ScanSet(seq.scans)
    from slamhip import dist as sd
    idx_all = np.arange(n)
    runs = {"all": (idx_all, k.icp_batch(ss, idx_all + 1, idx_all, inits, epsilon=EPS, max_iters=MAX_ITERS))}
    keys = sd.turn_keys(inits)
    for mode in ("contiguous", "balanced"):   # both shardings bench.py offers
        for nr in (2, 4, 8):   # EVERY rank's shard (the tier profile depends on the shard size)
            shards = sd.balanced_shards(keys, nr) if mode == "balanced" else sd.contiguous_shards(n, nr)
            for r, idx in enumerate(shards):
                runs[f"{mode}_ranks{nr}_rank{r}"] = (idx, k.icp_batch(ss, idx + 1, idx, inits[idx], epsilon=EPS,
                                                                       max_iters=MAX_ITERS))
    from joblib import Parallel, delayed
    t0 = time.perf_counter()
    ref = Parallel(n_jobs=workers, backend="loky", batch_size=16)(
        delayed(oracle_pair)(seq.scans[i + 1], seq.scans[i], inits[i].copy()) for i in range(n))
    dt = time.perf_counter() - t0
    rtf = np.stack([r[0] for r in ref])
    rerr = np.array([r[1] for r in ref])
    rit = np.array([r[2] for r in ref])
    m_eps = np.array([r[3] for r in ref])
    m_d = np.array([r[4] for r in ref])
    out = {"workload": f"C3 stream seed 2025, {n} consecutive pairs of 1081-point scans, scripts/main.py parameters",
           "oracle": "oracle/icp_oracle.py (vectorised, bit-exact with the reference's src/icp.py)",
           "oracle_seconds": round(dt, 1), "oracle_workers": workers, "runs": {}}
    for key, (sl, res) in runs.items():
        cnt = len(res.iters)
        dtf = np.abs(res.tf - rtf[sl]).max(axis=(1, 2))
        derr = np.abs(res.err - rerr[sl]) / np.maximum(1.0, np.abs(rerr[sl]))
        out["runs"][key] = {
            "pairs": cnt, "first_pair": int(sl[0]), "iters_equal": int(np.sum(res.iters == rit[sl])),
            "max_abs_tf_diff": float(dtf.max()), "max_rel_err_diff": float(derr.max()),
            "pairs_over_1e-9": int(np.sum((dtf > 1e-9) | (derr > 1e-9) | (res.iters != rit[sl]))),
            "longest_pair_iters": int(res.iters.max())}
    full = runs["all"][1]
    aerr = np.abs(full.err - rerr)
    margin = np.minimum(m_eps, m_d)
    ratio = margin / np.maximum(aerr, 1e-300)
    worst = np.argsort(ratio)[:5]
    out["stopping_margins"] = {
        "definition": "per pair: min over the oracle's iterations of |err_k - eps| and ||err_{k-1} - err_k| - 1e-4|; "
                      "abs_err_diff = |GPU err - oracle err| of the final iteration (10k run)",
        "min_margin_eps": float(m_eps.min()), "min_margin_delta": float(m_d.min()),
        "min_margin": float(margin.min()), "max_abs_err_diff": float(aerr.max()),
        "min_margin_over_err_diff": float(ratio.min()),
        "pairs_margin_below_1e3x_diff": int(np.sum(margin < 1e3 * aerr)),
        "closest_pairs": [{"pair": int(b), "margin": float(margin[b]), "abs_err_diff": float(aerr[b]),
                           "iters": int(rit[b])} for b in worst]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
