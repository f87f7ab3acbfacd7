"""The literal drop-in fan-out: scripts/main.py:240-247 runs the build's
``src.icp.icp`` under ``joblib.Parallel(backend="loky")`` unchanged, one
process per worker (each opens its own HIP context and reuses its pinned
staging buffers across calls).  64 consecutive pairs of the C3 stream (seed
2025, pairs 1100-1163: the 102-iteration pair 1118 included) with main.py's
parameters, n_jobs=4: iteration counts equal to the CPU oracle's, transforms
within 1e-9, errors within 1e-9 relative — and the same bits as one batched
launch of the same pairs (order-free sums)."""
import os

import numpy as np
import pytest

from conftest import PKG, REPO, homog

pytestmark = pytest.mark.gpu
TOL = 1e-9


def test_loky_fanout_of_the_dropin_icp():
    from joblib import Parallel, delayed
    import icp_oracle
    import src.icp as icp
    from slamhip import se2, synthetic
    seq = synthetic.make_sequence(10001, seed=2025)
    idx = range(1101, 1165)    # pair b = (scan b+1, scan b) for b in 1100..1163
    pc1 = [homog(seq.scans[i]) for i in idx]
    pc2 = [homog(seq.scans[i - 1]) for i in idx]
    inits = [se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in idx]
    # the workers import src.icp by name, as main.py's do: the drop-in package on their path
    # (and the oracle's directory for the CPU reference run below)
    old = os.environ.get("PYTHONPATH")
    os.environ["PYTHONPATH"] = os.pathsep.join([PKG, os.path.join(REPO, "oracle")] + ([old] if old else []))
    try:
        parallel = Parallel(n_jobs=4, verbose=0, backend="loky")
        tfs, errs = zip(*parallel(delayed(icp.icp)(a, b, init_transform=T.copy(), max_iters=100, epsilon=0.05)
                                  for a, b, T in zip(pc1, pc2, inits)))
        ref = Parallel(n_jobs=8, backend="loky")(delayed(icp_oracle.icp)(a, b, T.copy(), 0.05, 100)
                                                 for a, b, T in zip(pc1, pc2, inits))
    finally:
        if old is None:
            os.environ.pop("PYTHONPATH", None)
        else:
            os.environ["PYTHONPATH"] = old
    # (the loky pool is left to joblib: its workers exit when idle)
    last = np.stack([t[-1] for t in tfs])
    iters = np.array([len(t) - 1 for t in tfs])
    assert iters.max() >= 100   # pair 1118
    b_tf, b_err, b_it = icp.icp_batch(pc1, pc2, inits, epsilon=0.05, max_iters=100)
    assert np.array_equal(b_it, iters)
    assert np.array_equal(b_tf, last) and np.array_equal(b_err, np.array(errs))
    for k, (h, e) in enumerate(ref):
        assert iters[k] == len(h) - 1, k
        assert np.abs(last[k] - h[-1]).max() <= TOL, k
        assert abs(errs[k] - e) <= TOL * max(1.0, e), k
        assert all(np.abs(tfs[k][j] - h[j]).max() <= TOL for j in range(len(h))), k
