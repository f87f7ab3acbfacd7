"""GPU parity of the HIP ICP path against the reference (golden fixtures) and
the CPU oracle, through the C-ABI (slamhip) and the drop-in ``src.icp``.

Tolerances (north star: poses within 1e-5 of the CPU reference):
  * correspondences: bit-identical (exact fp64 distance, first-min rule);
  * transforms: |dT| <= 1e-9 (closed-form 2x2 Kabsch + tree reductions vs
    LAPACK SVD + NumPy summation order);
  * iteration counts: identical.
"""
import numpy as np
import pytest

from conftest import case_arrays, homog

pytestmark = pytest.mark.gpu
TOL = 1e-9
DEFAULT_ANGLE = (0, 0.3)   # the explicit settings' defaults (slam_icp_set_schedule_auto(1) restores the automatic profile)
DEFAULT_WIDE = (0, 1)
DEFAULT_BULK = (0, 2)


@pytest.fixture(scope="module")
def icp():
    import src.icp as m
    return m


@pytest.fixture(scope="module")
def k():
    from slamhip import icp as kk
    return kk


@pytest.fixture(scope="module")
def oracle():
    import icp_oracle
    return icp_oracle


def test_unit_vectors(golden, icp):
    u = golden("icp_unit.npz")
    for c in range(int(u["n_cases"])):
        pc1, pc2 = u[f"pc1_{c}"], u[f"pc2_{c}"]
        corr = icp.get_correspondences(pc1, pc2)
        assert np.array_equal(corr, u[f"corr_{c}"]), c
        assert np.allclose(icp.get_transform(pc1, pc2[corr]), u[f"tf_{c}"], rtol=0, atol=1e-12)
        e = icp.get_error(pc1, pc2[corr])
        assert abs(e - u[f"err_{c}"]) <= 1e-12 * max(1.0, abs(u[f"err_{c}"]))
        T, c1, e1 = icp.icp_iteration(pc1, pc2, u[f"init_{c}"].copy())
        assert np.array_equal(c1, u[f"it_corr_{c}"])
        assert np.allclose(T, u[f"it_T_{c}"], rtol=0, atol=1e-12)
        assert abs(e1 - u[f"it_err_{c}"]) <= 1e-12 * max(1.0, abs(u[f"it_err_{c}"]))
        assert icp.get_closest_point(pc1[3], pc2) == u[f"corr_{c}"][3]


def test_tie_first_index(golden, icp):
    u = golden("icp_unit.npz")
    pc2 = u["pc2_3"]          # rows 5, 17, 200 are identical
    assert icp.get_closest_point(pc2[17], pc2) == 5
    assert icp.get_closest_point(pc2[200], pc2) == 5


@pytest.mark.parametrize("c", range(12))
def test_icp_golden_cases(golden, icp, c):
    g = golden("icp_cases.npz")
    pc1, pc2, init, eps, mi, st, ro, hist, err = case_arrays(g, c)
    tfs, e = icp.icp(pc1, pc2, init, epsilon=eps, max_iters=mi, stopping_thresh=st, rotation_only=ro)
    assert tfs[0] is init
    assert np.array_equal(init, g["init_after"][c])        # in-place mutation semantics
    assert len(tfs) == len(hist), (len(tfs), len(hist))   # same number of iterations
    assert np.allclose(np.stack(tfs), hist, rtol=0, atol=TOL)
    assert isinstance(e, np.float64)
    assert abs(e - err) <= TOL * max(1.0, abs(err))


def test_first_iteration_correspondences(golden, icp):
    g = golden("icp_cases.npz")
    for c in range(len(g["err"])):
        pc1, pc2, init, *_ , ro = case_arrays(g, c)[:7]
        _, corr, _ = icp.icp_iteration(pc1, pc2, g["init"][c].copy(), rotation_only=ro)
        c0 = g["corr0"][g["corr0_off"][c]:g["corr0_off"][c + 1]]
        assert np.array_equal(corr, c0), c


def _sequence_pairs(n, seed, n_beams=1081):
    from slamhip import se2, synthetic
    seq = synthetic.make_sequence(n + 1, seed=seed, n_beams=n_beams)
    inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, n + 1)])
    return seq, inits


def test_batched_sequence_vs_oracle(k, oracle):
    """scripts/main.py:240-256 on a 48-pair synthetic stream (config C2 shape)."""
    n = 48
    seq, inits = _sequence_pairs(n, seed=1)
    res = k.icp_batch(seq.scans, np.arange(1, n + 1), np.arange(0, n), inits, epsilon=0.05, max_iters=100)
    for b in range(0, n, 6):   # oracle on every 6th pair keeps the test fast
        h, e = oracle.icp(homog(seq.scans[b + 1]), homog(seq.scans[b]), inits[b].copy(), 0.05, 100)
        assert res.iters[b] == len(h) - 1, b
        assert np.allclose(res.tf[b], h[-1], rtol=0, atol=TOL)
        assert abs(res.err[b] - e) <= TOL * max(1.0, e)
    # odometry chain (a8) matches the reference composition
    from slamhip import se2
    chain = se2.compose_chain(seq.odometry[0], res.tf)
    assert chain.shape == (n + 1, 3)
    assert np.abs(chain[:, :2] - seq.truth[:, :2] - (seq.odometry[0, :2] - seq.truth[0, :2])).max() < 0.5


def _oracle_final_tf(pc1, pc2, init):
    import icp_oracle
    h, _ = icp_oracle.icp(homog(pc1), homog(pc2), init, 0.05, 100)
    return h[-1], len(h) - 1


def test_c2_full_sequence_chain_vs_oracle():
    """Config C2 stand-in at full length (BASELINE.json configs[1], SURVEY.md
    §8(d)): the 1,000-scan seed-1 sequence through scripts/main.py stage 1
    (:236-256) — one batched launch on the GPU, the serial chain on the host —
    against the reference flow (oracle ICP per pair on the host cores, the
    same chain): every pair's iteration count equal, every chained pose within
    the north star's 1e-5 (measured: ~1e-13)."""
    import os
    from joblib import Parallel, delayed
    from slamhip import pipeline, se2, synthetic
    n = 1000
    seq = synthetic.make_sequence(n, seed=1)
    r = pipeline.scan_matching(seq.odometry, seq.scans)
    workers = max(1, min(16, len(os.sched_getaffinity(0))))
    ref = Parallel(n_jobs=workers, backend="loky", batch_size=8)(
        delayed(_oracle_final_tf)(seq.scans[i], seq.scans[i - 1], se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]))
        for i in range(1, n))
    assert np.array_equal(r.iters, np.array([it for _, it in ref]))
    chain = se2.compose_chain(seq.odometry[0], np.stack([t for t, _ in ref]))
    assert r.poses.shape == (n, 3)
    assert np.abs(r.poses - chain).max() <= 1e-5
    assert np.abs(r.tf - np.stack([t for t, _ in ref])).max() <= TOL


def test_batch_is_order_independent_and_deterministic(k):
    n = 40
    seq, inits = _sequence_pairs(n, seed=7, n_beams=361)
    src, dst = np.arange(1, n + 1), np.arange(0, n)
    r1 = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=100)
    r2 = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=100)
    assert np.array_equal(r1.tf, r2.tf) and np.array_equal(r1.err, r2.err)
    perm = np.random.default_rng(0).permutation(n)
    r3 = k.icp_batch(seq.scans, src[perm], dst[perm], inits[perm], epsilon=0.05, max_iters=100)
    assert np.array_equal(r3.tf, r1.tf[perm]) and np.array_equal(r3.iters, r1.iters[perm])


def test_every_instance_agrees(k, oracle):
    """All compiled (BLOCK, QPT) shapes that fit the scan give the same answer
    as the oracle — and the same BITS as each other: the per-pair sums are
    order-free (common.hpp rsum_add), so no result depends on the workgroup
    shape / query layout a pair ran on."""
    import ctypes
    from slamhip import _abi
    lib = _abi.lib()
    n = 6
    seq, inits = _sequence_pairs(n, seed=11, n_beams=301)
    ref = [oracle.icp(homog(seq.scans[b + 1]), homog(seq.scans[b]), inits[b].copy(), 0.05, 100)
           for b in range(n)]
    bl, q = ctypes.c_int32(), ctypes.c_int32()
    first = None
    try:
        for i in range(lib.slam_icp_num_instances()):
            lib.slam_icp_instance_shape(i, ctypes.byref(bl), ctypes.byref(q))
            if bl.value * q.value < 301:
                continue
            lib.slam_icp_force_instance(i)
            for mode in (2, 0):
                assert lib.slam_icp_set_screen(mode) == 0
                res = k.icp_batch(seq.scans, np.arange(1, n + 1), np.arange(0, n), inits, epsilon=0.05,
                                  max_iters=100, history=True)
                for b in range(n):
                    assert res.iters[b] == len(ref[b][0]) - 1, (i, b)
                    assert np.allclose(res.tf[b], ref[b][0][-1], rtol=0, atol=TOL), (i, b)
                if first is None:
                    first = res
                    continue
                assert np.array_equal(res.iters, first.iters), (i, mode)
                assert np.array_equal(res.tf, first.tf) and np.array_equal(res.err, first.err), (i, mode)
                for h0, h1 in zip(first.hist, res.hist):
                    assert np.array_equal(h0, h1), (i, mode)
    finally:
        lib.slam_icp_force_instance(-1)
        lib.slam_icp_set_screen(2)


def test_large_ragged_scans_tile_path(k, oracle):
    """pc2 larger than the LDS-resident capacity (4096 points) and a pc1 that
    needs the 512x16 instance: exercises the streamed-tile path."""
    rng = np.random.default_rng(3)
    n2, n1 = 5000, 4500
    pc2 = rng.uniform(-10, 10, size=(n2, 2))
    th = 0.02
    R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
    pc1 = (pc2[rng.choice(n2, n1, replace=False)] - [0.05, 0.02]) @ R.T + rng.normal(0, 0.003, (n1, 2))
    init = np.eye(3)
    res = k.icp_batch([pc1, pc2], [0], [1], init[None], epsilon=1e-9, max_iters=3, stopping_thresh=1e-15)
    h, e = oracle.icp(homog(pc1), homog(pc2), init.copy(), 1e-9, 3, 1e-15)
    assert res.iters[0] == len(h) - 1 == 5
    assert np.allclose(res.tf[0], h[-1], rtol=0, atol=TOL)
    _, corr, _ = k.icp_step([pc1, pc2], [0], [1], np.eye(3)[None])
    assert np.array_equal(corr[0], oracle.correspondences(homog(pc1), homog(pc2)))


def test_exact_recovery_and_identity(k):
    from slamhip import se2
    rng = np.random.default_rng(5)
    pc = rng.uniform(-5, 5, size=(700, 2))
    res = k.icp_batch([pc, pc], [0], [1], np.eye(3)[None], epsilon=1e-30, max_iters=5, history=True)
    assert res.err[0] == 0.0 and np.allclose(res.tf[0], np.eye(3), atol=1e-15)
    T = se2.pose_to_mat([0.01, -0.02, 0.003])
    pc2 = (T[:2, :2] @ pc.T).T + T[:2, 2]
    res = k.icp_batch([pc, pc2], [0], [1], np.eye(3)[None], epsilon=1e-20, max_iters=50, stopping_thresh=0)
    assert np.allclose(res.tf[0], T, atol=1e-12)


def test_bad_inputs_raise(icp):
    pc = np.c_[np.zeros((4, 2)), np.full(4, 2.0)]
    with pytest.raises(ValueError):
        icp.get_correspondences(pc, pc)
    with pytest.raises(ValueError):
        icp.icp(np.zeros((0, 3)), np.ones((3, 3)))


def test_nn_modes_identical(k):
    """Exact fp64 scan, fp32 screen and pruned fp32 screen: bit-identical
    correspondences, hence bit-identical transforms, errors and iterations."""
    from slamhip import _abi
    lib = _abi.lib()
    n = 24
    seq, inits = _sequence_pairs(n, seed=9)
    outs = []
    try:
        for mode in (0, 1, 2):
            assert lib.slam_icp_set_screen(mode) == 0
            outs.append(k.icp_batch(seq.scans, np.arange(1, n + 1), np.arange(0, n), inits, epsilon=0.05,
                                    max_iters=100, history=True))
            _, corr, _ = k.icp_step(seq.scans, np.arange(1, n + 1), np.arange(0, n), inits)
            outs[-1].corr = np.concatenate(corr)
    finally:
        lib.slam_icp_set_screen(2)
    for o in outs[1:]:
        assert np.array_equal(o.corr, outs[0].corr)
        assert np.array_equal(o.iters, outs[0].iters)
        assert np.array_equal(o.tf, outs[0].tf) and np.array_equal(o.err, outs[0].err)
        for h0, h1 in zip(outs[0].hist, o.hist):
            assert np.array_equal(h0, h1)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_small_and_degenerate_scans(k, oracle, mode):
    """Scan sizes around the pruned search's edges (fewer candidates than one
    window / one 32-chunk, n1 != n2), duplicate points (first-index ties),
    collinear clouds and a single-point target: iteration counts, transforms
    and first-iteration correspondences vs the oracle, in every NN mode."""
    from slamhip import _abi
    lib = _abi.lib()
    rng = np.random.default_rng(17)
    cases = []
    # (n1 > 1, n2 = 1) is left out of the transform check: every match is the
    # same point, the centred cross-covariance is rounding noise and the
    # rotation is undefined (its correspondences are checked below)
    for n1, n2 in [(1, 1), (1, 7), (5, 9), (17, 23), (24, 25), (33, 31), (40, 64), (65, 97), (130, 129)]:
        pc2 = rng.uniform(-3, 3, size=(n2, 2))
        pc1 = pc2[rng.integers(0, n2, n1)] + rng.normal(0, 0.05, size=(n1, 2))
        cases.append((pc1, pc2))
    dup = rng.uniform(-2, 2, size=(40, 2))
    dup = np.concatenate([dup, dup[::3], dup[5:9]])              # exact duplicates in pc2
    cases.append((dup[:30] + 0.01, dup))
    line = np.c_[np.linspace(-4, 4, 90), 0.5 * np.linspace(-4, 4, 90)]   # collinear
    cases.append((line[::2] + [0.02, -0.01], line))
    scans = [c for pair in cases for c in pair]
    B = len(cases)
    src, dst = np.arange(0, 2 * B, 2), np.arange(1, 2 * B, 2)
    inits = np.stack([np.eye(3)] * B)
    try:
        assert lib.slam_icp_set_screen(mode) == 0
        res = k.icp_batch(scans, src, dst, inits, epsilon=1e-12, max_iters=20, stopping_thresh=1e-14)
        _, corr, _ = k.icp_step(scans, src, dst, inits)
    finally:
        lib.slam_icp_set_screen(2)
    for b, (pc1, pc2) in enumerate(cases):
        h, e = oracle.icp(homog(pc1), homog(pc2), np.eye(3), 1e-12, 20, 1e-14)
        assert res.iters[b] == len(h) - 1, (b, mode)
        assert np.allclose(res.tf[b], h[-1], rtol=0, atol=1e-9), (b, mode)
        assert np.array_equal(corr[b], oracle.correspondences(homog(pc1), homog(pc2))), (b, mode)
    one = rng.uniform(-1, 1, size=(1, 2))
    _, c1, _ = k.icp_step([rng.uniform(-1, 1, size=(3, 2)), one], [0], [1], np.eye(3)[None])
    assert c1[0].tolist() == [0, 0, 0]


def test_far_coordinates_use_exact_path(k, oracle):
    """|coordinates| >= 1e18 disable the fp32 screen (finite squares not
    guaranteed): the kernel falls back to the exact scan for every query."""
    rng = np.random.default_rng(4)
    pc2 = rng.uniform(-3, 3, size=(200, 2)) * 1e18
    pc1 = pc2[:150] * (1 + 1e-9)
    _, corr, _ = k.icp_step([pc1, pc2], [0], [1], np.eye(3)[None])
    assert np.array_equal(corr[0], oracle.correspondences(homog(pc1), homog(pc2)))


def _hard_clouds():
    """Scans that stress the carried clearance of the pruned screen: large
    first motions followed by small ones, unstructured clouds, exact ties on
    a lattice, and clustered duplicates."""
    rng = np.random.default_rng(31)
    scans, pairs = [], []

    def add(a, b, init):
        scans.append(a)
        scans.append(b)
        pairs.append((len(scans) - 2, len(scans) - 1, init))

    def rot(th, tx=0.0, ty=0.0):
        return np.array([[np.cos(th), -np.sin(th), tx], [np.sin(th), np.cos(th), ty], [0, 0, 1.0]])

    for th in (0.05, 0.3, 0.8):
        p2 = rng.uniform(-5, 5, size=(1081, 2))
        p1 = (p2 - [0.3, -0.2]) @ rot(th)[:2, :2] + rng.normal(0, 0.01, p2.shape)
        add(p1, p2, np.eye(3))
    g = np.stack(np.meshgrid(np.arange(33), np.arange(32)), -1).reshape(-1, 2) * 0.25   # exact ties
    add(g[:1000] + 0.125, g, rot(0.02, 0.1, -0.05))
    c = np.repeat(rng.uniform(-3, 3, size=(120, 2)), 9, axis=0) + rng.normal(0, 1e-3, (1080, 2))
    add(c[::-1] + 0.05, c, rot(-0.1))
    from slamhip import se2, synthetic
    seq = synthetic.make_sequence(7, seed=77)
    for i in range(1, 7):   # lidar pairs with a large heading error in the initial guess
        add(seq.scans[i], seq.scans[i - 1], se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) @ rot(0.4 * (-1) ** i))
    return scans, pairs


def test_nn_modes_identical_hard(k):
    """The pruned screen (carried clearance, group masks, visits) and the
    exhaustive fp64 scan give bit-identical transform histories on clouds
    built to break the pruning bounds."""
    from slamhip import _abi
    lib = _abi.lib()
    scans, pairs = _hard_clouds()
    src = np.array([p[0] for p in pairs])
    dst = np.array([p[1] for p in pairs])
    inits = np.stack([p[2] for p in pairs])
    outs = []
    try:
        for mode in (0, 2):
            assert lib.slam_icp_set_screen(mode) == 0
            outs.append(k.icp_batch(scans, src, dst, inits, epsilon=1e-9, max_iters=60, stopping_thresh=1e-12,
                                    history=True))
    finally:
        lib.slam_icp_set_screen(2)
    a, b = outs
    assert a.iters.min() > 3
    assert np.array_equal(a.iters, b.iters)
    assert np.array_equal(a.tf, b.tf) and np.array_equal(a.err, b.err)
    for h0, h1 in zip(a.hist, b.hist):
        assert np.array_equal(h0, h1)


def test_schedule_is_invisible(k):
    """The phased scheduler (probe phase, pause, re-ordered resume) returns
    bit-identical transforms, errors, iteration counts and histories to one
    launch, for every probe length, including pairs that stop inside the
    probe phase, exactly at its end, and with history recording."""
    from slamhip import _abi
    lib = _abi.lib()
    n = 300
    seq, inits = _sequence_pairs(n, seed=12, n_beams=361)
    src, dst = np.arange(1, n + 1), np.arange(0, n)
    outs = []
    try:
        assert lib.slam_icp_set_schedule_heads(0) == 0   # bit-identity of the phases alone
        for probe in (0, 1, 3, 8, 17):
            assert lib.slam_icp_set_schedule(probe, 1) == 0
            outs.append(k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=100, history=True))
        assert lib.slam_icp_set_schedule(5, 1) == 0   # rotation-only and a max_iters stop inside phase 2
        outs.append(k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=6, rotation_only=True))
        assert lib.slam_icp_set_schedule(0, 1) == 0
        ref_ro = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=6, rotation_only=True)
    finally:
        lib.slam_icp_set_schedule(-1, 1024)
        lib.slam_icp_set_schedule_auto(1)
    a = outs[0]
    assert a.iters.min() < 8 < a.iters.max()
    for o in outs[1:-1]:
        assert np.array_equal(o.iters, a.iters)
        assert np.array_equal(o.tf, a.tf) and np.array_equal(o.err, a.err)
        for h0, h1 in zip(a.hist, o.hist):
            assert np.array_equal(h0, h1)
    assert np.array_equal(outs[-1].tf, ref_ro.tf) and np.array_equal(outs[-1].iters, ref_ro.iters)
    assert np.array_equal(outs[-1].err, ref_ro.err)


def test_default_schedule_large_batch(k):
    """A batch above the scheduler threshold (2,100 pairs) through the default
    two-phase path: with and without the CU-exclusive head launch (the
    slowest-keyed pairs on the 512-thread instance) it equals the single
    launch bit for bit."""
    from slamhip import _abi
    lib = _abi.lib()
    n = 2100
    seq, inits = _sequence_pairs(n, seed=21, n_beams=181)
    src, dst = np.arange(1, n + 1), np.arange(0, n)
    phased = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=100)
    try:
        assert lib.slam_icp_set_schedule_heads(0) == 0
        plain = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=100)
        assert lib.slam_icp_set_schedule(0, 1024) == 0
        single = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=100)
    finally:
        lib.slam_icp_set_schedule(-1, 1024)
        lib.slam_icp_set_schedule_auto(1)
    assert phased.iters.max() > 5
    assert np.array_equal(plain.iters, single.iters)
    assert np.array_equal(plain.tf, single.tf) and np.array_equal(plain.err, single.err)
    assert np.array_equal(phased.iters, single.iters)
    assert np.array_equal(phased.tf, single.tf) and np.array_equal(phased.err, single.err)


def test_mid_batch_with_a_large_scan(k, oracle):
    """A 2,100-pair batch (the automatic profile's 2,048-8,192 range: the angle
    pre-tier as bulk gangs) in which ONE scan has 4,525 points, above the
    LDS-resident candidate cap of 4,096: the pre-tier and the pruned screen
    must step aside for the whole batch (the gangs stage pc2 in LDS), so
    every pair, the turning ones included, equals the single launch bit for
    bit and the oracle within 1e-9 — no EINVAL, no pair left unstarted."""
    from slamhip import _abi
    lib = _abi.lib()
    n = 2100
    seq, inits = _sequence_pairs(n, seed=21, n_beams=181)
    rng = np.random.default_rng(11)
    scans = list(seq.scans)
    big = 1000
    scans[big] = np.repeat(scans[big], 25, axis=0) + rng.normal(0.0, 1e-3, (25 * len(scans[big]), 2))
    assert len(scans[big]) > 4096
    ang = np.abs(np.arctan2(inits[:, 1, 0], inits[:, 0, 0]))
    turning = np.flatnonzero(ang > 0.3)
    assert len(turning) > 0
    src, dst = np.arange(1, n + 1), np.arange(0, n)
    lib.slam_icp_gang_timeouts()   # clear
    auto = k.icp_batch(scans, src, dst, inits, epsilon=0.05, max_iters=100)
    assert lib.slam_icp_gang_timeouts() == 0
    try:
        assert lib.slam_icp_set_schedule(0, 1024) == 0
        single = k.icp_batch(scans, src, dst, inits, epsilon=0.05, max_iters=100)
    finally:
        lib.slam_icp_set_schedule(-1, 1024)
        lib.slam_icp_set_schedule_auto(1)
    assert (auto.iters > 0).all()
    assert np.array_equal(auto.iters, single.iters)
    assert np.array_equal(auto.tf, single.tf) and np.array_equal(auto.err, single.err)
    for b in sorted(set([big - 1, big]) | set(turning[:4].tolist())):
        h, e = oracle.icp(homog(scans[b + 1]), homog(scans[b]), inits[b].copy(), 0.05, 100)
        assert auto.iters[b] == len(h) - 1, b
        assert np.abs(auto.tf[b] - h[-1]).max() <= TOL, b
        assert abs(auto.err[b] - e) <= TOL * max(1.0, e), b


def test_gangs_are_bit_identical(k):
    """Gangs (a pair's 64-query groups dealt over 2..17 workgroups that
    exchange their exact partial sums every iteration) and teams (parts = 0:
    one workgroup per query group, the group's search split over its 4 waves)
    return the single launch's transforms, errors, iteration counts and
    histories bit for bit: every part count, every pair a gang (64 of 64
    heads), and the tiers with CU-exclusive heads beside them."""
    from slamhip import _abi
    lib = _abi.lib()
    n = 1100
    seq, inits = _sequence_pairs(n, seed=2025)
    src, dst = np.arange(1, n + 1), np.arange(0, n)
    try:
        assert lib.slam_icp_set_schedule(0, 1024) == 0
        single = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=100, history=True)
        assert lib.slam_icp_set_schedule(-1, 1024) == 0
        runs = {}
        for gangs, parts in ((8, 4), (64, 2), (64, 3), (64, 5), (64, 9), (64, 17), (1, 4), (64, 0), (8, 0)):
            assert lib.slam_icp_set_schedule_gangs(gangs, parts) == 0
            runs[(gangs, parts)] = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=100, history=True)
            assert lib.slam_icp_gang_timeouts() == 0
        # the wide tier (brute-force screen over candidate slices), alone and before gangs
        # (groups 2: two query groups per 16-wave workgroup, one workgroup per CU)
        for wide, share, gangs, groups in ((64, 1, 0, 1), (8, 2, 16, 1), (3, 4, 24, 1), (24, 1, 0, 2), (64, 2, 8, 2)):
            assert lib.slam_icp_set_wide_groups(groups) == 0
            assert lib.slam_icp_set_schedule_gangs(gangs, 4) == 0
            assert lib.slam_icp_set_schedule_wide(wide, share) == 0
            runs[("wide", wide, share, gangs, groups)] = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05,
                                                                     max_iters=100, history=True)
            assert lib.slam_icp_gang_timeouts() == 0
        assert lib.slam_icp_set_wide_groups(1) == 0
        assert lib.slam_icp_set_schedule_wide(0, 1) == 0
        # the angle pre-tier: the turning pairs on the wide tier from their
        # initial transforms, beside phase 1 of the rest (with gangs, with heads only)
        # (kind 0: wide workgroups; 2 / 3: bulk gangs of that many workgroups)
        for amax, athr, gangs, kind in ((24, 0.3, 24, 0), (64, 0.05, 24, 0), (8, 0.3, 0, 0), (48, 0.3, 24, 3),
                                        (96, 0.05, 0, 2), (200, 0.05, 24, 3), (40, 0.05, 0, 20), (64, 0.05, 24, 4),
                                        (64, 0.05, 0, 6)):
            # kind 20: the wide pre-tier with two query groups per workgroup
            assert lib.slam_icp_set_wide_groups(2 if kind == 20 else 1) == 0
            kind = 0 if kind == 20 else kind
            assert lib.slam_icp_set_schedule_gangs(gangs, 4) == 0
            assert lib.slam_icp_set_angle_tier(amax, athr) == 0
            assert lib.slam_icp_set_angle_tier_kind(kind) == 0
            runs[("angle", amax, athr, gangs, kind)] = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05,
                                                                   max_iters=100, history=True)
            assert lib.slam_icp_gang_timeouts() == 0
        # the mixed pre-tier: its largest turns on wide workgroups, the rest on gangs of 3
        for amax, mix, share in ((48, 8, 2), (96, 16, 4), (24, 24, 1)):
            assert lib.slam_icp_set_angle_tier(amax, 0.05) == 0
            assert lib.slam_icp_set_angle_tier_kind(3) == 0
            assert lib.slam_icp_set_angle_tier_mix(mix, share) == 0
            runs[("mix", amax, mix, share)] = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=100,
                                                          history=True)
            assert lib.slam_icp_gang_timeouts() == 0
        assert lib.slam_icp_set_angle_tier_mix(0, 2) == 0
        assert lib.slam_icp_set_wide_groups(1) == 0
        assert lib.slam_icp_set_angle_tier(*DEFAULT_ANGLE) == 0
        assert lib.slam_icp_set_angle_tier_kind(0) == 0
        # bulk gangs: both phases' bulk as gangs of 2 / 3 ordinary workgroups
        for parts in (2, 3):
            assert lib.slam_icp_set_bulk_gangs(4096, parts) == 0
            assert lib.slam_icp_set_schedule_gangs(24, 4) == 0
            runs[("bulk", parts)] = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=100, history=True)
            assert lib.slam_icp_gang_timeouts() == 0
        assert lib.slam_icp_set_bulk_gangs(*DEFAULT_BULK) == 0
        assert lib.slam_icp_set_schedule_gangs(64, 4) == 0   # rotation-only, max_iters stop inside phase 2
        ro = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=7, rotation_only=True)
        assert lib.slam_icp_set_schedule(0, 1024) == 0
        ro_single = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=7, rotation_only=True)
        assert lib.slam_icp_set_schedule_gangs(1, 1) != 0   # a gang needs two parts
    finally:
        lib.slam_icp_set_wide_groups(1)
        lib.slam_icp_set_schedule(-1, 1024)
        lib.slam_icp_set_bulk_gangs(*DEFAULT_BULK)
        lib.slam_icp_set_schedule_auto(1)
    assert single.iters.max() > 30
    for key, r in runs.items():
        assert np.array_equal(r.iters, single.iters), key
        assert np.array_equal(r.tf, single.tf) and np.array_equal(r.err, single.err), key
        for h0, h1 in zip(single.hist, r.hist):
            assert np.array_equal(h0, h1), key
    assert np.array_equal(ro.iters, ro_single.iters)
    assert np.array_equal(ro.tf, ro_single.tf) and np.array_equal(ro.err, ro_single.err)


def test_gang_timeouts_are_repaired(k):
    """A gang part that waits too long for its partners stops without writing;
    after phase 2 the scheduler re-runs every unfinished gang pair on one
    workgroup from its phase-1 state.  With the wait forced down to one tick
    (timeouts in most exchanges) the results are still bit-identical to the
    single launch, for gangs and for teams, and the timeouts are reported."""
    from slamhip import _abi
    lib = _abi.lib()
    n = 1100
    seq, inits = _sequence_pairs(n, seed=2025)
    src, dst = np.arange(1, n + 1), np.arange(0, n)
    try:
        assert lib.slam_icp_set_schedule(0, 1024) == 0
        single = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=100, history=True)
        assert lib.slam_icp_set_schedule(-1, 1024) == 0
        assert lib.slam_icp_set_gang_wait(1) == 0
        lib.slam_icp_gang_timeouts()   # clear
        for gangs, parts, wide, bulk, angle, kind, groups in ((64, 4, 0, 0, 0, 0, 1), (16, 0, 0, 0, 0, 0, 1),
                                                              (0, 4, 16, 0, 0, 0, 1), (8, 4, 0, 2, 0, 0, 1),
                                                              (0, 4, 0, 3, 0, 0, 1), (0, 4, 0, 0, 16, 0, 1),
                                                              (24, 4, 0, 0, 48, 3, 1), (0, 4, 16, 0, 0, 0, 2),
                                                              (0, 4, 0, 0, 16, 0, 2)):
            assert lib.slam_icp_set_wide_groups(groups) == 0
            assert lib.slam_icp_set_schedule_gangs(gangs, parts) == 0
            assert lib.slam_icp_set_schedule_wide(wide, 1) == 0
            assert lib.slam_icp_set_bulk_gangs(4096 if bulk else 0, max(bulk, 2)) == 0
            assert lib.slam_icp_set_angle_tier(angle, 0.1) == 0
            assert lib.slam_icp_set_angle_tier_kind(kind) == 0
            r = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=100, history=True)
            assert lib.slam_icp_gang_timeouts() > 0, (gangs, parts, wide)
            assert np.array_equal(r.iters, single.iters), (gangs, parts)
            assert np.array_equal(r.tf, single.tf) and np.array_equal(r.err, single.err), (gangs, parts)
            for h0, h1 in zip(single.hist, r.hist):
                assert np.array_equal(h0, h1), (gangs, parts)
    finally:
        lib.slam_icp_set_wide_groups(1)
        lib.slam_icp_set_gang_wait(0)
        lib.slam_icp_set_schedule(-1, 1024)
        lib.slam_icp_set_bulk_gangs(*DEFAULT_BULK)
        lib.slam_icp_set_schedule_auto(1)
    assert lib.slam_icp_gang_timeouts() == 0


def test_drain_tier_is_bit_identical(k):
    """The drain tier (phase 2's last running pairs paused and finished on wide
    workgroups): every setting, and forced exchange timeouts (the wide pairs
    then finish in the repair launch), give the drain-off results bit for bit,
    history included, on a 2,500-pair stream and a 10,000-pair-size batch path
    (B > 8,192: the three-kernel sort)."""
    from slamhip import _abi
    lib = _abi.lib()
    n = 2500
    seq, inits = _sequence_pairs(n, seed=2025)
    src, dst = np.arange(1, n + 1), np.arange(0, n)
    try:
        assert lib.slam_icp_set_drain(0) == 0
        ref = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=100, history=True)
        for d, wait in ((1, 0), (8, 0), (24, 0), (64, 0), (24, 1)):
            assert lib.slam_icp_set_drain(d) == 0
            assert lib.slam_icp_set_gang_wait(wait) == 0
            lib.slam_icp_gang_timeouts()   # clear
            r = k.icp_batch(seq.scans, src, dst, inits, epsilon=0.05, max_iters=100, history=True)
            if wait:
                assert lib.slam_icp_gang_timeouts() > 0, d
            assert np.array_equal(r.iters, ref.iters), d
            assert np.array_equal(r.tf, ref.tf) and np.array_equal(r.err, ref.err), d
            for h0, h1 in zip(ref.hist, r.hist):
                assert np.array_equal(h0, h1), d
        # the large-batch path: 9,000 pairs (3 x the stream, B > 8,192)
        assert lib.slam_icp_set_gang_wait(0) == 0
        s3, d3, i3 = np.tile(src, 3)[:9000], np.tile(dst, 3)[:9000], np.tile(inits, (3, 1, 1))[:9000]
        assert lib.slam_icp_set_drain(0) == 0
        big0 = k.icp_batch(seq.scans, s3, d3, i3, epsilon=0.05, max_iters=100)
        assert lib.slam_icp_set_drain(24) == 0
        big1 = k.icp_batch(seq.scans, s3, d3, i3, epsilon=0.05, max_iters=100)
        assert np.array_equal(big1.iters, big0.iters) and np.array_equal(big1.tf, big0.tf)
        assert np.array_equal(big0.iters[:n], ref.iters) and np.array_equal(big0.tf[:n], ref.tf)
    finally:
        lib.slam_icp_set_gang_wait(0)
        lib.slam_icp_set_drain(-1)
    assert lib.slam_icp_gang_timeouts() == 0


_OCCUPIER = """
import sys, time
sys.path.insert(0, sys.argv[1])
import torch
from slamhip import _abi
torch.cuda.set_device(0)
lib = _abi.lib()
assert lib.slam_icp_diag_occupy(int(sys.argv[2]), int(sys.argv[3]), None) == 0
print("launched", flush=True)
torch.cuda.synchronize()
print("done", flush=True)
"""


def test_occupied_cus_do_not_stall_the_exchange_tiers(k):
    """Another PROCESS holding all but 32 CUs (one CU-exclusive workgroup each)
    for 0.6 s while an 8-rank-size shard (1,250 pairs; the wide pre-tier needs
    9 whole CUs per turning pair) runs: wide pairs whose parts are not all
    resident give up after the first exchange's 4 ms wait, mark the pair's
    slots so the partners stop at once, and run in the repair launch — the
    batch ends in tens of ms, not at the end of the occupation, bit-identical
    to an unoccupied run, the timeouts reported (tools/occupy_probe.py:
    ~18 ms; with all but 8 CUs held even a one-kernel torch op waits out the
    occupation, so that is not a test of the library)."""
    import os
    import select
    import subprocess
    import sys
    import time
    import torch
    from conftest import PKG
    from slamhip import _abi
    lib = _abi.lib()
    n = 1250
    seq, inits = _sequence_pairs(n, seed=2025)
    ss = k.ScanSet(seq.scans)
    b = k.IcpBatch(ss, np.arange(1, n + 1), np.arange(0, n), inits, epsilon=0.05, max_iters=100)
    b.launch()
    ref = b.result()
    assert lib.slam_icp_gang_timeouts() == 0
    assert (np.abs(np.arctan2(inits[:, 1, 0], inits[:, 0, 0])) > 0.3).sum() >= 8   # wide pre-tier pairs
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    occ = subprocess.Popen([sys.executable, "-c", _OCCUPIER, PKG, str(n_cu - 32), "60000000"],   # 0.6 s
                           stdout=subprocess.PIPE, text=True, env=dict(os.environ))
    try:
        ready, _, _ = select.select([occ.stdout], [], [], 90)
        assert ready and occ.stdout.readline().strip() == "launched"
        time.sleep(0.05)   # the occupying workgroups are resident
        t0 = time.perf_counter()
        b.launch()
        done = torch.cuda.Event()
        done.record()
        done.synchronize()
        dt = time.perf_counter() - t0
        assert occ.wait(timeout=30) == 0
    finally:
        if occ.poll() is None:
            occ.kill()
    r = b.result()
    assert np.array_equal(r.iters, ref.iters)
    assert np.array_equal(r.tf, ref.tf) and np.array_equal(r.err, ref.err)
    assert lib.slam_icp_gang_timeouts() > 0
    assert dt < 0.15, dt


@pytest.mark.parametrize("B", [9000, 5000, 4096, 1250, 37])
def test_scheduler_order_is_a_stable_sort(B):
    """Phase 2's visiting order is the scheduler's stable bucket sort: the same
    permutation every run, unfinished pairs by bucket of log2 |dE| (largest
    |dE| first, 8 buckets per octave), pair index ascending inside a bucket,
    finished and out-of-bounds pairs last in index order, pairs that never
    started (out_iters 0: a timed-out phase-1 gang; key never written) first.
    B > 8,192: the three-kernel sort; B <= 8,192: the one-workgroup sort of
    the strong-scaling shards."""
    import ctypes
    import torch
    from slamhip import _abi
    lib = _abi.lib()
    rng = np.random.default_rng(4)
    thresh = 1e-4
    kq = rng.integers(-40, 120, B)                             # bucket 128 - 8 log2(key / thresh) = 127 - kq
    key = (thresh * np.exp2((kq + 0.5) / 8.0)).astype(np.float32)   # mid-bucket: no rounding ambiguity
    u = rng.random(B)
    iters = np.where(u < 0.2, 7, -4).astype(np.int32)             # 20 % finished in phase 1
    iters[(u >= 0.2) & (u < 0.23)] = 0                            # never started: bucket 0
    iters[(u >= 0.23) & (u < 0.25)] = np.iinfo(np.int32).min      # out of bounds: last
    key[iters == 0] = np.float32(np.nan)                          # unwritten key: never read
    dev = torch.device("cuda", 0)
    d_it = torch.tensor(iters, device=dev)
    d_key = torch.tensor(key, device=dev)
    outs = []
    for _ in range(3):
        d_ord = torch.full((B,), -1, dtype=torch.int32, device=dev)
        assert lib.slam_icp_sched_sort(ctypes.c_void_p(d_it.data_ptr()), ctypes.c_void_p(d_key.data_ptr()), B,
                                       ctypes.c_float(thresh), ctypes.c_void_p(d_ord.data_ptr()), None) == 0
        torch.cuda.synchronize()
        outs.append(d_ord.cpu().numpy())
    assert all(np.array_equal(o, outs[0]) for o in outs[1:])
    bucket = np.where((iters > 0) | (iters == np.iinfo(np.int32).min), 256,
                      np.where(iters == 0, 0, np.clip(127 - kq, 0, 255)))
    want = np.lexsort((np.arange(B), bucket))
    assert np.array_equal(outs[0], want)


def test_default_schedule_c3_shape_vs_oracle(k, oracle):
    """The benchmarked path itself: 2,400 consecutive pairs of 1081-point scans
    (the C3 stream generator, seed 2025) through the DEFAULT two-phase
    scheduler; a strided sample plus the longest-running pairs against the
    CPU oracle (scripts/main.py:240-247 parameters): iteration counts equal,
    transforms within 1e-9, errors within 1e-9 relative."""
    n = 2400
    seq, inits = _sequence_pairs(n, seed=2025)
    assert min(len(s) for s in seq.scans) > 1000
    res = k.icp_batch(seq.scans, np.arange(1, n + 1), np.arange(0, n), inits, epsilon=0.05, max_iters=100)
    sample = sorted(set(range(0, n, 200)) | set(np.argsort(res.iters)[-4:].tolist()))
    assert res.iters.max() > 30          # the long tail reaches deep into phase 2
    for b in sample:
        h, e = oracle.icp(homog(seq.scans[b + 1]), homog(seq.scans[b]), inits[b].copy(), 0.05, 100)
        assert res.iters[b] == len(h) - 1, b
        assert np.abs(res.tf[b] - h[-1]).max() <= TOL, b
        assert abs(res.err[b] - e) <= TOL * max(1.0, e), b


def test_c3_full_stream_and_gpu_count_independence(k, oracle):
    """The headline configuration itself (BASELINE.json configs[2]): ONE
    10,000-pair stream of 1081-beam scans (SURVEY.md §8(d) generator, seed
    2025) through the DEFAULT path — the launch bench.py times (two-phase
    scheduler, no head pairs at this size).  A strided sample plus the longest
    pairs against the CPU oracle (scripts/main.py:240-247 parameters); then
    the first and last shards of 2 / 4 / 8 ranks (5,000 / 2,500 / 1,250
    pairs: CU-exclusive head pairs on the 512-thread instance) are
    BIT-identical to the matching rows of the 10k run — a pair's result does
    not depend on the number of GPUs the stream is sharded over."""
    from slamhip import dist as sd
    n = 10000
    seq, inits = _sequence_pairs(n, seed=2025)
    ss = k.ScanSet(seq.scans)
    full = k.IcpBatch(ss, np.arange(1, n + 1), np.arange(0, n), inits, epsilon=0.05, max_iters=100)
    full.launch()
    res = full.result()
    assert res.iters.max() > 90          # the C3 tail (pairs 1118, 7264) is in the run
    for world in (2, 4, 8):
        for rank in (0, world - 1):
            lo, hi, _ = sd.shard_range(n, world, rank)
            sh = k.IcpBatch(ss, np.arange(lo + 1, hi + 1), np.arange(lo, hi), inits[lo:hi], epsilon=0.05,
                            max_iters=100)
            sh.launch()
            r = sh.result()
            assert np.array_equal(r.iters, res.iters[lo:hi]), (world, rank)
            assert np.array_equal(r.tf, res.tf[lo:hi]) and np.array_equal(r.err, res.err[lo:hi]), (world, rank)
    sample = sorted(set(range(0, n, 500)) | set(np.argsort(res.iters)[-3:].tolist()))
    for b in sample:
        h, e = oracle.icp(homog(seq.scans[b + 1]), homog(seq.scans[b]), inits[b].copy(), 0.05, 100)
        assert res.iters[b] == len(h) - 1, b
        assert np.abs(res.tf[b] - h[-1]).max() <= TOL, b
        assert abs(res.err[b] - e) <= TOL * max(1.0, e), b


def test_understated_bounds_are_flagged(k):
    """A raw C caller that passes max_n1 / max_n2 below the real scan sizes
    gets SLAM_EINVAL from slam_icp_status (the offending pairs are not
    computed), not silently wrong results; correct bounds then work again."""
    from slamhip import _abi
    n = 6
    seq, inits = _sequence_pairs(n, seed=3, n_beams=361)
    ss = k.ScanSet(seq.scans)
    for attr, val in (("max_n2", 200), ("max_n1", 100)):
        b = k.IcpBatch(ss, np.arange(1, n + 1), np.arange(0, n), inits, epsilon=0.05, max_iters=100)
        setattr(b, attr, val)
        b.launch()
        with pytest.raises(_abi.SlamHipError, match="bounds"):
            b.result()
        assert (b.out_iters[:n].cpu().numpy() == np.iinfo(np.int32).min).all()
    good = k.IcpBatch(ss, np.arange(1, n + 1), np.arange(0, n), inits, epsilon=0.05, max_iters=100)
    good.launch()
    assert (good.result().iters > 0).all()


def test_large_query_scan_lds_fallback(k, oracle):
    """A 6,000-point query scan against 4,000 candidates: the 512x16 instance's
    per-query LDS state does not fit beside 4,096 candidates, so the launch
    takes the full fp32 screen (same results) instead of the pruned one."""
    from slamhip import se2
    rng = np.random.default_rng(5)
    th = np.sort(rng.uniform(-2.3, 2.3, 4000))
    r = 3 + 0.5 * np.sin(5 * th)
    pc2 = np.c_[r * np.cos(th), r * np.sin(th)]
    th1 = np.sort(rng.uniform(-2.3, 2.3, 6000))
    r1 = 3 + 0.5 * np.sin(5 * th1)
    T = se2.pose_to_mat([0.05, -0.03, 0.02])
    pc1 = (np.linalg.inv(T) @ np.c_[r1 * np.cos(th1), r1 * np.sin(th1), np.ones(6000)].T).T[:, :2]
    res = k.icp_batch([pc1, pc2], [0], [1], np.eye(3)[None], epsilon=0.05, max_iters=30)
    h, e = oracle.icp(homog(pc1), homog(pc2), np.eye(3), 0.05, 30)
    assert res.iters[0] == len(h) - 1
    assert np.abs(res.tf[0] - h[-1]).max() <= TOL

