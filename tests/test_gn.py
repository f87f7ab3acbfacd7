"""Gauss-Newton pose-graph solve: planner host logic (CPU) and GPU parity
against the float64 oracle (oracle/gn_oracle.py).

The reference has no GN, so parity is "HIP vs the build's
own CPU restatement" and is unpinned against the reference; tolerance 1e-8 on
poses after several iterations (band Cholesky vs SuperLU rounding)."""
import numpy as np
import pytest

import gn_oracle as go


def _random_graph(N, n_loops, seed):
    from slamhip import se2
    rng = np.random.default_rng(seed)
    truth = np.cumsum(rng.normal(0, [0.3, 0.3, 0.2], size=(N, 3)), axis=0)
    ea, eb, tf = [], [], []

    def rel(a, b):
        c, s = np.cos(truth[a, 2]), np.sin(truth[a, 2])
        d = truth[b, :2] - truth[a, :2]
        return se2.pose_to_mat([c * d[0] + s * d[1], -s * d[0] + c * d[1], truth[b, 2] - truth[a, 2]])

    for i in range(N - 1):
        ea.append(i)
        eb.append(i + 1)
        tf.append(rel(i, i + 1) @ se2.pose_to_mat(rng.normal(0, [0.02, 0.02, 0.01])))
    for _ in range(n_loops):
        a, b = rng.choice(N, 2, replace=False)
        ea.append(int(a))
        eb.append(int(b))
        tf.append(rel(a, b))
    guess = truth + rng.normal(0, [0.1, 0.1, 0.05], size=(N, 3))
    guess[0] = truth[0]
    return guess, np.array(ea), np.array(eb), np.stack(tf)


def test_plan_covers_every_edge():
    from slamhip import gn
    guess, ea, eb, tf = _random_graph(60, 40, 1)
    p = gn.GnPlan(len(guess), ea, eb)
    assert p.nv == 3 * 59 and p.node_col[0] == -1
    cols = p.node_col
    assert sorted(cols[cols >= 0]) == list(range(0, p.nv, 3))
    # every non-self edge appears in the diagonal slots of its free endpoints
    # and in exactly one pair slot when both are free
    seen_diag, seen_pair = {}, {}
    for s in range(p.n_slots):
        r0, c0 = p.slot_rc[s]
        for it in p.slot_items[p.slot_ptr[s]:p.slot_ptr[s + 1]]:
            key = (int(it) >> 1, int(it) & 1)
            (seen_diag if r0 == c0 else seen_pair)[key] = seen_diag.get(key, 0) + 1
            assert r0 >= c0 and r0 - c0 <= p.W
    for e in range(len(ea)):
        if ea[e] == eb[e]:
            continue
        if cols[ea[e]] >= 0:
            assert (e, 0) in seen_diag
        if cols[eb[e]] >= 0:
            assert (e, 1) in seen_diag
    assert len(seen_pair) == sum(1 for e in range(len(ea)) if cols[ea[e]] >= 0 and cols[eb[e]] >= 0)
    # bandwidth is tight
    both = (cols[ea] >= 0) & (cols[eb] >= 0)
    assert p.W == max(2, np.abs(cols[ea][both] - cols[eb][both]).max() + 2)


def test_place_major_order_on_c4():
    """C4's lap structure: the place-major order (places = components of the
    loop-closure edges, RCM over the place graph) gives a 62-scalar band
    (BCR blocks of 64 rows) where RCM over the poses gives 77 (80-row blocks);
    band_order keeps RCM where places do not narrow the band."""
    import scipy.sparse as sp
    from scipy.sparse.csgraph import reverse_cuthill_mckee
    from slamhip import gn, synthetic
    guess, ea, eb, tf, truth = synthetic.lap_graph_c4()
    N = len(guess)
    order, name, w = gn.band_order(N, ea, eb)
    assert name == "place-major" and w == 62
    assert gn.GnPlan(N, ea, eb, order=order).W == 62
    order = gn.place_order(N, np.asarray(ea, np.int64), np.asarray(eb, np.int64))
    assert sorted(order.tolist()) == list(range(N))
    adj = sp.coo_matrix((np.ones(2 * len(ea)), (np.r_[ea, eb], np.r_[eb, ea])), shape=(N, N)).tocsr()
    assert gn.GnPlan(N, ea, eb, order=reverse_cuthill_mckee(adj, symmetric_mode=True)).W == 77
    # sparse loops (incomplete places): RCM stays
    guess, ea, eb, tf, truth = synthetic.lap_graph_c4(poses_per_side=25, num_loops=3, n_loops=200)
    assert gn.band_order(len(guess), ea, eb)[1] == "rcm"


def test_border_plan():
    """Band + border plans: C4 cut at the fixed node's place (27 border
    scalars, band 32); the border's coupling rows; a given border on a random
    graph; columns a permutation with the border last."""
    from slamhip import gn, synthetic
    guess, ea, eb, tf, truth = synthetic.lap_graph_c4()
    N = len(guess)
    p = gn.GnPlan(N, ea, eb)
    assert p.ordering == "place-major + border" and p.W == 32 and p.nv - p.nv_band == 27
    cols = p.node_col
    assert sorted(cols[cols >= 0]) == list(range(0, p.nv, 3)) and cols[0] == -1
    border = np.flatnonzero(cols >= p.nv_band)
    assert len(border) == 9 and set(border % 500) == {0}   # the other laps' poses at place 0
    ea, eb = np.asarray(ea), np.asarray(eb)
    ca, cb = cols[ea], cols[eb]
    rows = set()
    for a, b in zip(ca, cb):
        if a >= 0 and b >= 0 and (a >= p.nv_band) != (b >= p.nv_band):
            rows.update(range(min(a, b), min(a, b) + 3))
    assert sorted(rows) == p.nbr_rows.tolist()
    band = (ca >= 0) & (cb >= 0) & (ca < p.nv_band) & (cb < p.nv_band)
    assert np.abs(ca[band] - cb[band]).max() + 2 == p.W
    guess, ea, eb, tf = _random_graph(90, 30, 5)
    q = gn.GnPlan(len(guess), ea, eb, border=[3, 17, 44, 60])
    assert q.nv - q.nv_band == 12 and all(q.node_col[[3, 17, 44, 60]] >= q.nv_band)
    with pytest.raises(ValueError):
        gn.GnPlan(len(guess), ea, eb, border=list(range(1, 12)))


def test_oracle_converges_on_c4():
    from slamhip import synthetic
    guess, ea, eb, tf, truth = synthetic.lap_graph_c4(poses_per_side=25, num_loops=4, n_loops=300)
    p, chis = go.optimize(guess, ea, eb, tf, iterations=5)
    assert chis[-1] < 1e-3 * chis[0]
    assert np.abs(p[:, :2] - truth[:, :2]).max() < 0.1


@pytest.mark.gpu
@pytest.mark.parametrize("iters", [1, 3])
@pytest.mark.parametrize("mode", [1, 2])
def test_gn_small_vs_oracle(solver, iters, mode):
    from slamhip import gn
    solver(mode)
    guess, ea, eb, tf = _random_graph(80, 30, 2)
    ref, ref_chi = go.optimize(guess, ea, eb, tf, iterations=iters)
    got, chi = gn.optimize(guess, ea, eb, tf, iterations=iters)
    assert np.allclose(chi, ref_chi, rtol=1e-9, atol=1e-9)
    assert np.abs(got[:, :2] - ref[:, :2]).max() <= 1e-8
    assert np.abs(go.wrap(got[:, 2] - ref[:, 2])).max() <= 1e-8


@pytest.fixture
def solver():
    """Select the GN linear solver for one test (1 band Cholesky, 2 block cyclic reduction)."""
    from slamhip import _abi
    lib = _abi.lib()

    def use(mode):
        assert lib.slam_gn_set_solver(mode) == 0
    yield use
    lib.slam_gn_set_solver(0)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
def test_gn_c4_vs_oracle(solver, mode):
    """Config C4: 5,000 nodes / 20,000 edges, 5 iterations, both linear solvers."""
    from slamhip import _abi, gn, synthetic
    solver(mode)
    guess, ea, eb, tf, truth = synthetic.lap_graph_c4()
    if mode == 2:   # default plan: place-major band of 32 scalars + a 27-scalar border
        p = gn.GnPlan(len(guess), ea, eb)
        assert p.nv - p.nv_band == 27 and p.W == 32
        assert _abi.lib().slam_gn_bcr_block_rows(p.nv_band, p.W) > 0
    else:           # band Cholesky: the default plan takes no border under mode 1
        p = gn.plan_for(len(guess), ea, eb)
        assert p.nv == p.nv_band
        q = gn.GnPlan(len(guess), ea, eb, allow_border=True)
        assert q.nv_band < q.nv
    ref, ref_chi = go.optimize(guess, ea, eb, tf, iterations=5)
    got, chi = gn.optimize(guess, ea, eb, tf, iterations=5, plan=p)
    assert np.allclose(chi, ref_chi, rtol=1e-8)
    assert np.abs(got[:, :2] - ref[:, :2]).max() <= 1e-8
    assert np.abs(go.wrap(got[:, 2] - ref[:, 2])).max() <= 1e-8
    assert chi[-1] < 1e-3 * chi[0]


@pytest.mark.gpu
@pytest.mark.parametrize("border", [[5], [3, 17, 44, 60], [1, 2, 20, 21, 40, 41, 70, 71, 89, 88]])
def test_gn_border_random_graph(border):
    """A given border on a random graph (the band of the rest by RCM / place
    order, the border solved by the Schur complement after the multi-RHS BCR)
    against the oracle; the border's scalars take 1, 2 and 3 right-hand-side
    column tiles' worth of columns (3, 12 and 30 scalars)."""
    from slamhip import _abi, gn
    guess, ea, eb, tf = _random_graph(120, 25, 6)
    p = gn.GnPlan(len(guess), ea, eb, border=border)
    assert p.nv - p.nv_band == 3 * len(border)
    if _abi.lib().slam_gn_bcr_block_rows(p.nv_band, p.W) == 0:
        pytest.skip("band too wide for the cyclic-reduction solver")
    ref, ref_chi = go.optimize(guess, ea, eb, tf, iterations=3)
    got, chi = gn.optimize(guess, ea, eb, tf, iterations=3, plan=p)
    assert np.allclose(chi, ref_chi, rtol=1e-9, atol=1e-9)
    assert np.abs(got[:, :2] - ref[:, :2]).max() <= 1e-8
    assert np.abs(go.wrap(got[:, 2] - ref[:, 2])).max() <= 1e-8


@pytest.mark.gpu
def test_gn_wide_band_global_window():
    """Random long-range loops: the band exceeds the LDS window, exercising the
    global-memory Cholesky window."""
    from slamhip import _abi, gn
    guess, ea, eb, tf = _random_graph(150, 120, 3)
    plan = gn.GnPlan(len(guess), ea, eb)
    assert plan.W > _abi.lib().slam_gn_max_lds_band()
    ref, ref_chi = go.optimize(guess, ea, eb, tf, iterations=2)
    got, chi = gn.optimize(guess, ea, eb, tf, iterations=2)
    assert np.allclose(chi, ref_chi, rtol=1e-9)
    assert np.abs(got[:, :2] - ref[:, :2]).max() <= 1e-8


@pytest.mark.gpu
def test_optimize_pose_graph_dropin():
    """src.pose_graph_optimization.optimize_pose_graph on a reference-style
    PoseGraph (odometry edges from PoseGraph.__init__, identity loop edges):
    the GPU solve of the converted measurements equals the oracle's."""
    import src.pose_graph as pgm
    import src.pose_graph_optimization as pgo
    from slamhip import synthetic
    poses, loops = synthetic.lap_pose_graph(seed=0)
    pg = pgm.PoseGraph(poses.copy())
    for a, b in loops:
        pg.add_constraint(a, b, np.eye(3))
    ea, eb, tf = pgo.gn_measurements(pg)      # constructor deltas -> node frames; loop edges inverted
    ref, ref_chi = go.optimize(poses.copy(), ea, eb, tf, iterations=3)
    obj = pg.poses
    chis = pgo.optimize_pose_graph(pg, iterations=3, return_history=True)
    assert pg.poses is obj
    assert np.allclose(chis, ref_chi, rtol=1e-8)
    assert np.abs(pg.poses[:, :2] - ref[:, :2]).max() <= 1e-8


@pytest.mark.gpu
@pytest.mark.parametrize("n_nodes", [40, 600])
@pytest.mark.parametrize("mode", [1, 2])
def test_gn_narrow_band(solver, n_nodes, mode):
    """Bands narrower than the 16-column Cholesky block (W < S): pure chains
    (W = 5) and a loop sequence whose RCM order folds the ring (W = 14) — the
    look-ahead must not read panel rows beyond the band."""
    from slamhip import gn, synthetic
    import src.pose_graph as pgm
    solver(mode)
    s = synthetic.make_loop_sequence(n_nodes, seed=4)
    pg = pgm.PoseGraph(s.odometry.copy())
    for i, j in s.loop_pairs:
        pg.add_constraint(int(i), int(j), np.eye(3))
    ea, eb, tf = pg.edge_arrays()
    assert gn.GnPlan(n_nodes, ea, eb).W < 16
    ref, ref_chi = go.optimize(s.odometry.copy(), ea, eb, tf, iterations=3)
    got, chi = gn.optimize(s.odometry.copy(), ea, eb, tf, iterations=3)
    assert np.allclose(chi, ref_chi, rtol=1e-8)
    assert np.abs(got[:, :2] - ref[:, :2]).max() <= 1e-8


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(25, 3, 200), (40, 4, 500), (25, 6, 400), (30, 8, 800), (60, 12, 2000)])
def test_gn_bcr_block_sizes(shape):
    """Lap graphs whose RCM bands give cyclic-reduction blocks of 32, 48, 64
    and 96 rows (register tiles 2..6), and one too wide for it (W = 125 ->
    band Cholesky): both paths against the oracle."""
    from slamhip import _abi, gn, synthetic
    pps, nl, nloops = shape
    guess, ea, eb, tf, truth = synthetic.lap_graph_c4(poses_per_side=pps, num_loops=nl, n_loops=nloops)
    p = gn.GnPlan(len(guess), ea, eb)
    Wb = _abi.lib().slam_gn_bcr_block_rows(p.nv_band, p.W)
    assert (Wb == 0) == (p.W > 96)
    ref, ref_chi = go.optimize(guess, ea, eb, tf, iterations=3)
    got, chi = gn.optimize(guess, ea, eb, tf, iterations=3)
    assert np.allclose(chi, ref_chi, rtol=1e-8)
    assert np.abs(got[:, :2] - ref[:, :2]).max() <= 1e-8


@pytest.mark.gpu
def test_gn_graph_replay_matches_eager():
    """The captured HIP graph of k GN steps gives the eager launches' bits."""
    from slamhip import gn, synthetic
    guess, ea, eb, tf, truth = synthetic.lap_graph_c4(poses_per_side=25, num_loops=4, n_loops=300)
    a = gn.GaussNewton(guess, ea, eb, tf)
    chi_e = np.concatenate([a.run(1, graph=False), a.run(3, graph=False)])
    b = gn.GaussNewton(guess, ea, eb, tf)
    chi_g = np.concatenate([b.run(1, graph=False), b.run(3, graph=True)])
    assert np.array_equal(chi_e, chi_g)
    assert np.array_equal(a.host_poses(), b.host_poses())


@pytest.mark.gpu
def test_gn_fused_back_substitution_and_fallback():
    """The Schur path's XCD-local back-substitution (every level in one launch,
    tagged hand-offs; default) equals the per-level launches bit for bit (C4,
    6 iterations, eager and graph-replayed); with its wait forced down to one
    tick every fused step times out, GaussNewton warns, restores the poses and
    re-runs with the per-level launches: the same bits again."""
    import warnings
    from slamhip import _abi, gn, synthetic
    lib = _abi.lib()
    guess, ea, eb, tf, truth = synthetic.lap_graph_c4()
    try:
        assert lib.slam_gn_set_fused_back(0) == 0
        a = gn.GaussNewton(guess, ea, eb, tf)
        chi_a = np.concatenate([a.run(1, graph=False), a.run(5, graph=True)])
        assert lib.slam_gn_set_fused_back(1) == 0 and lib.slam_gn_get_fused_back() == 1
        b = gn.GaussNewton(guess, ea, eb, tf)
        chi_b = np.concatenate([b.run(1, graph=False), b.run(5, graph=True)])
        assert np.array_equal(chi_a, chi_b)
        assert np.array_equal(a.host_poses(), b.host_poses())
        # another instance holding a graph captured WITH the fused kernel
        d = gn.GaussNewton(guess, ea, eb, tf)
        d.run(1, graph=False)
        d.run(5, graph=True)
        n_fb = gn.FUSED_BACK_FALLBACKS
        assert lib.slam_gn_set_fused_wait(1) == 0
        c = gn.GaussNewton(guess, ea, eb, tf)
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            chi_c = np.concatenate([c.run(1, graph=False), c.run(5, graph=False)])
        assert any("timed out" in str(x.message) for x in w)
        assert lib.slam_gn_get_fused_back() == 0
        assert gn.FUSED_BACK_FALLBACKS == n_fb + 1
        assert np.array_equal(chi_a, chi_c)
        assert np.array_equal(a.host_poses(), c.host_poses())
        # d must not replay its fused graph once the fallback turned the kernel off
        import torch
        d.poses.copy_(torch.as_tensor(guess, dtype=torch.float64).reshape(d.poses.shape))
        chi_d = np.concatenate([d.run(1, graph=False), d.run(5, graph=True)])
        assert np.array_equal(chi_a, chi_d)
        assert np.array_equal(a.host_poses(), d.host_poses())
    finally:
        lib.slam_gn_set_fused_wait(0)
        lib.slam_gn_set_fused_back(1)


def test_oracle_jacobians_match_finite_differences():
    """The GN oracle's analytic Jacobians A = de/dx_a, B = de/dx_b against
    central differences of its own residual (self-consistency of the oracle)."""
    guess, ea, eb, tf = _random_graph(30, 20, 7)
    z = go.edge_measurements(tf)
    w = go.information(ea, eb)
    e0, A, B = go.linearize(guess, ea, eb, z, w)
    h = 1e-6
    for side, J in ((ea, A), (eb, B)):
        for c in range(3):
            num = np.zeros_like(e0)
            for sgn in (1, -1):
                p = guess.copy()
                # perturb node side[e] of every edge separately: one edge at a time
                for e in range(len(ea)):
                    q = guess.copy()
                    q[side[e], c] += sgn * h
                    ee, _, _ = go.linearize(q, ea[e:e + 1], eb[e:e + 1], z[e:e + 1], w[e:e + 1])
                    num[e] += sgn * ee[0]
            num /= 2 * h
            self_loop = ea == eb
            assert np.abs(num[~self_loop] - J[~self_loop, :, c]).max() < 1e-6


def test_gn_measurements_of_a_consistent_graph_have_zero_chi2():
    """PoseGraph(poses) + exact ICP-convention loop edges (X_a = X_b T): after
    optimize_pose_graph's conversion every residual vanishes at the initial
    poses, so GN would leave them unchanged (CPU: the oracle's chi2)."""
    import src.pose_graph as pgm
    import src.pose_graph_optimization as pgo
    from slamhip import se2, synthetic
    s = synthetic.make_loop_sequence(400, seed=3, n_beams=31)
    pg = pgm.PoseGraph(s.truth.copy())
    for a, b in s.loop_pairs:
        T = np.linalg.inv(se2.pose_to_mat(s.truth[b])) @ se2.pose_to_mat(s.truth[a])   # X_a = X_b T
        pg.add_constraint(int(a), int(b), T)
    ea, eb, z = pgo.gn_measurements(pg)
    _, _, _, chi2 = go.build_system(s.truth.copy(), ea.astype(np.int64), eb.astype(np.int64),
                                    go.edge_measurements(z), go.information(ea, eb))
    assert chi2 < 1e-20
    # the raw (unconverted) edges are NOT consistent once headings turn
    ra, rb, rtf = pg.edge_arrays()
    _, _, _, chi2_raw = go.build_system(s.truth.copy(), ra.astype(np.int64), rb.astype(np.int64),
                                        go.edge_measurements(rtf), go.information(ra, rb))
    assert chi2_raw > 1.0
    # after a pickle round trip the headings come from the saved poses: same z
    q = pgm.PoseGraph(None)
    q.poses, q.graph = pg.poses, pg.graph
    assert np.allclose(pgo.gn_measurements(q)[2], z, atol=1e-15)


def test_gn_measurements_follow_recorded_conventions(tmp_path):
    """Each constraint is converted by the convention recorded when it was
    added: "icp" (X_a = X_b T, the manual / image closures), "relative"
    (X_b = X_a T, detect_proximity's icp(pc_j, pc_i)), an overwritten
    constructor edge stops being a global delta, and the annotations survive
    the reference's (poses, DiGraph) pickle: chi2 = 0 at the true poses."""
    import src.pose_graph as pgm
    import src.pose_graph_optimization as pgo
    from slamhip import se2, synthetic
    s = synthetic.make_loop_sequence(400, seed=3, n_beams=31)
    X = [se2.pose_to_mat(p) for p in s.truth]
    pg = pgm.PoseGraph(s.truth.copy())
    for k, (a, b) in enumerate(s.loop_pairs):
        a, b = int(a), int(b)
        if k % 2:
            pg.add_constraint(a, b, np.linalg.inv(X[b]) @ X[a], convention="icp")
        else:
            pg.add_constraint(a, b, np.linalg.inv(X[a]) @ X[b], convention="relative")
    pg.add_constraint(7, 8, np.linalg.inv(X[7]) @ X[8], convention="relative")   # overwrites a constructor edge

    def chi2(g):
        ea, eb, z = pgo.gn_measurements(g)
        return go.build_system(s.truth.copy(), ea.astype(np.int64), eb.astype(np.int64),
                               go.edge_measurements(z), go.information(ea, eb))[3]
    assert chi2(pg) < 1e-20
    f = str(tmp_path / "g.pickle")
    pg.save(f)
    q = pgm.PoseGraph(None)
    q.load(f)
    assert chi2(q) < 1e-20
    # the default for unrecorded constraints is loop_edges ("icp"): the relative ones are then wrong
    r = pgm.PoseGraph(s.truth.copy())
    for a, b in s.loop_pairs[:4]:
        r.add_constraint(int(a), int(b), np.linalg.inv(X[int(a)]) @ X[int(b)])
    ea, eb, z = pgo.gn_measurements(r, loop_edges="relative")
    assert go.build_system(s.truth.copy(), ea.astype(np.int64), eb.astype(np.int64), go.edge_measurements(z),
                           go.information(ea, eb))[3] < 1e-20
    with pytest.raises(ValueError):
        pg.add_constraint(0, 5, np.eye(3), convention="global")


def test_unannotated_pickle_plus_annotated_closures(tmp_path):
    """A graph pickled without annotations (the reference's own PoseGraph, or
    this repo before the annotations) that then gets closures added with a
    convention (scripts/main_batched.py: load, then manual closures): the
    shape rule is applied PER EDGE, so its (a, a+1) edges stay constructor
    deltas and chi2 = 0 at the true poses.  A constraint added on an (a, a+1)
    edge without a convention is NOT a delta (it follows loop_edges)."""
    import pickle

    import networkx as nx

    import src.pose_graph as pgm
    import src.pose_graph_optimization as pgo
    from slamhip import se2, synthetic
    s = synthetic.make_loop_sequence(400, seed=3, n_beams=31)
    X = [se2.pose_to_mat(p) for p in s.truth]
    g = nx.DiGraph()   # the reference's constructor (src/pose_graph.py:32-36): "object" only
    g.add_edges_from((i, i + 1, {"object": se2.odom_change_to_mat(s.truth[i + 1] - s.truth[i])})
                     for i in range(len(s.truth) - 1))
    f = str(tmp_path / "ref.pickle")
    with open(f, "wb") as fh:
        pickle.dump((s.truth.copy(), g), fh)
    q = pgm.PoseGraph(None)
    q.load(f)
    for a, b in s.loop_pairs:
        a, b = int(a), int(b)
        q.add_constraint(a, b, np.linalg.inv(X[b]) @ X[a], convention="icp")

    def chi2(gr, **kw):
        ea, eb, z = pgo.gn_measurements(gr, **kw)
        return go.build_system(s.truth.copy(), ea.astype(np.int64), eb.astype(np.int64),
                               go.edge_measurements(z), go.information(ea, eb))[3]
    assert chi2(q) < 1e-20
    # a convention-less constraint on (a, a+1): a relative measurement under loop_edges="relative"
    q.add_constraint(10, 11, np.linalg.inv(X[10]) @ X[11])
    assert chi2(q, loop_edges="relative") < 1e-20
    assert chi2(q, loop_edges="icp") > 1e-8


def test_older_pickle_bare_constraint_in_annotated_graph_warns(tmp_path):
    """An older pickle of this build: constructor edges annotated with their
    headings, and an add_constraint (a, a+1) edge saved before the
    ``constraint`` flag existed (heading popped, no convention).  The shape
    rule does not apply in a graph that carries headings: the bare edge
    follows loop_edges, with a warning."""
    import warnings

    import src.pose_graph as pgm
    import src.pose_graph_optimization as pgo
    from slamhip import se2, synthetic
    s = synthetic.make_loop_sequence(200, seed=5, n_beams=31)
    X = [se2.pose_to_mat(p) for p in s.truth]
    q = pgm.PoseGraph(s.truth.copy())
    q.add_constraint(20, 21, np.linalg.inv(X[20]) @ X[21])    # relative: X_21 = X_20 T
    del q.graph.edges[20, 21]["constraint"]                   # as an older pickle stored it
    q._flat = None

    def chi2(**kw):
        ea, eb, z = pgo.gn_measurements(q, **kw)
        return go.build_system(s.truth.copy(), ea.astype(np.int64), eb.astype(np.int64),
                               go.edge_measurements(z), go.information(ea, eb))[3]
    with pytest.warns(UserWarning, match="unannotated"):
        assert chi2(loop_edges="relative") < 1e-20
    with pytest.warns(UserWarning):
        assert chi2(loop_edges="icp") > 1e-8
    # a fully unannotated graph: no warning, the shape rule
    for _, _, d in q.graph.edges(data=True):
        d.pop("heading", None)
    q._flat = None
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        pgo.gn_measurements(q)


def test_edge_arrays_cache_invalidate():
    """Edits that keep the edge count are not seen by the cache;
    PoseGraph.invalidate() drops it (and the drop-in SGD solver keyed on it)."""
    import src.pose_graph as pgm
    poses = np.c_[np.arange(6.0), np.zeros(6), np.zeros(6)]
    pg = pgm.PoseGraph(poses)
    a = pg.edge_arrays()
    pg.graph[1][2]["object"] = 2 * np.eye(3)
    assert pg.edge_arrays() is a
    pg._sgd_solver = ("stale", None)
    pg.invalidate()
    b = pg.edge_arrays()
    assert b is not a and np.array_equal(b[2][1], 2 * np.eye(3))
    assert not hasattr(pg, "_sgd_solver")


def test_edge_arrays_cache_follows_the_graph():
    """PoseGraph.edge_arrays() is cached between SGD calls and rebuilt after
    add_constraint / flip / load or a direct change of the graph."""
    import src.pose_graph as pgm
    poses = np.c_[np.arange(6.0), np.zeros(6), np.zeros(6)]
    pg = pgm.PoseGraph(poses)
    a = pg.edge_arrays()
    assert pg.edge_arrays() is a and not a[2].flags.writeable
    pg.add_constraint(0, 4, np.eye(3))
    b = pg.edge_arrays()
    assert b is not a and len(b[0]) == 6
    pg.graph.add_edge(1, 5, object=np.eye(3))    # behind the class's back
    assert len(pg.edge_arrays()[0]) == 7
    c = pg.edge_arrays()
    pg.flip()
    d = pg.edge_arrays()
    assert d is not c and sorted(zip(d[0].tolist(), d[1].tolist())) == sorted((5 - b, 5 - a) for a, b in
                                                                             zip(c[0].tolist(), c[1].tolist()))


@pytest.mark.gpu
def test_detect_proximity_edges_feed_gn_consistently():
    """detect_proximity (icp(pc_j, pc_i), X_j = X_i T) followed by
    gn_measurements: at the true poses the loop residuals are ICP-accurate
    (cm) — the inverted reading of the same edges is off by twice the pairs'
    offsets (laps ~0.3 m apart)."""
    import src.loop_closure_detection as lcd
    import src.pose_graph as pgm
    import src.pose_graph_optimization as pgo
    from slamhip import synthetic
    # laps 0.3 m apart (lap_jitter): the proximity pairs' offsets dwarf ICP's cm errors
    s = synthetic.make_loop_sequence(1200, seed=3, n_beams=361, lap_jitter=0.3)   # pairs ~0.3 m apart
    pg = pgm.PoseGraph(s.truth.copy())
    lcd.detect_proximity(pg, s.scans, min_dist_along_path=2, max_dist=1, err_thresh=110)
    ea, eb, z = pgo.gn_measurements(pg)
    loop = eb != ea + 1
    assert loop.sum() > 3
    def loop_res(zz):
        e, _, _ = go.linearize(s.truth.copy(), ea.astype(np.int64), eb.astype(np.int64), go.edge_measurements(zz),
                               go.information(ea, eb))
        return np.hypot(e[loop][:, 0], e[loop][:, 1])
    inv = z.copy()
    inv[loop] = np.linalg.inv(z[loop])
    good, bad = loop_res(z), loop_res(inv)
    assert np.median(good) < 0.03 and np.median(bad) > 5 * np.median(good), (np.median(good), np.median(bad))
    same = pgo.gn_measurements(pg, loop_edges="icp")[2]   # unchanged: the edges carry their convention
    assert np.array_equal(same, z)


@pytest.mark.gpu
def test_pipeline_gn_reduces_drift():
    """The batched driver's GN path (scan matching -> PoseGraph -> manual loop
    closures -> optimize(method="gn")) on a loop sequence: the optimised
    trajectory is closer to the ground truth than the ICP chain, and GN on the
    unchanged chain graph (no loop edges) leaves it where it is."""
    import src.pose_graph as pgm
    from slamhip import pipeline, synthetic
    s = synthetic.make_loop_sequence(1200, seed=6)
    r = pipeline.scan_matching(s.odometry, s.scans)
    # no loop edges: the converted odometry edges are consistent -> no motion
    pg0 = pgm.PoseGraph(r.poses.copy())
    chis = __import__("src.pose_graph_optimization", fromlist=["x"]).optimize_pose_graph(
        pg0, iterations=2, return_history=True)
    assert chis[0] < 1e-12 and np.abs(pg0.poses[:, :2] - r.poses[:, :2]).max() < 1e-9
    pg = pgm.PoseGraph(r.poses.copy())
    ok = pipeline.manual_loop_closures(pg, s.scans, s.loop_pairs)
    assert ok.mean() > 0.8
    pipeline.optimize(pg, s.scans, method="gn", gn_iterations=5)

    def ate(p):   # position error after aligning the first pose (the chain starts at odometry[0])
        return float(np.sqrt(np.mean(np.sum((p[:, :2] - s.truth[:, :2]) ** 2, axis=1))))
    assert ate(pg.poses) < 0.7 * ate(r.poses)


def test_plan_cache_keys_on_structure():
    """optimize_pose_graph re-uses the symbolic plan of an identical structure
    and never the plan of a different one."""
    from slamhip import gn
    ea = np.array([0, 1, 2, 0], np.int32)
    eb = np.array([1, 2, 3, 3], np.int32)
    p1 = gn.plan_for(4, ea, eb)
    assert gn.plan_for(4, ea.copy(), eb.copy()) is p1
    p2 = gn.plan_for(4, ea, np.array([1, 2, 3, 2], np.int32))
    assert p2 is not p1 and p2.n_slots != p1.n_slots or not np.array_equal(p2.slot_items, p1.slot_items)
    assert gn.plan_for(5, ea, eb) is not p1


def _loop_plan_slots(N, ea, eb, node_col, order):
    """The per-edge loop construction of the H slot lists (the plan's original
    form), kept as the reference for the vectorised one."""
    diag_items = [[] for _ in range(N)]
    pair_items = {}
    for e in range(len(ea)):
        a, b = int(ea[e]), int(eb[e])
        if a == b:
            continue
        if node_col[a] >= 0:
            diag_items[a].append(2 * e)
        if node_col[b] >= 0:
            diag_items[b].append(2 * e + 1)
        if node_col[a] >= 0 and node_col[b] >= 0:
            row, col = (a, b) if node_col[a] > node_col[b] else (b, a)
            pair_items.setdefault((row, col), []).append(2 * e + (0 if row == a else 1))
    rc, ptr, items = [], [0], []
    for n in order:
        rc.append((node_col[n], node_col[n]))
        items.extend(diag_items[n])
        ptr.append(len(items))
    for (row, col), its in pair_items.items():
        rc.append((node_col[row], node_col[col]))
        items.extend(its)
        ptr.append(len(items))
    return np.asarray(rc).reshape(-1, 2), np.asarray(ptr), np.asarray(items if items else [0])


@pytest.mark.parametrize("case", ["c4", "random", "selfloops"])
def test_plan_matches_loop_construction(case):
    """The vectorised symbolic plan lists the same slots and the same items in
    the same order as the per-edge loop (the assembly's summation order)."""
    from slamhip import gn, synthetic
    rng = np.random.default_rng(3)
    if case == "c4":
        guess, ea, eb, _, _ = synthetic.lap_graph_c4()
        N, fixed = len(guess), 0
    else:
        N = 300
        ea = np.r_[np.arange(N - 1), rng.integers(0, N, 500)]
        eb = np.r_[np.arange(1, N), rng.integers(0, N, 500)]
        if case == "selfloops":
            ea[::37] = eb[::37]          # self-loops, and repeated pairs below
            ea = np.r_[ea, ea[:40]]
            eb = np.r_[eb, eb[:40]]
        fixed = 7
    p = gn.GnPlan(N, ea, eb, fixed)
    order = np.argsort(np.where(p.node_col >= 0, p.node_col, np.iinfo(np.int32).max), kind="stable")[:p.nv // 3]
    rc, ptr, items = _loop_plan_slots(N, np.asarray(ea), np.asarray(eb), p.node_col, order)
    assert np.array_equal(p.slot_rc, rc) and np.array_equal(p.slot_ptr, ptr) and np.array_equal(p.slot_items, items)


def test_plan_without_edges():
    """A graph without edges (one pose, or poses not yet linked) plans: the
    band order's early exit returns its width too."""
    from slamhip import gn
    p = gn.GnPlan(1, [], [])
    assert p.nv == 0 and p.n_slots == 0
    q = gn.GnPlan(4, np.zeros(0, np.int64), np.zeros(0, np.int64), allow_border=True)
    assert q.nv == 9 and q.W == 2 and q.nv == q.nv_band
    order, name, w = gn.band_order(4, [], [])
    assert sorted(order.tolist()) == [0, 1, 2, 3] and w == 2


def test_plan_border_gated_by_solver_mode():
    """Under slam_gn_set_solver(1) (band Cholesky, no border) the default plan
    has no border; mode 0 restores the bordered C4 plan."""
    from slamhip import _abi, gn, synthetic
    lib = _abi.lib()
    guess, ea, eb, tf, _ = synthetic.lap_graph_c4()
    try:
        assert lib.slam_gn_set_solver(1) == 0 and lib.slam_gn_get_solver() == 1
        p1 = gn.plan_for(len(guess), ea, eb)
        assert p1.nv == p1.nv_band
    finally:
        lib.slam_gn_set_solver(0)
    p0 = gn.plan_for(len(guess), ea, eb)
    assert p0.nv - p0.nv_band == 27 and p0 is not p1


def _bcr_schur_numpy(D, E, b, y, C, rb, nb):
    """The Schur-accumulating bordered block cyclic reduction restated in NumPy
    (eager updates; csrc/gn_bcr_gj.hip applies the same ones one level late):
    returns (x_band, x_border, blocks whose reduced border rows were nonzero
    at their elimination, in elimination order)."""
    D = [d.copy() for d in D]
    A = {}                       # couplings A[j, i] (row block j, column block i), both directions
    for i in range(nb - 1):
        A[(i + 1, i)] = E[i].copy()
        A[(i, i + 1)] = E[i].T.copy()
    R = [np.c_[b[i], y[i]] for i in range(nb)]   # [b_i | y_i]
    S = C.copy()
    s_ = rb.copy()
    elim, zs, Xs, Ys, coupled = [], {}, {}, {}, []
    s = 1
    while s < nb:
        for i in range(s, nb, 2 * s):
            p, n = i - s, i + s
            G = np.linalg.inv(D[i])
            z = G @ R[i]
            P = R[i].T @ z
            if np.any(R[i][:, 1:] != 0):
                coupled.append(i)
            S -= P[1:, 1:]
            s_ -= P[1:, 0]
            zs[i] = z
            Xs[i] = G @ A[(i, p)]
            D[p] -= A[(p, i)] @ Xs[i]
            R[p] = R[p] - A[(p, i)] @ z
            if n < nb:
                Ys[i] = G @ A[(i, n)]
                D[n] -= A[(n, i)] @ Ys[i]
                R[n] = R[n] - A[(n, i)] @ z
                A[(n, p)] = -A[(n, i)] @ Xs[i]
                A[(p, n)] = A[(n, p)].T
            elim.append((s, i))
        s *= 2
    G0 = np.linalg.inv(D[0])
    X0 = G0 @ R[0]
    P0 = R[0].T @ X0
    S -= P0[1:, 1:]
    s_ -= P0[1:, 0]
    xb = np.linalg.solve(S, s_)
    x = {0: X0[:, 0] - X0[:, 1:] @ xb}
    for (s, i) in reversed(elim):
        p, n = i - s, i + s
        v = zs[i][:, 0] - zs[i][:, 1:] @ xb - Xs[i] @ x[p]
        if n < nb:
            v = v - Ys[i] @ x[n]
        x[i] = v
    return np.concatenate([x[i] for i in range(nb)]), xb, coupled


@pytest.mark.parametrize("nb,wb,nbd,seed", [(13, 4, 5, 0), (32, 3, 7, 1), (47, 2, 3, 2)])
def test_schur_slots_match_a_numeric_reduction(nb, wb, nbd, seed):
    """The symbolic list of border-coupled blocks (gn.schur_slots) equals the
    blocks whose reduced border rows are nonzero in a numeric run of the
    Schur-accumulating cyclic reduction, and that reduction (Schur complement
    summed over the eliminated blocks, one-column back-substitution) solves
    the bordered system: against np.linalg.solve at 1e-9."""
    from unittest import mock

    from slamhip import gn
    rng = np.random.default_rng(seed)
    n = nb * wb
    D = [np.eye(wb) * 6 + (lambda m: m + m.T)(rng.normal(0, 0.3, (wb, wb))) for _ in range(nb)]
    E = [rng.normal(0, 0.5, (wb, wb)) for _ in range(nb - 1)]
    rows = np.r_[np.arange(wb + 1), np.arange(n - wb - 2, n)]   # the band's two ends couple to the border
    Bm = np.zeros((n, nbd))
    Bm[rows] = rng.normal(0, 0.4, (len(rows), nbd))
    C = np.eye(nbd) * 8 + (lambda m: m + m.T)(rng.normal(0, 0.2, (nbd, nbd)))
    H = np.zeros((n + nbd, n + nbd))
    for i in range(nb):
        H[i * wb:(i + 1) * wb, i * wb:(i + 1) * wb] = D[i]
    for i in range(nb - 1):
        H[(i + 1) * wb:(i + 2) * wb, i * wb:(i + 1) * wb] = E[i]
        H[i * wb:(i + 1) * wb, (i + 1) * wb:(i + 2) * wb] = E[i].T
    H[:n, n:] = Bm
    H[n:, :n] = Bm.T
    H[n:, n:] = C
    rhs = rng.normal(0, 1, n + nbd)
    want = np.linalg.solve(H, rhs)
    b = [rhs[i * wb:(i + 1) * wb] for i in range(nb)]
    y = [Bm[i * wb:(i + 1) * wb] for i in range(nb)]
    xa, xb, coupled = _bcr_schur_numpy(D, E, b, y, C, rhs[n:], nb)
    assert np.abs(np.r_[xa, xb] - want).max() <= 1e-9 * max(1.0, np.abs(want).max())

    class FakeLib:
        def slam_gn_bcr_block_rows(self, nv, W):
            return wb

        def slam_gn_schur_supported(self):
            return 1
    with mock.patch.object(gn._abi, "lib", lambda: FakeLib()):
        pslot, blocks = gn.schur_slots(rows.astype(np.int32), n, wb)
    assert blocks.tolist() == coupled
    assert (pslot >= 0).sum() == len(coupled) and pslot[blocks].tolist() == list(range(len(blocks)))


def test_c4_schur_plan_couples_few_blocks():
    """C4's bordered plan: the border couples the band's two ends only, so six
    eliminated blocks (one per level the last block's coupling climbs) carry
    a Schur contribution, plus the top block."""
    from slamhip import gn, synthetic
    guess, ea, eb, tf, _ = synthetic.lap_graph_c4()
    p = gn.GnPlan(len(guess), ea, eb)
    assert p.nv - p.nv_band == 27 and p.pslot is not None
    assert p.schur_blocks.tolist() == [467, 466, 464, 448, 384, 256]
