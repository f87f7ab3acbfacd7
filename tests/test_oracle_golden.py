"""Pin the CPU oracle (oracle/icp_oracle.py, oracle/pgo_oracle.py) against the
golden vectors produced by the reference itself (tests/golden/gen_golden.py).

NumPy restatements must match BIT FOR BIT on the machine that generated the
fixtures (same NumPy/OpenBLAS); on other hosts the BLAS/libm rounding may
differ, so the comparison falls back to tight tolerances there.
"""
import numpy as np
import pytest

import icp_oracle as io
import pgo_oracle as po
from conftest import case_arrays


def _eq(a, b, tol):
    a, b = np.asarray(a), np.asarray(b)
    if np.array_equal(a, b):
        return True
    return np.allclose(a, b, rtol=0, atol=tol)


def test_unit_vectors_bitexact(golden):
    u = golden("icp_unit.npz")
    for k in range(int(u["n_cases"])):
        pc1, pc2 = u[f"pc1_{k}"], u[f"pc2_{k}"]
        corr = io.correspondences(pc1, pc2)
        assert np.array_equal(corr, u[f"corr_{k}"])
        assert _eq(io.kabsch(pc1, pc2[corr]), u[f"tf_{k}"], 1e-12)
        assert _eq(io.sq_error(pc1, pc2[corr]), u[f"err_{k}"], 1e-12)
        T, c1, e1 = io.icp_iteration(pc1, pc2, u[f"init_{k}"].copy())
        assert np.array_equal(c1, u[f"it_corr_{k}"])
        assert _eq(T, u[f"it_T_{k}"], 1e-12)
        assert _eq(e1, u[f"it_err_{k}"], 1e-12)


def test_loop_mode_matches_vectorised(golden):
    u = golden("icp_unit.npz")
    pc1, pc2 = u["pc1_3"], u["pc2_3"]
    assert np.array_equal(io.correspondences_loop(pc1, pc2), io.correspondences(pc1, pc2))


def test_tie_rule_first_index(golden):
    u = golden("icp_unit.npz")
    pc2 = u["pc2_3"]
    q = pc2[17:18].copy()   # duplicates at rows 5, 17, 200 -> first index 5
    assert io.correspondences(q, pc2)[0] == 5


@pytest.mark.parametrize("k", range(12))
def test_icp_cases_bitexact(golden, k):
    g = golden("icp_cases.npz")
    pc1, pc2, init, eps, mi, st, ro, hist, err = case_arrays(g, k)
    tfs, e = io.icp(pc1, pc2, init, eps, mi, st, ro)
    assert len(tfs) == len(hist)
    assert _eq(np.stack(tfs), hist, 1e-10)
    assert _eq(e, err, 1e-10)
    assert np.array_equal(init, g["init_after"][k])   # rotation_only mutation
    c0 = g["corr0"][g["corr0_off"][k]:g["corr0_off"][k + 1]]
    _, c, _ = io.icp_iteration(pc1, pc2, g["init"][k].copy(), ro)
    assert np.array_equal(c, c0)


def test_max_iters_rule(golden):
    g = golden("icp_cases.npz")
    labels = list(g["labels"])
    k = labels.index("max_iters")
    assert int(g["n_iter"][k]) == int(g["params"][k][1]) + 2   # at most max_iters + 2


def test_sgd_restatement(golden):
    s = golden("sgd.npz")
    poses = s["poses0"].copy()
    edges = (s["ea"], s["eb"], s["tf"])
    for k in range(20):
        po.sgd_step(poses, *edges, learning_rate=1 / float(k + 1))
        if k + 1 in (1, 5, 20):
            ref = s[f"poses_step{k + 1}"]
            assert np.allclose(poses[:, :2], ref[:, :2], rtol=0, atol=1e-9)
            assert np.allclose(po.wrap(poses[:, 2] - ref[:, 2]), 0, atol=1e-9)
    po.orient_from_positions(poses)
    assert np.allclose(poses, s["poses_recomputed"], rtol=0, atol=1e-9)


def test_sgd_flip_run(golden):
    s = golden("sgd.npz")
    pg = po.FlatGraph(s["poses0"].copy(), s["ea"], s["eb"], s["tf"])
    for it in range(1, 11):
        if it % 5 == 0:
            pg.flip()
        po.sgd_step(pg.poses, pg.ea, pg.eb, pg.tf)
    assert np.array_equal(pg.ea, s["flip_ea"]) and np.array_equal(pg.eb, s["flip_eb"])
    assert np.allclose(pg.poses[:, :2], s["poses_flip10"][:, :2], rtol=0, atol=1e-9)


def test_orientation_icp_recompute(golden):
    s = golden("sgd.npz")
    off = s["rc_off"]
    scans = [s["rc_scans"][off[i]:off[i + 1]] for i in range(len(off) - 1)]
    poses = s["rc_poses0"].copy()
    po.recompute_orientation(poses, scans, 100, 0.05, icp_recompute=True, icp_fn=io.icp)
    assert np.allclose(poses, s["rc_poses"], rtol=0, atol=1e-12)
