"""Gauss-Newton SE(2) pose-graph optimisation on the GPU.

Host side of ``slam_gn_iteration_f64`` (csrc/gn_kernels.hip).  The symbolic
work is done once per graph STRUCTURE (it does not change across iterations):

1. node ordering: reverse Cuthill-McKee over the node adjacency (SciPy) or
   the place-major order (``place_order``), whichever band is narrower, the
   gauge node removed; node n owns scalar columns node_col[n] .. +2 of H;
2. half-bandwidth W (scalars) of H in that order;
3. H block slots: one per free node (diagonal block) and one per connected
   free node pair (off-diagonal block of the lower band), each with the list
   of edge contributions it sums, in edge order (deterministic assembly).

Everything per iteration runs on the device: linearisation, assembly, band
Cholesky, substitution, pose update.  Problem definition (residual, Jacobians,
information 2 I / 5 I as src/pose_graph.py:61-73 exports them) is documented
in csrc/gn_kernels.hip and oracle/gn_oracle.py.
"""
import os
import time

import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import connected_components, reverse_cuthill_mckee

from . import _abi
from . import device as dv

ODOM_INFO = 2.0
LOOP_INFO = 5.0


def _band_w(order, ea, eb, N, fixed):
    order = order[order != fixed]
    rank = np.full(N, -1, dtype=np.int64)
    rank[order] = np.arange(len(order))
    ra, rb = rank[ea], rank[eb]
    ok = (ra >= 0) & (rb >= 0)
    return int(3 * np.abs(ra[ok] - rb[ok]).max() + 2) if ok.any() else 2


def place_order(N, ea, eb):
    """Place-major node order for trajectory graphs (lap structure).

    A pose graph from scripts/main.py is an odometry chain (edges i -> i+1)
    plus loop closures between poses that revisit a place.  The connected
    components of the loop-closure edges alone are the places (C4: 500 places
    of the 10 laps' poses); the chain links consecutive places.  Reverse
    Cuthill-McKee over that place graph, with every place's poses kept together
    in pose order, puts a lap edge (p, lap) -> (p + 1, lap) two places apart
    even where RCM over the poses folds the loop unevenly: C4's band is 62
    scalars instead of RCM's 77 (BCR blocks of 64 rows instead of 80)."""
    nc, lab, Q = _places(N, ea, eb)
    return _place_major(N, lab, Q, np.ones(nc, dtype=bool))


def _places(N, ea, eb):
    """Places (components of the loop-closure edges) and the place graph."""
    loop = np.abs(eb - ea) != 1
    L = sp.coo_matrix((np.ones(int(loop.sum())), (ea[loop], eb[loop])), shape=(N, N))
    nc, lab = connected_components(L, directed=False)
    ca, cb = lab[ea], lab[eb]
    x = ca != cb
    Q = sp.coo_matrix((np.ones(2 * int(x.sum()) + nc), (np.r_[ca[x], cb[x], np.arange(nc)],
                                                         np.r_[cb[x], ca[x], np.arange(nc)])), shape=(nc, nc)).tocsr()
    return nc, lab, Q


def _place_major(N, lab, Q, keep):
    """Poses of the kept places, place-major in RCM order of the kept place graph."""
    idx = np.flatnonzero(keep)
    qo = idx[reverse_cuthill_mckee(Q[idx][:, idx].tocsr(), symmetric_mode=True)]
    qr = np.full(len(keep), -1, dtype=np.int64)
    qr[qo] = np.arange(len(qo))
    nodes = np.flatnonzero(qr[lab] >= 0)
    return nodes[np.lexsort((nodes, qr[lab[nodes]]))]


MAX_BORDER = 31   # scalars (csrc/gn_kernels.hip kGnBorderMax)
BCR_MAX_WB = 96   # widest cyclic-reduction block (csrc/gn_bcr.hip kBcrMaxWb); a border needs that solver


def border_order(N, ea, eb, fixed=0):
    """Band + border order for loop trajectories (C4: ten laps of one square).

    The place graph of a lap trajectory is a ring, and any order of a ring
    folds it (place_order: two places per band step, C4 W = 62).  Taking one
    place's poses out as a border cuts the ring into a path of places, whose
    place-major order has a band of one place (C4: W = 32, BCR blocks of 32
    rows); the border (<= MAX_BORDER scalars) is eliminated by a Schur
    complement after the band solve (slam_gn_iteration_bordered_f64).  The
    candidates are the place holding the fixed node and places spread along
    the ring; returns (order of the band nodes, border nodes, W) of the
    narrowest band, or None."""
    ea = np.asarray(ea, dtype=np.int64)
    eb = np.asarray(eb, dtype=np.int64)
    if len(ea) == 0:
        return None
    nc, lab, Q = _places(N, ea, eb)
    ring = reverse_cuthill_mckee(Q, symmetric_mode=True)
    cands = [int(lab[fixed])] + [int(ring[int(f * (nc - 1))]) for f in (0.0, 0.25, 0.5, 0.75)]
    best = None
    for c in dict.fromkeys(cands):
        bnodes = np.flatnonzero((lab == c) & (np.arange(N) != fixed))
        if len(bnodes) == 0 or 3 * len(bnodes) > MAX_BORDER:
            continue
        keep = np.ones(nc, dtype=bool)
        keep[c] = False
        if not keep.any():
            continue
        band = _place_major(N, lab, Q, keep)
        w = _band_w(band, ea, eb, N, fixed)
        if best is None or w < best[2]:
            best = (band, bnodes, w)
    return best


def band_order(N, ea, eb, fixed=0):
    """Node order for the band solvers: reverse Cuthill-McKee over the poses
    or the place-major order (place_order), whichever gives the narrower band
    (the BCR cost grows with the band rounded up to 16 rows).  Returns
    (order, name, W)."""
    ea = np.asarray(ea, dtype=np.int64)
    eb = np.asarray(eb, dtype=np.int64)
    adj = sp.coo_matrix((np.ones(2 * len(ea) + N), (np.r_[ea, eb, np.arange(N)], np.r_[eb, ea, np.arange(N)])),
                        shape=(N, N)).tocsr()
    best = (reverse_cuthill_mckee(adj, symmetric_mode=True), "rcm")
    w_best = _band_w(best[0], ea, eb, N, fixed)
    if len(ea) == 0:
        return best + (w_best,)
    po = place_order(N, ea, eb)
    w = _band_w(po, ea, eb, N, fixed)
    if (w + 15) // 16 < (w_best + 15) // 16 or ((w + 15) // 16 == (w_best + 15) // 16 and w < w_best):
        best = (po, "place-major")
        w_best = w
    return best + (w_best,)


class GnPlan:
    """Symbolic analysis of one graph structure."""

    def __init__(self, N, ea, eb, fixed=0, order=None, border=None, allow_border=None):
        """order: node order of the band (default: band_order); border: nodes
        solved as a dense border after the band (default: border_order when
        its band needs fewer 16-row blocks than the unbordered one; [] none).
        allow_border (default: unless slam_gn_set_solver(1) forces the band
        Cholesky, which takes no border) gates the default border."""
        ea = np.asarray(ea, dtype=np.int64)
        eb = np.asarray(eb, dtype=np.int64)
        self.N = N
        self.fixed = fixed
        if allow_border is None:
            allow_border = _border_allowed()
        if order is None and border is None and not allow_border:
            order, self.ordering, _ = band_order(N, ea, eb, fixed)
        elif order is None and border is None:
            order, self.ordering, w0 = band_order(N, ea, eb, fixed)
            bo = border_order(N, ea, eb, fixed)
            wb = (bo[2] + 15) // 16 * 16 if bo is not None else 0
            if bo is not None and wb < (w0 + 15) // 16 * 16 and wb <= BCR_MAX_WB and \
                    (3 * N - 3 - 3 * len(bo[1])) // wb >= 4:
                order, border, self.ordering = bo[0], bo[1], "place-major + border"
        elif order is None:
            bset = np.zeros(N, dtype=bool)
            bset[np.asarray(border, dtype=np.int64)] = True
            keep = np.flatnonzero(~bset)
            sub = np.flatnonzero(np.isin(ea, keep) & np.isin(eb, keep))
            remap = np.full(N, -1, dtype=np.int64)
            remap[keep] = np.arange(len(keep))
            o, self.ordering, _ = band_order(len(keep), remap[ea[sub]], remap[eb[sub]], -1)
            order = keep[o]
            self.ordering += " + given border"
        else:
            self.ordering = "given"
        border = np.asarray([] if border is None else border, dtype=np.int64)
        border = border[border != fixed]
        order = np.asarray(order, dtype=np.int64)
        order = order[(order != fixed) & ~np.isin(order, border)]
        if 3 * len(border) > MAX_BORDER:
            raise ValueError(f"border of {3 * len(border)} scalars (at most {MAX_BORDER})")
        node_col = np.full(N, -1, dtype=np.int32)
        node_col[order] = 3 * np.arange(len(order), dtype=np.int32)
        node_col[border] = 3 * (len(order) + np.arange(len(border), dtype=np.int32))
        self.node_col = node_col
        self.nv = 3 * (len(order) + len(border))
        self.nv_band = 3 * len(order)
        ca, cb = node_col[ea], node_col[eb]
        both = (ca >= 0) & (cb >= 0) & (ca < self.nv_band) & (cb < self.nv_band)
        self.W = int(max(2, (np.abs(ca[both] - cb[both]).max() + 2) if both.any() else 2))
        # band rows coupled to the border (B's nonzero rows)
        xb = (ca >= 0) & (cb >= 0) & ((ca >= self.nv_band) != (cb >= self.nv_band))
        bn = np.where(ca[xb] < self.nv_band, ca[xb], cb[xb])
        self.nbr_rows = np.unique((bn[:, None] + np.arange(3)[None, :]).ravel()).astype(np.int32)
        self.pslot = self.schur_blocks = None
        if self.nv_band < self.nv:
            self.pslot, self.schur_blocks = schur_slots(self.nbr_rows, self.nv_band, self.W)
        order = np.r_[order, border]   # every free node in column order (slots below)

        # diagonal slots: free node n (in RCM order), items 2e + side (a: 0, b: 1) in
        # edge order; pair slots: one per connected free pair (row = the node with
        # the larger column), in order of first appearance, items in edge order.
        # Vectorised; the slot and item order is the one the assembly sums in
        # (tests/test_gn.py::test_plan_matches_loop_construction).
        e = np.arange(len(ea), dtype=np.int64)
        ok = ea != eb                                   # a self-loop adds nothing to H
        rank = np.full(N, -1, dtype=np.int64)
        rank[order] = np.arange(len(order))
        fa, fb = ok & (node_col[ea] >= 0), ok & (node_col[eb] >= 0)
        dn = np.r_[ea[fa], eb[fb]]
        di = np.r_[2 * e[fa], 2 * e[fb] + 1]
        de = np.r_[e[fa], e[fb]]
        srt = np.lexsort((de, rank[dn]))
        diag_counts = np.bincount(rank[dn], minlength=len(order))
        both = fa & fb
        pa, pb, pe = ea[both], eb[both], e[both]
        a_row = node_col[pa] > node_col[pb]
        row = np.where(a_row, pa, pb)
        col = np.where(a_row, pb, pa)
        key = row.astype(np.int64) * N + col
        uk, first, inv = np.unique(key, return_index=True, return_inverse=True)
        prank = np.empty(len(uk), dtype=np.int64)
        prank[np.argsort(first, kind="stable")] = np.arange(len(uk))
        pr = prank[inv]
        psrt = np.lexsort((pe, pr))
        pitems = 2 * pe + np.where(a_row, 0, 1)
        prow = np.empty(len(uk), dtype=np.int64)
        pcol = np.empty(len(uk), dtype=np.int64)
        prow[pr] = row
        pcol[pr] = col
        rc = np.r_[np.stack([node_col[order], node_col[order]], 1).reshape(-1, 2),
                   np.stack([node_col[prow], node_col[pcol]], 1).reshape(-1, 2)]
        counts = np.r_[diag_counts, np.bincount(pr, minlength=len(uk))]
        items = np.r_[di[srt], pitems[psrt]]
        ptr = np.r_[0, np.cumsum(counts)]
        self.slot_rc = np.asarray(rc, dtype=np.int32).reshape(-1, 2)
        self.slot_ptr = np.asarray(ptr, dtype=np.int32)
        self.slot_items = np.asarray(items if len(items) else [0], dtype=np.int32)
        self.n_slots = len(rc)


def _border_allowed():
    """A default border needs the cyclic-reduction solver: not while the
    band Cholesky is forced (slam_gn_set_solver(1))."""
    try:
        return int(_abi.lib().slam_gn_get_solver()) != 1
    except (OSError, AttributeError):
        return True


MAX_SCHUR_SLOTS = 64   # more coupled blocks than this: the multi-column back-substitution path


def schur_slots(nbr_rows, nv_band, W):
    """The blocks whose reduced rows couple to the border during the block
    cyclic reduction, symbolically: a band block
    couples if it holds a row of nbr_rows; eliminating a coupled odd block i
    at level s (i = s, 3s, ...) passes the coupling to its neighbours i - s and
    i + s (the RHS update b_j -= A[j, i] z_i).  Every coupled block eliminated
    adds Y_i^T D_i^-1 Y_i to the border's Schur complement: returns (pslot, the
    list in elimination order) with pslot[i] = its slot, -1 elsewhere, or
    (None, None) when the cyclic reduction does not apply or the list exceeds
    MAX_SCHUR_SLOTS (slam_gn_iteration_bordered_f64 then)."""
    try:
        Wb = int(_abi.lib().slam_gn_bcr_block_rows(nv_band, W))
    except (OSError, ImportError, AttributeError):
        return None, None
    if Wb <= 0 or not os.environ.get("SLAMHIP_GN_SCHUR", "1") == "1":
        return None, None
    try:   # the solver this process runs must be the explicit-inverse reduction
        if not int(_abi.lib().slam_gn_schur_supported()):
            return None, None
    except AttributeError:
        return None, None
    nb = (nv_band + Wb - 1) // Wb
    nz = np.zeros(nb, dtype=bool)
    nz[np.asarray(nbr_rows, dtype=np.int64) // Wb] = True
    blocks = []
    s = 1
    while s < nb:
        for i in range(s, nb, 2 * s):
            if nz[i]:
                blocks.append(i)
                nz[i - s] = True
                if i + s < nb:
                    nz[i + s] = True
        s *= 2
    if len(blocks) > MAX_SCHUR_SLOTS:
        return None, None
    pslot = np.full(nb, -1, dtype=np.int32)
    pslot[blocks] = np.arange(len(blocks), dtype=np.int32)
    return pslot, np.asarray(blocks, dtype=np.int32)


_PLANS = {}   # structure -> GnPlan (a pipeline re-optimises the same graph structure)
# times the XCD-local back-substitution timed out and a run was repeated with
# a launch per level (process-wide; bench.py reports it)
FUSED_BACK_FALLBACKS = 0


def plan_for(N, ea, eb, fixed=0):
    """The GnPlan of a graph structure, cached: the symbolic analysis (RCM
    order, band width, slot lists) depends only on (N, edge endpoints, fixed)."""
    ea = np.ascontiguousarray(ea, dtype=np.int32)
    eb = np.ascontiguousarray(eb, dtype=np.int32)
    allow = _border_allowed()
    key = (int(N), int(fixed), allow, ea.tobytes(), eb.tobytes())
    p = _PLANS.get(key)
    if p is None:
        if len(_PLANS) >= 8:
            _PLANS.pop(next(iter(_PLANS)))
        p = _PLANS[key] = GnPlan(N, ea, eb, fixed, allow_border=allow)
    return p


class GaussNewton:
    def __init__(self, poses, ea, eb, tf, odom_information=ODOM_INFO, loop_information=LOOP_INFO, fixed=0,
                 device=None, plan=None):
        poses = np.ascontiguousarray(poses, dtype=np.float64)
        ea = np.asarray(ea, dtype=np.int32)
        eb = np.asarray(eb, dtype=np.int32)
        self.N, self.E = len(poses), len(ea)
        self.plan = plan if plan is not None else plan_for(self.N, ea, eb, fixed)
        w = np.where(np.abs(eb.astype(np.int64) - ea) == 1, odom_information, loop_information).astype(np.float64)
        self.poses = dv.to_dev(poses, np.float64, device)
        dev = self.poses.device
        self.ea = dv.to_dev(ea, np.int32, dev)
        self.eb = dv.to_dev(eb, np.int32, dev)
        self.tf = dv.to_dev(np.asarray(tf, dtype=np.float64).reshape(-1, 9), np.float64, dev)
        self.w = dv.to_dev(w, np.float64, dev)
        p = self.plan
        self.node_col = dv.to_dev(p.node_col, np.int32, dev)
        self.slot_rc = dv.to_dev(p.slot_rc, np.int32, dev)
        self.slot_ptr = dv.to_dev(p.slot_ptr, np.int32, dev)
        self.slot_items = dv.to_dev(p.slot_items, np.int32, dev)
        self.nbr_rows = dv.to_dev(p.nbr_rows if len(p.nbr_rows) else np.zeros(1, np.int32), np.int32, dev)
        n = int(_abi.lib().slam_gn_work_size_bordered(self.N, self.E, p.W, p.nv - p.nv_band)
                if p.nv_band < p.nv else _abi.lib().slam_gn_work_size(self.N, self.E, p.W))
        self.work = dv.empty((n,), np.float64, dev)
        self.status = dv.to_dev(np.zeros(1, np.int32), np.int32, dev)
        if p.pslot is not None:   # the Schur-accumulating bordered path
            mc = 16 * ((p.nv - p.nv_band + 16) // 16)
            self.pslot = dv.to_dev(p.pslot, np.int32, dev)

            self.pwork = dv.empty((max(len(p.schur_blocks), 1) * mc * mc,), np.float64, dev)
        self.chi2 = None
        self._eager_done = False
        self._graphs = {}

    def iterate(self, chi2_out, stream=None):
        """One asynchronous GN iteration; chi2 (before the step) -> chi2_out (device)."""
        p = self.plan
        if p.nv_band < p.nv and p.pslot is not None:
            _abi.check(_abi.lib().slam_gn_iteration_schur_f64(
                dv.ptr(self.poses), self.N, dv.ptr(self.ea), dv.ptr(self.eb), dv.ptr(self.tf), dv.ptr(self.w),
                self.E, dv.ptr(self.node_col), dv.ptr(self.slot_rc), dv.ptr(self.slot_ptr), dv.ptr(self.slot_items),
                p.n_slots, p.nv, p.W, p.nv_band, dv.ptr(self.pslot), len(p.schur_blocks), dv.ptr(self.pwork),
                dv.ptr(self.work), dv.ptr(chi2_out), dv.ptr(self.status), dv.stream_handle(stream)),
                "slam_gn_iteration_schur_f64")
            return
        if p.nv_band < p.nv:
            _abi.check(_abi.lib().slam_gn_iteration_bordered_f64(
                dv.ptr(self.poses), self.N, dv.ptr(self.ea), dv.ptr(self.eb), dv.ptr(self.tf), dv.ptr(self.w),
                self.E, dv.ptr(self.node_col), dv.ptr(self.slot_rc), dv.ptr(self.slot_ptr), dv.ptr(self.slot_items),
                p.n_slots, p.nv, p.W, p.nv_band, dv.ptr(self.nbr_rows), len(p.nbr_rows), dv.ptr(self.work),
                dv.ptr(chi2_out), dv.ptr(self.status), dv.stream_handle(stream)), "slam_gn_iteration_bordered_f64")
            return
        _abi.check(_abi.lib().slam_gn_iteration_f64(
            dv.ptr(self.poses), self.N, dv.ptr(self.ea), dv.ptr(self.eb), dv.ptr(self.tf), dv.ptr(self.w), self.E,
            dv.ptr(self.node_col), dv.ptr(self.slot_rc), dv.ptr(self.slot_ptr), dv.ptr(self.slot_items),
            p.n_slots, p.nv, p.W, dv.ptr(self.work), dv.ptr(chi2_out), dv.ptr(self.status),
            dv.stream_handle(stream)), "slam_gn_iteration_f64")

    def run(self, iterations=10, tol=None, stream=None, graph=None):
        """Run `iterations` steps; returns the chi2 before every step (host).

        After one eager run (which also sets the kernels' one-time attributes),
        the launch sequence of `iterations` steps (~30 kernels per step) is
        captured once into a HIP graph and replayed (``graph=False`` forces
        eager launches)."""
        t = dv.torch()
        if tol is not None and iterations > 1:
            # early exit: one step at a time, stop once chi2 (before each step)
            # changes by less than tol relative to the previous one
            out = []
            for _ in range(iterations):
                out.append(float(self.run(1, None, stream, graph)[0]))
                if len(out) > 1 and abs(out[-2] - out[-1]) <= tol * max(abs(out[-2]), 1e-300):
                    break
            self.chi2 = np.asarray(out)
            return self.chi2
        if stream is not None:
            # every torch op of the run (status reset, chi2 buffer, read-backs)
            # on the caller's stream, ordered with the launches
            with t.cuda.stream(stream):
                return self._run(iterations, stream, False)
        return self._run(iterations, None, graph)

    def _run(self, iterations, stream, graph):
        t = dv.torch()
        self.status.zero_()   # a failed earlier run must not poison this one
        lib = _abi.lib()
        # the fused back-substitution rests on the round-robin XCD dispatch; if a
        # wait times out (status bit 2) the steps are re-run without it
        fused = bool(self.plan.pslot is not None and self.plan.nv_band < self.plan.nv and lib.slam_gn_get_fused_back())
        backup = self.poses.clone() if fused else None
        if graph is None:
            graph = self._eager_done and stream is None and iterations > 0
        if graph:
            # keyed by the fused switch too: a graph captured with the fused
            # kernel is never replayed after any instance's fallback turned it off
            ent = self._graphs.get((iterations, fused))
            if ent is None:
                chis = t.zeros(iterations, dtype=t.float64, device=self.poses.device)
                g = t.cuda.CUDAGraph()
                with t.cuda.graph(g):
                    for k in range(iterations):
                        self.iterate(chis[k:k + 1])
                ent = self._graphs[(iterations, fused)] = (g, chis)
            g, chis = ent
            g.replay()
        else:
            chis = t.zeros(max(iterations, 1), dtype=t.float64, device=self.poses.device)
            for k in range(iterations):
                self.iterate(chis[k:k + 1], stream)
            self._eager_done = True
        out = chis[:iterations].cpu().numpy().copy()
        st = int(self.status.cpu().numpy()[0])
        if st & 2 and backup is not None:
            import warnings
            warnings.warn("Gauss-Newton: the XCD-local back-substitution timed out (workgroup dispatch not "
                          "round-robin over the XCDs?); re-running with one launch per level", RuntimeWarning)
            global FUSED_BACK_FALLBACKS
            FUSED_BACK_FALLBACKS += 1
            lib.slam_gn_set_fused_back(0)
            self._graphs.clear()
            self.poses.copy_(backup)
            return self._run(iterations, stream, graph)
        if st & 2:
            raise _abi.SlamHipError("Gauss-Newton: the fused back-substitution timed out waiting for a block")
        if st != 0:
            raise _abi.SlamHipError("Gauss-Newton: H is not positive definite (disconnected graph?)")
        self.chi2 = out
        return out

    def host_poses(self):
        return self.poses.cpu().numpy().reshape(self.N, 3)


def optimize(poses, ea, eb, tf, iterations=10, **kw):
    s = GaussNewton(poses, ea, eb, tf, **kw)
    chis = s.run(iterations)
    return s.host_poses(), chis


def bench_c4(iterations=10, reps=5):
    """GN iterations/s on config C4 (5k nodes / 20k edges), for bench.py: the
    MEDIAN of `reps` timed runs of `iterations` steps (best and worst beside it)."""
    from . import synthetic
    t = dv.torch()
    guess, ea, eb, tf, _ = synthetic.lap_graph_c4()
    t0 = time.perf_counter()
    plan = GnPlan(len(guess), ea, eb)
    plan_s = time.perf_counter() - t0
    s = GaussNewton(guess, ea, eb, tf, plan=plan)
    s.run(2)   # warm-up: the eager run (kernel attributes)
    s.run(iterations)   # and the capture of the `iterations`-step graph the timed runs replay
    dts = []
    for _ in range(reps):
        s.poses.copy_(dv.to_dev(guess, np.float64, s.poses.device))
        t.cuda.synchronize()
        t0 = time.perf_counter()
        chis = s.run(iterations)
        dts.append(time.perf_counter() - t0)
    med = float(np.median(dts))
    # end to end, as a caller sees it: host arrays in, plan (cold: symbolic
    # analysis; warm: cached structure), upload, `iterations` eager steps, poses out
    _PLANS.clear()
    ends = []
    for _ in range(2):
        t.cuda.synchronize()
        t0 = time.perf_counter()
        optimize(guess, ea, eb, tf, iterations)
        ends.append((time.perf_counter() - t0) * 1e3)
    return {"gn_iters_per_sec": round(iterations / med, 2), "gn_ms_per_iter": round(med / iterations * 1e3, 4),
            "gn_iters_per_sec_best_worst": [round(iterations / min(dts), 2), round(iterations / max(dts), 2)],
            "gn_timing": "median of %d runs of %d iterations (HIP graph replay, host clock around each run)" % (
                reps, iterations),
            "gn_fused_back_fallbacks": FUSED_BACK_FALLBACKS,
            "gn_call_ms_cold_plan": round(ends[0], 2), "gn_call_ms_cached_plan": round(ends[1], 2),
            "gn_call_note": "optimize(): %d iterations from host arrays incl. plan, upload, eager launches, "
                            "download" % iterations,
            "gn_graph": f"{len(guess)} nodes / {len(ea)} edges (C4)", "gn_band_W": plan.W,
            "gn_ordering": plan.ordering,
            "gn_plan_s": round(plan_s, 3), "gn_chi2_first_last": [float(chis[0]), float(chis[-1])],
            "gn_border_scalars": plan.nv - plan.nv_band,
            "gn_solver": "block cyclic reduction (Wb=%d)" % _abi.lib().slam_gn_bcr_block_rows(plan.nv_band, plan.W)
            + ((" + border Schur complement accumulated in the elimination (%d coupled blocks)" % len(plan.schur_blocks)
                if plan.pslot is not None else " + border Schur complement") if plan.nv_band < plan.nv else "")
            if _abi.lib().slam_gn_bcr_block_rows(plan.nv_band, plan.W) > 0 else "band Cholesky"}
