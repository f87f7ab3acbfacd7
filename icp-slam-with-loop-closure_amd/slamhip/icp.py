"""Batched ICP on the GPU: the throughput API behind the drop-in ``src/icp.py``.

One call runs ``icp()`` (reference ``src/icp.py:72-97``) for B independent
scan pairs in ONE kernel launch (one pair per workgroup), replacing the
reference's joblib fan-out (``scripts/main.py:240-247``).

Layout in HBM (see DESIGN.md §Data layout):
  pts       (P, 2) float64  every scan's (x, y) rows back to back
  scan_off  (S+1,) int64    scan s = pts[scan_off[s]:scan_off[s+1]]
  src, dst  (B,)   int32    pc1 / pc2 scan index of pair b
  init      (B, 9) float64  row-major 3x3
A scan stream (pairs (i, i-1), as main.py builds them) therefore stores every
scan once although it appears in two pairs.
"""
from dataclasses import dataclass

import numpy as np

from . import _abi
from . import device as dv


def _xy(scan):
    """(m, 2) float64 rows of a reference point cloud ((m, 2) or homogeneous (m, 3))."""
    a = np.asarray(scan, dtype=np.float64)
    if a.ndim != 2 or a.shape[1] not in (2, 3):
        raise ValueError(f"point cloud must be (n, 2) or homogeneous (n, 3), got {a.shape}")
    if a.shape[1] == 3 and not np.all(a[:, 2] == 1.0):
        raise ValueError("homogeneous coordinate must be exactly 1 (np.c_[points, ones])")
    if len(a) == 0:
        raise ValueError("empty point cloud")
    return a[:, :2]


def _se2_rows(mats, B):
    m = np.asarray(mats, dtype=np.float64).reshape(B, 3, 3)
    if not (np.all(m[:, 2, 0] == 0) and np.all(m[:, 2, 1] == 0) and np.all(m[:, 2, 2] == 1)):
        raise ValueError("transforms must be SE(2) homogeneous matrices with last row [0, 0, 1]")
    return m.reshape(B, 9)


class ScanSet:
    """Ragged scans packed into device memory once, shared by many pairs."""

    def __init__(self, scans, device=None):
        xy = [_xy(s) for s in scans]
        self.lens = np.array([len(s) for s in xy], dtype=np.int64)
        self.off = np.zeros(len(xy) + 1, dtype=np.int64)
        self.off[1:] = np.cumsum(self.lens)
        host = np.concatenate(xy, axis=0) if xy else np.zeros((0, 2))
        self.host_pts = host
        self.pts = dv.to_dev(host, np.float64, device)
        self.scan_off = dv.to_dev(self.off, np.int64, device)
        self.device = self.pts.device

    def __len__(self):
        return len(self.lens)


@dataclass
class IcpResult:
    tf: np.ndarray        # (B, 3, 3) transforms[-1]
    err: np.ndarray       # (B,) returned error
    iters: np.ndarray     # (B,) ICP iterations (len(transforms) - 1)
    hist: list = None     # B arrays (iters+1, 3, 3) when history was requested


class IcpBatch:
    """A prepared batch of B pairs; ``launch()`` is asynchronous on a stream."""

    def __init__(self, scanset, src, dst, init, epsilon=0.01, max_iters=100,
                 stopping_thresh=0.0001, rotation_only=False, history=False):
        self.ss = scanset
        src = np.asarray(src, dtype=np.int32)
        dst = np.asarray(dst, dtype=np.int32)
        if src.shape != dst.shape or src.ndim != 1:
            raise ValueError("src/dst must be equal-length 1-D index arrays")
        S = len(scanset)
        if len(src) and (src.min() < 0 or dst.min() < 0 or src.max() >= S or dst.max() >= S):
            raise ValueError("scan index out of range")
        self.B = B = len(src)
        self.epsilon = float(epsilon)
        self.max_iters = int(max_iters)
        self.stopping_thresh = float(stopping_thresh)
        self.rotation_only = bool(rotation_only)
        self.max_n1 = int(scanset.lens[src].max()) if B else 1
        self.max_n2 = int(scanset.lens[dst].max()) if B else 1
        if self.max_n1 > _abi.lib().slam_icp_max_query_points():
            raise ValueError(f"pc1 of {self.max_n1} points exceeds the kernel capacity "
                             f"{_abi.lib().slam_icp_max_query_points()}")
        dev = scanset.device
        self.src = dv.to_dev(src, np.int32, dev)
        self.dst = dv.to_dev(dst, np.int32, dev)
        self.init = dv.to_dev(_se2_rows(init, B), np.float64, dev)
        self.hist_stride = (self.max_iters + 3) if history else 0
        self.out_tf = dv.empty((max(B, 1), 9), np.float64, dev)
        self.out_err = dv.empty((max(B, 1),), np.float64, dev)
        self.out_iters = dv.empty((max(B, 1),), np.int32, dev)
        self.out_hist = dv.empty((max(B, 1), self.hist_stride, 9), np.float64, dev) if history else None

    def launch(self, stream=None):
        if self.B == 0:
            return
        L = _abi.lib()
        _abi.check(L.slam_icp_batch_f64(
            dv.ptr(self.ss.pts), dv.ptr(self.ss.scan_off), dv.ptr(self.src), dv.ptr(self.dst),
            dv.ptr(self.init), self.B, self.epsilon, self.max_iters, self.stopping_thresh,
            int(self.rotation_only), self.max_n1, self.max_n2, self.hist_stride, dv.ptr(self.out_hist),
            dv.ptr(self.out_tf), dv.ptr(self.out_err), dv.ptr(self.out_iters), dv.stream_handle(stream)),
            "slam_icp_batch_f64")

    def check(self, stream=None):
        """Synchronise and raise if the kernel flagged a pair outside the launch bounds."""
        _abi.check(_abi.lib().slam_icp_status(dv.stream_handle(stream)), "slam_icp_batch_f64")

    def result(self):
        B = self.B
        if B:
            self.check()
        tf = self.out_tf[:B].cpu().numpy().reshape(B, 3, 3)
        err = self.out_err[:B].cpu().numpy()
        iters = self.out_iters[:B].cpu().numpy().astype(np.int64)
        hist = None
        if self.out_hist is not None:
            h = self.out_hist[:B].cpu().numpy().reshape(B, self.hist_stride, 3, 3)
            hist = [h[b, :iters[b] + 1] for b in range(B)]
        return IcpResult(tf, err, iters, hist)


def icp_batch(scans, src, dst, init, epsilon=0.01, max_iters=100, stopping_thresh=0.0001,
              rotation_only=False, history=False, device=None, stream=None):
    """ICP for B pairs (src[b] -> dst[b]) over a list of scans; returns IcpResult."""
    ss = scans if isinstance(scans, ScanSet) else ScanSet(scans, device)
    batch = IcpBatch(ss, src, dst, init, epsilon, max_iters, stopping_thresh, rotation_only, history)
    batch.launch(stream)
    return batch.result()


class _PairStaging:
    """Pinned host and device byte buffers reused by single-pair calls: one
    host->device copy of every input, one device->host copy of every output."""

    def __init__(self, device):
        self.device = device
        self.cap_in = self.cap_out = 0

    def buffers(self, n_in, n_out):
        t = dv.torch()
        if n_in > self.cap_in:
            self.cap_in = max(n_in, 2 * self.cap_in)
            self.h_in = t.empty(self.cap_in, dtype=t.uint8).pin_memory()
            self.d_in = t.empty(self.cap_in, dtype=t.uint8, device=self.device)
        if n_out > self.cap_out:
            self.cap_out = max(n_out, 2 * self.cap_out)
            self.h_out = t.empty(self.cap_out, dtype=t.uint8).pin_memory()
            self.d_out = t.empty(self.cap_out, dtype=t.uint8, device=self.device)
        return self.h_in, self.d_in, self.h_out, self.d_out


_STAGING = {}


def _a16(n):
    return (n + 15) // 16 * 16


def icp_pair(pc1, pc2, init, epsilon=0.01, max_iters=100, stopping_thresh=0.0001, rotation_only=False):
    """ONE pair with its transform history (the drop-in ``icp()``'s call):
    inputs packed into one pinned staging buffer (one copy in), outputs in one
    device buffer (one copy out).  Returns (hist (iters+1, 3, 3), err, iters)."""
    t = dv.require_gpu()
    a, b = _xy(pc1), _xy(pc2)
    n1, n2 = len(a), len(b)
    if n1 > _abi.lib().slam_icp_max_query_points():
        raise ValueError(f"pc1 of {n1} points exceeds the kernel capacity {_abi.lib().slam_icp_max_query_points()}")
    T0 = _se2_rows(init, 1)
    max_iters = int(max_iters)
    stride = max_iters + 3
    o_pts, o_off = 0, _a16(16 * (n1 + n2))
    o_idx, o_init = o_off + 32, o_off + 48
    n_in = o_init + 80
    o_hist, o_tf = 0, _a16(72 * stride)
    o_err, o_it = o_tf + 80, o_tf + 96
    n_out = o_it + 16
    dev = t.cuda.current_device()
    st = _STAGING.get(dev)
    if st is None:
        st = _STAGING[dev] = _PairStaging(t.device("cuda", dev))
    h_in, d_in, h_out, d_out = st.buffers(n_in, n_out)
    stream = t.cuda.current_stream()
    stream.synchronize()   # the staging buffers of the previous call are free
    hb = h_in.numpy()
    pts = np.frombuffer(hb, dtype=np.float64, count=2 * (n1 + n2), offset=o_pts).reshape(-1, 2)
    pts[:n1] = a
    pts[n1:] = b
    np.frombuffer(hb, dtype=np.int64, count=3, offset=o_off)[:] = (0, n1, n1 + n2)
    np.frombuffer(hb, dtype=np.int32, count=2, offset=o_idx)[:] = (0, 1)
    np.frombuffer(hb, dtype=np.float64, count=9, offset=o_init)[:] = T0[0]
    d_in[:n_in].copy_(h_in[:n_in], non_blocking=True)
    base, ob = d_in.data_ptr(), d_out.data_ptr()
    _abi.check(_abi.lib().slam_icp_batch_f64(
        base + o_pts, base + o_off, base + o_idx, base + o_idx + 4, base + o_init, 1, float(epsilon), max_iters,
        float(stopping_thresh), int(bool(rotation_only)), n1, n2, stride, ob + o_hist, ob + o_tf, ob + o_err,
        ob + o_it, stream.cuda_stream), "slam_icp_batch_f64")
    h_out[:n_out].copy_(d_out[:n_out], non_blocking=True)
    stream.synchronize()
    ho = h_out.numpy()
    iters = int(np.frombuffer(ho, dtype=np.int32, count=1, offset=o_it)[0])
    if iters == np.iinfo(np.int32).min:   # the kernel flagged the pair: report (and clear) it
        _abi.check(_abi.lib().slam_icp_status(stream.cuda_stream), "slam_icp_batch_f64")
    hist = np.frombuffer(ho, dtype=np.float64, count=9 * stride, offset=o_hist).reshape(stride, 3, 3)
    err = np.float64(np.frombuffer(ho, dtype=np.float64, count=1, offset=o_err)[0])
    return hist[:iters + 1].copy(), err, iters


def icp_pairs(pc1_list, pc2_list, inits, **kw):
    """ICP over explicit (pc1, pc2, init) triples (the shape of the reference's
    ``delayed(icp.icp)(pc1, pc2, init_transform=...)`` fan-out)."""
    scans = []
    for a, b in zip(pc1_list, pc2_list):
        scans.append(a)
        scans.append(b)
    B = len(pc1_list)
    return icp_batch(scans, np.arange(0, 2 * B, 2), np.arange(1, 2 * B, 2), inits, **kw)


def icp_step(scans, src, dst, T_in, rotation_only=False, device=None, stream=None):
    """One ``icp_iteration`` per pair: returns (T_out (B,3,3), corr list, err (B,))."""
    ss = scans if isinstance(scans, ScanSet) else ScanSet(scans, device)
    src = np.asarray(src, dtype=np.int32)
    dst = np.asarray(dst, dtype=np.int32)
    B = len(src)
    n1 = ss.lens[src]
    corr_off = np.zeros(B, dtype=np.int64)
    corr_off[1:] = np.cumsum(n1)[:-1]
    dev = ss.device
    d_src = dv.to_dev(src, np.int32, dev)
    d_dst = dv.to_dev(dst, np.int32, dev)
    d_T = dv.to_dev(_se2_rows(T_in, B), np.float64, dev)
    d_off = dv.to_dev(corr_off, np.int64, dev)
    T_out = dv.empty((B, 9), np.float64, dev)
    err = dv.empty((B,), np.float64, dev)
    corr = dv.empty((int(n1.sum()),), np.int64, dev)
    L = _abi.lib()
    _abi.check(L.slam_icp_step_f64(
        dv.ptr(ss.pts), dv.ptr(ss.scan_off), dv.ptr(d_src), dv.ptr(d_dst), dv.ptr(d_T), B,
        int(bool(rotation_only)), int(n1.max()), int(ss.lens[dst].max()), dv.ptr(T_out), dv.ptr(corr),
        dv.ptr(d_off), dv.ptr(err), dv.stream_handle(stream)), "slam_icp_step_f64")
    _abi.check(L.slam_icp_status(dv.stream_handle(stream)), "slam_icp_step_f64")
    c = corr.cpu().numpy()
    corr_list = [c[corr_off[b]:corr_off[b] + n1[b]] for b in range(B)]
    return T_out.cpu().numpy().reshape(B, 3, 3), corr_list, err.cpu().numpy()


def kabsch(a, b, device=None, stream=None):
    """get_transform + get_error of matched rows on the GPU: (T (3,3), err)."""
    xa, xb = _xy(a), _xy(b)
    if len(xa) != len(xb):
        raise ValueError("matched clouds must have the same number of rows")
    da = dv.to_dev(xa, np.float64, device)
    db = dv.to_dev(xb, np.float64, da.device)
    T = dv.empty((9,), np.float64, da.device)
    e = dv.empty((1,), np.float64, da.device)
    _abi.check(_abi.lib().slam_kabsch2d_f64(dv.ptr(da), dv.ptr(db), len(xa), dv.ptr(T), dv.ptr(e),
                                            dv.stream_handle(stream)), "slam_kabsch2d_f64")
    return T.cpu().numpy().reshape(3, 3), np.float64(e.cpu().numpy()[0])
