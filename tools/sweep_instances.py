"""Diagnostics: time slam_icp_batch_f64 for every compiled (BLOCK, QPT)
instance (and several batch sizes) on the C3 workload.  GPU only."""
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))

import torch  # noqa: E402
from slamhip import _abi, se2, synthetic  # noqa: E402
from slamhip import icp as k  # noqa: E402


def main():
    pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    beams = int(sys.argv[2]) if len(sys.argv) > 2 else 1081
    seq = synthetic.make_sequence(pairs + 1, seed=2025, n_beams=beams)
    inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, pairs + 1)])
    ss = k.ScanSet(seq.scans)
    lib = _abi.lib()
    lib.slam_icp_set_screen(int(os.environ.get("SLAMHIP_SCREEN", "2")))
    b, q = ctypes.c_int32(), ctypes.c_int32()
    rows = []
    only = os.environ.get("SWEEP_INSTANCES")
    cand = [int(x) for x in only.split(",")] if only else [-1] + list(range(lib.slam_icp_num_instances()))
    sizes = (pairs,) if only else (pairs // 4, pairs // 2, pairs)
    for i in cand:
        if i >= 0:
            lib.slam_icp_instance_shape(i, ctypes.byref(b), ctypes.byref(q))
            if b.value * q.value < ss.lens.max():
                continue
        lib.slam_icp_force_instance(i)
        for B in sizes:
            batch = k.IcpBatch(ss, np.arange(1, B + 1), np.arange(0, B), inits[:B], epsilon=0.05, max_iters=100)
            batch.launch()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(3):
                e0.record()
                batch.launch()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            r = batch.result()
            evals = float(np.sum(r.iters * ss.lens[1:B + 1] * ss.lens[0:B]))
            ms = min(ts)
            sel = lib.slam_icp_selected_instance(int(ss.lens.max()))
            lib.slam_icp_instance_shape(sel, ctypes.byref(b), ctypes.byref(q))
            rows.append({"instance": f"{b.value}x{q.value}", "forced": i, "B": B, "ms": round(ms, 3),
                         "pairs_per_s": round(B / ms * 1e3, 1), "Geval_per_s": round(evals / ms / 1e6, 1),
                         "mean_iters": round(float(r.iters.mean()), 3)})
            print(json.dumps(rows[-1]), flush=True)
    lib.slam_icp_force_instance(-1)


if __name__ == "__main__":
    main()
