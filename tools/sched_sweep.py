"""Scheduler settings vs batch size, in one process: rank 0's shard of the C3
stream (first P pairs) for P in 1250 / 2500 / 5000 / 10000, timed with HIP
events (median of 7 launches) under each setting
"heads,gangs,parts,wide,share,bulk_below,bulk_parts,probe[,warm[,sort_one]]"
(probe -1: automatic; warm default 0 and sort_one 1, the product defaults).  SWEEP_SIZES=1250,2500 picks
the batch sizes.  GPU only.

    python tools/sched_sweep.py [setting ...]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "icp-slam-with-loop-closure_amd"))

DEFAULT = [
    "64,24,4,0,1,0,2,4",     # round-3 defaults
    "16,8,4,0,1,0,2,4",
    "16,4,4,1,1,0,2,4",
    "8,0,4,1,1,0,2,4",
    "0,0,4,0,1,0,2,4",
    "0,0,4,0,1,8192,2,4",
    "16,8,4,0,1,8192,2,4",
    "16,4,4,1,1,8192,2,4",
    "0,0,4,0,1,0,2,0",
    "0,0,4,0,1,0,2,2",
    "16,8,4,0,1,0,2,2",
]


def main():
    import torch
    torch.cuda.set_device(0)
    from slamhip import _abi, se2, synthetic
    from slamhip import icp as k
    lib = _abi.lib()
    settings = sys.argv[1:] or DEFAULT
    sizes = [int(x) for x in os.environ.get("SWEEP_SIZES", "1250,2500,5000,10000").split(",")]
    seq = synthetic.make_sequence(10001, seed=2025)
    inits = np.stack([se2.pose_to_mat(seq.odometry[i] - seq.odometry[i - 1]) for i in range(1, 10001)])
    ss = k.ScanSet(seq.scans)
    batches = {P: k.IcpBatch(ss, np.arange(1, P + 1), np.arange(0, P), inits[:P], epsilon=0.05, max_iters=100)
               for P in sizes}
    ref = {}
    try:
        for st in settings:
            v = [int(x) for x in st.split(",")]
            h, g, gp, w, ws, bb, bp, pr = v[:8]
            assert lib.slam_icp_set_schedule_warm(v[8] if len(v) > 8 else 0) == 0
            assert lib.slam_icp_set_schedule_heads(h) == 0
            assert lib.slam_icp_set_schedule_gangs(g, gp) == 0
            assert lib.slam_icp_set_schedule_wide(w, ws) == 0
            assert lib.slam_icp_set_bulk_gangs(bb, bp) == 0
            assert lib.slam_icp_set_schedule(pr, 1024) == 0
            assert lib.slam_icp_set_sched_sort_one(v[9] if len(v) > 9 else 1) == 0
            out = []
            for P in sizes:
                b = batches[P]
                b.launch()
                torch.cuda.synchronize()
                ts = []
                for _ in range(7):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    b.launch()
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1))
                r = b.result()
                if P not in ref:
                    ref[P] = r
                same = np.array_equal(r.tf, ref[P].tf) and np.array_equal(r.iters, ref[P].iters)
                out.append(f"{P}:{np.median(ts):.3f}{'' if same else '!'}")
            print(f"h,g,k,w,s,bb,bp,probe {st:22s} " + " ".join(out), flush=True)
    finally:
        lib.slam_icp_set_schedule_auto(1)
        lib.slam_icp_set_bulk_gangs(0, 2)
        lib.slam_icp_set_schedule(-1, 1024)
        lib.slam_icp_set_schedule_warm(0)
        lib.slam_icp_set_sched_sort_one(1)


if __name__ == "__main__":
    main()
