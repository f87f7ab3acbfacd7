"""Co-residency probe: another process holds `n_cu - free` CUs (one CU-exclusive workgroup
each, `slam_icp_diag_occupy`) for 0.6 s while this process times (a) a trivial torch kernel,
(b) the 1,250-pair C3 shard with every latency tier off, (c) the same shard with the
automatic tier profile. Prints one line per case: wall time, exchange timeouts.
Usage: python tools/occupy_probe.py [free_cus ...]"""
import os
import select
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "icp-slam-with-loop-closure_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from slamhip import _abi, icp as k  # noqa: E402

OCC = """
import sys, time
sys.path.insert(0, sys.argv[1])
import torch
from slamhip import _abi
torch.cuda.set_device(0)
lib = _abi.lib()
assert lib.slam_icp_diag_occupy(int(sys.argv[2]), int(sys.argv[3]), None) == 0
t0 = time.perf_counter()
print("launched", flush=True)
torch.cuda.synchronize()
print("done %.3f" % (time.perf_counter() - t0), flush=True)
"""


def occupied(n_wg, fn):
    p = subprocess.Popen([sys.executable, "-c", OCC, PKG, str(n_wg), "60000000"],
                         stdout=subprocess.PIPE, text=True)
    try:
        ready, _, _ = select.select([p.stdout], [], [], 90)
        assert ready and p.stdout.readline().strip() == "launched"
        time.sleep(0.05)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        tail = p.stdout.read().strip()
        assert p.wait(timeout=30) == 0
    finally:
        if p.poll() is None:
            p.kill()
    return dt, tail


def main():
    frees = [int(x) for x in sys.argv[1:]] or [8, 32]
    lib = _abi.lib()
    n = 1250
    from test_icp_gpu import _sequence_pairs
    seq, inits = _sequence_pairs(n, seed=2025)
    ss = k.ScanSet(seq.scans)
    b = k.IcpBatch(ss, np.arange(1, n + 1), np.arange(0, n), inits, epsilon=0.05, max_iters=100)
    x = torch.ones(1 << 20, device="cuda")

    def plain():
        lib.slam_icp_set_schedule_auto(0)
        lib.slam_icp_set_schedule_gangs(0, 4)
        lib.slam_icp_set_schedule_heads(0)
        lib.slam_icp_set_schedule_wide(0, 1)
        lib.slam_icp_set_angle_tier(0, 0.3)
        lib.slam_icp_set_gang_first_wait(0)   # (the drain tier still runs: its first-exchange wait)

    def auto():
        lib.slam_icp_set_schedule_auto(1)
        lib.slam_icp_set_gang_first_wait(0)   # the default first-exchange wait (4 ms)

    def auto_w200():   # every exchange waiting the full 0.2 s (the round-5 behaviour)
        lib.slam_icp_set_schedule_auto(1)
        lib.slam_icp_set_gang_first_wait(20000000)

    for setup in (plain, auto):
        setup()
        b.launch()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        b.launch()
        torch.cuda.synchronize()
        print("%-6s unoccupied %.4f s timeouts %d" % (setup.__name__, time.perf_counter() - t0,
                                                     lib.slam_icp_gang_timeouts()), flush=True)
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    for free in frees:
        dt, tail = occupied(n_cu - free, lambda: (x.add_(1), x.sum().item()))
        print("free %3d trivial   %.4f s  occupier %s" % (free, dt, tail), flush=True)
        for setup in (plain, auto, auto_w200):
            setup()
            lib.slam_icp_gang_timeouts()
            dt, tail = occupied(n_cu - free, b.launch)
            print("free %3d %-9s %.4f s  timeouts %d  occupier %s" % (
                free, setup.__name__, dt, lib.slam_icp_gang_timeouts(), tail), flush=True)
    auto()


if __name__ == "__main__":
    main()
