"""bench.py's N > 1 path on the box's one GPU (the driver has no 8-GPU node):
torchrun starts 2 ranks of bench.py as a fresh child process — the launcher
runs before anything in that child touches the GPU — both on cuda:0
(SLAMHIP_ONE_DEVICE=1) with the gloo exchange, a 400-pair stream split 200 /
200 by the default cost-balanced sharding.  Rank 0's JSON line must carry n_gpus 2, pairs_total 400, every rank's
shard and kernel time, and green parity on its shard against the CPU
oracle.  Reference fan-out: /root/reference/scripts/main.py:240-247."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_bench_two_ranks_one_gpu():
    env = dict(os.environ, SLAMHIP_ONE_DEVICE="1", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--pairs", "400", "--steps", "2", "--warmup", "1",
           "--dist-backend", "gloo", "--no-pgo"]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["pairs_total"] == 400 and out["config"]["parallelism"] == "dp2"
    assert out["scaling"] == "strong" and out["value"] > 0
    pr = out["per_rank"]
    assert pr["pairs"] == [200, 200] and pr["max_shard_pairs"] == 200 and len(pr["kernel_ms"]) == 2
    assert all(k > 0 for k in pr["kernel_ms"])
    # the default cost-balanced sharding: the gathered edges, un-permuted, hold rank 0's results
    assert pr["shard"] == "balanced" and pr["all_gather_unpermuted_ok_rank0"] is True
    assert pr["exchange_timeouts"] == [0, 0] and len(pr["longest_pair_iterations"]) == 2
    assert out["exchange_timeouts"] == 0
    assert out["parity"]["ok"] and out["parity"]["iters_equal"] and out["parity"]["pairs"] >= 2
