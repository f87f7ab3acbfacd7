"""World-size-2 gloo test of the multi-GPU exchange (CPU): pairs are sharded by
slamhip.dist.shard_range, each rank packs its per-pair results, one all-gather
reassembles them in pair order, and the odometry chain built from the gathered
edges equals the single-process chain.  The per-pair "ICP results" here come
from the CPU oracle (no GPU in this container); on the GPU box bench.py runs
the same exchange over RCCL."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import PKG, REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_pairs, q):
    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import torch
    import torch.distributed as dist
    from slamhip import dist as sd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(0)
    tf_all = rng.normal(size=(n_pairs, 3, 3))
    err_all = rng.uniform(size=n_pairs)
    it_all = rng.integers(1, 20, size=n_pairs)
    lo, hi, per = sd.shard_range(n_pairs, world, rank)
    local = sd.pack(torch.from_numpy(tf_all[lo:hi].copy()), torch.from_numpy(err_all[lo:hi].copy()),
                    torch.from_numpy(it_all[lo:hi].copy()), per)
    g = sd.all_gather_results(local)
    tf, err, its = sd.unpack(g, n_pairs)
    ok = np.array_equal(tf, tf_all) and np.array_equal(err, err_all) and np.array_equal(its, it_all)
    q.put((rank, ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("n_pairs", [10, 7])
def test_gloo_allgather_world2(n_pairs):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_pairs, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res


def test_shard_range_covers():
    from slamhip import dist as sd
    for n in (0, 1, 7, 10, 10000):
        for w in (1, 2, 3, 8):
            seen = []
            for r in range(w):
                lo, hi, per = sd.shard_range(n, w, r)
                assert hi - lo <= per
                seen.extend(range(lo, hi))
            assert seen == list(range(n))
