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


def _chain_worker(rank, world, port, n_pairs, q):
    """Strong sharding of one scan stream (bench.py's default multi-GPU mode):
    rank r runs the CPU oracle's icp() on its contiguous, possibly short shard,
    then slamhip.dist.sharded_chain all-gathers the edges and composes the
    odometry chain (scripts/main.py:240-256)."""
    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import torch.distributed as dist
    import icp_oracle
    from slamhip import dist as sd
    from slamhip import se2, synthetic
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seq = synthetic.make_sequence(n_pairs + 1, seed=11, n_beams=61)
    lo, hi, _ = sd.shard_range(n_pairs, world, rank)
    tfs, errs, its = [], [], []
    for b in range(lo, hi):
        h, e = icp_oracle.icp(np.c_[seq.scans[b + 1], np.ones(len(seq.scans[b + 1]))],
                              np.c_[seq.scans[b], np.ones(len(seq.scans[b]))],
                              se2.pose_to_mat(seq.odometry[b + 1] - seq.odometry[b]), 0.05, 100)
        tfs.append(h[-1])
        errs.append(e)
        its.append(len(h) - 1)
    chain, tf, err, it = sd.sharded_chain(seq.odometry[0], np.reshape(tfs, (-1, 3, 3)), n_pairs,
                                          iters_local=its, err_local=errs)
    q.put((rank, chain, tf, err, it))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_pairs", [(2, 9), (3, 10), (3, 2)])
def test_sharded_icp_chain_equals_single_process(world, n_pairs):
    """Ragged shards (10 pairs on 3 ranks: 4/4/2; 2 pairs on 3 ranks: one rank
    empty) -> per-shard ICP -> one all-gather -> compose_chain on every rank
    equals the single-process chain bit for bit."""
    import icp_oracle
    from slamhip import se2, synthetic
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_chain_worker, args=(r, world, port, n_pairs, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    seq = synthetic.make_sequence(n_pairs + 1, seed=11, n_beams=61)
    tfs, its = [], []
    for b in range(n_pairs):
        h, _ = icp_oracle.icp(np.c_[seq.scans[b + 1], np.ones(len(seq.scans[b + 1]))],
                              np.c_[seq.scans[b], np.ones(len(seq.scans[b]))],
                              se2.pose_to_mat(seq.odometry[b + 1] - seq.odometry[b]), 0.05, 100)
        tfs.append(h[-1])
        its.append(len(h) - 1)
    ref = se2.compose_chain(seq.odometry[0], np.stack(tfs))
    for rank, chain, tf, err, it in res:
        assert np.array_equal(chain, ref), rank
        assert np.array_equal(tf, np.stack(tfs)) and it.tolist() == its, rank
