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


def test_balanced_shards_partition_and_balance():
    """slamhip.dist.balanced_shards: a partition of the pairs (every index
    once, ascending within a shard), pair counts within one of each other,
    the turning pairs (key > thresh) dealt within one of each other, largest
    turns spread (the top `world` keys on distinct ranks), deterministic; edge
    cases: fewer pairs than ranks, every pair turning, none turning."""
    from slamhip import dist as sd
    rng = np.random.default_rng(3)
    cases = [(rng.uniform(0, 0.35, 10000), 8), (rng.uniform(0, 0.35, 9999), 3), (rng.uniform(0, 1, 5), 8),
             (np.full(11, 2.0), 4), (np.zeros(13), 4), (rng.uniform(0, 3, 64), 1), (np.zeros(0), 2)]
    for keys, w in cases:
        sh = sd.balanced_shards(keys, w)
        assert len(sh) == w
        allidx = np.concatenate(sh) if len(keys) else np.zeros(0, np.int64)
        assert sorted(allidx.tolist()) == list(range(len(keys)))
        assert all(np.all(np.diff(x) > 0) for x in sh)
        n = [len(x) for x in sh]
        assert max(n) - min(n) <= 1, n
        h = [int((keys[x] > sd.TURN_THRESH).sum()) for x in sh]
        assert max(h) - min(h) <= 1, h
        top = np.argsort(-keys, kind="stable")[:min(w, int((keys > sd.TURN_THRESH).sum()))]
        owners = [next(r for r, x in enumerate(sh) if t in x) for t in top]
        assert len(set(owners)) == len(owners)
        assert all(np.array_equal(a, b) for a, b in zip(sh, sd.balanced_shards(keys, w)))
    inits = np.stack([np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
                      for a in (0.1, -2.0, 3.0, 0.0)])
    assert np.allclose(sd.turn_keys(inits), [0.1, 2.0, 3.0, 0.0])


def test_unpack_shards_restores_pair_order():
    from slamhip import dist as sd
    import torch
    rng = np.random.default_rng(1)
    n, w = 37, 3
    shards = sd.balanced_shards(rng.uniform(0, 1, n), w)
    tf_all, err_all, it_all = rng.normal(size=(n, 3, 3)), rng.uniform(size=n), rng.integers(1, 50, n)
    rows = max(len(x) for x in shards)
    g = torch.stack([sd.pack(torch.from_numpy(tf_all[x].copy()), torch.from_numpy(err_all[x].copy()),
                             torch.from_numpy(it_all[x].copy()), rows) for x in shards])
    tf, err, its = sd.unpack_shards(g, shards)
    assert np.array_equal(tf, tf_all) and np.array_equal(err, err_all) and np.array_equal(its, it_all)
    scans = [np.full((3, 2), float(i)) for i in range(n + 1)]
    idx = shards[1]
    loc, s_l, d_l = sd.local_scans(scans, idx + 1, idx)
    assert all(np.array_equal(loc[a], scans[i + 1]) and np.array_equal(loc[b], scans[i])
               for a, b, i in zip(s_l, d_l, idx))
    assert len(loc) == len(np.unique(np.r_[idx, idx + 1]))


def _chain_worker(rank, world, port, n_pairs, q, mode="contiguous"):
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
    inits = np.stack([se2.pose_to_mat(seq.odometry[b + 1] - seq.odometry[b]) for b in range(n_pairs)])
    # balanced: a low threshold, so the short test stream has turning pairs to deal
    shards = (sd.balanced_shards(sd.turn_keys(inits), world, thresh=0.02) if mode == "balanced"
              else sd.contiguous_shards(n_pairs, world))
    tfs, errs, its = [], [], []
    for b in shards[rank]:
        h, e = icp_oracle.icp(np.c_[seq.scans[b + 1], np.ones(len(seq.scans[b + 1]))],
                              np.c_[seq.scans[b], np.ones(len(seq.scans[b]))],
                              se2.pose_to_mat(seq.odometry[b + 1] - seq.odometry[b]), 0.05, 100)
        tfs.append(h[-1])
        errs.append(e)
        its.append(len(h) - 1)
    chain, tf, err, it = sd.sharded_chain(seq.odometry[0], np.reshape(tfs, (-1, 3, 3)), n_pairs,
                                          iters_local=its, err_local=errs,
                                          shards=shards if mode == "balanced" else None)
    q.put((rank, chain, tf, err, it))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_pairs,mode", [(2, 9, "contiguous"), (3, 10, "contiguous"), (3, 2, "contiguous"),
                                              (2, 9, "balanced"), (3, 10, "balanced")])
def test_sharded_icp_chain_equals_single_process(world, n_pairs, mode):
    """Ragged shards (10 pairs on 3 ranks: 4/4/2; 2 pairs on 3 ranks: one rank
    empty), or cost-balanced index-list shards -> per-shard ICP -> one
    all-gather -> un-permute -> compose_chain on every rank equals the
    single-process chain bit for bit."""
    import icp_oracle
    from slamhip import se2, synthetic
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_chain_worker, args=(r, world, port, n_pairs, q, mode)) for r in range(world)]
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
