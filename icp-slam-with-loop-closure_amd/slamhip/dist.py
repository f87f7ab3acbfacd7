"""Multi-GPU sharding of batched ICP (one process per GPU, torch.distributed).

Scan pairs are independent, so each rank owns a contiguous shard of the pair
list, runs ONE batched launch on its own GPU, and the per-pair results (the
SE(2) edge, its error and iteration count: 11 float64) are exchanged with a
single all-gather — over RCCL/xGMI with the "nccl" backend on ROCm, or gloo
on CPU for tests.  That is the only collective: the serial odometry chain
(scripts/main.py:249-256) then runs on every rank from the gathered edges.
"""
import numpy as np

RESULT_WIDTH = 11   # 9 (transform) + error + iterations


def shard_range(n_items, world, rank):
    """Contiguous [lo, hi) of `n_items` for `rank` (ceil-split, last may be short)."""
    per = (n_items + world - 1) // world if world > 0 else n_items
    lo = min(rank * per, n_items)
    return lo, min(lo + per, n_items), per


def pack(tf, err, iters, rows, out=None):
    """Results of B local pairs -> (rows, 11) float64 tensor (zero padded)."""
    import torch
    B = tf.shape[0]
    if out is None:
        out = torch.zeros((rows, RESULT_WIDTH), dtype=torch.float64, device=tf.device)
    if B:
        out[:B, :9] = tf.reshape(B, 9)
        out[:B, 9] = err.reshape(B)
        out[:B, 10] = iters.reshape(B).to(torch.float64)
    return out


def all_gather_results(local, group=None, out=None):
    """(rows, 11) per rank -> (world, rows, 11) on every rank: ONE
    all_gather_into_tensor over RCCL ("nccl" backend); with gloo (CPU tests,
    dry runs) the rows go through host tensors."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if out is None:
        out = torch.empty((world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "gloo":
        parts = [torch.empty(tuple(local.shape), dtype=local.dtype) for _ in range(world)]
        dist.all_gather(parts, local.cpu(), group=group)
        out.copy_(torch.stack(parts))
    else:
        dist.all_gather_into_tensor(out, local, group=group)
    return out


def sharded_chain(odometry0, tf_local, n_items, group=None, iters_local=None, err_local=None):
    """Every rank's ICP edges of its contiguous shard -> the full odometry chain
    (scripts/main.py:249-256) on every rank.  Returns (poses (n+1, 3), tf, err, iters)."""
    import torch
    import torch.distributed as dist
    from . import se2
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi, per = shard_range(n_items, world, rank)
    B = hi - lo
    tf = torch.as_tensor(np.asarray(tf_local, dtype=np.float64).reshape(B, 9))
    err = torch.as_tensor(np.zeros(B) if err_local is None else np.asarray(err_local, dtype=np.float64))
    its = torch.as_tensor(np.zeros(B, np.int64) if iters_local is None else np.asarray(iters_local))
    local = pack(tf, err, its, max(per, 1))
    if dist.get_backend(group) != "gloo":   # RCCL gathers device tensors only
        local = local.to(torch.device("cuda", torch.cuda.current_device()))
    g = all_gather_results(local, group)
    tf_all, err_all, it_all = unpack(g, n_items)
    return se2.compose_chain(np.asarray(odometry0, dtype=np.float64), tf_all), tf_all, err_all, it_all


def unpack(gathered, n_items):
    """(world, rows, 11) -> host (tf (n,3,3), err (n,), iters (n,)) in pair order."""
    g = gathered.reshape(-1, RESULT_WIDTH)[:n_items].cpu().numpy()
    return g[:, :9].reshape(-1, 3, 3), g[:, 9].copy(), g[:, 10].astype(np.int64)
