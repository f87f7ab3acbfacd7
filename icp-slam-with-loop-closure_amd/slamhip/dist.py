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


def all_gather_results(local, group=None):
    """(rows, 11) per rank -> (world, rows, 11) on every rank."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = torch.empty((world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "gloo":
        dist.all_gather(list(out.unbind(0)), local, group=group)
    else:
        dist.all_gather_into_tensor(out, local, group=group)
    return out


def unpack(gathered, n_items):
    """(world, rows, 11) -> host (tf (n,3,3), err (n,), iters (n,)) in pair order."""
    g = gathered.reshape(-1, RESULT_WIDTH)[:n_items].cpu().numpy()
    return g[:, :9].reshape(-1, 3, 3), g[:, 9].copy(), g[:, 10].astype(np.int64)
