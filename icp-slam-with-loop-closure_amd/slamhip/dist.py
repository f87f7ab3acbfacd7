"""Multi-GPU sharding of batched ICP (one process per GPU, torch.distributed).

Scan pairs are independent, so each rank owns a shard of the pair list, runs
ONE batched launch on its own GPU, and the per-pair results (the SE(2) edge,
its error and iteration count: 11 float64) are exchanged with a single
all-gather — over RCCL/xGMI with the "nccl" backend on ROCm, or gloo on CPU
for tests.  That is the only collective: the serial odometry chain
(scripts/main.py:249-256) then runs on every rank from the gathered edges.

Two shardings of one pair list:
  * ``shard_range``: contiguous index slices (the survey's default);
  * ``balanced_shards`` (bench.py's default): cost-balanced by a key known
    BEFORE any iteration runs — the turn of the pair's initial transform.
    A strong-scaling shard's time is set by its few long pairs, and on the
    C3 stream every pair of >= 60 ICP iterations starts from a turn of
    0.5-3 rad, so the turning pairs are dealt over the
    ranks (snake order, largest turn first) and the rest split in contiguous
    runs that make every rank's pair count equal.  A pair's result does not
    depend on its shard (order-free sums: bit-identical), only the gathered
    rows have to be put back in pair order (``unpack_shards``).
"""
import numpy as np

RESULT_WIDTH = 11   # 9 (transform) + error + iterations
TURN_THRESH = 0.3   # rad: a pair turning more than this is dealt (the library's angle pre-tier threshold)


def turn_keys(inits):
    """|rotation angle| of each initial transform (B, 3, 3) -> (B,) rad."""
    m = np.asarray(inits, dtype=np.float64).reshape(-1, 3, 3)
    return np.abs(np.arctan2(m[:, 1, 0], m[:, 0, 0]))


def balanced_shards(keys, world, thresh=TURN_THRESH):
    """Per-rank ascending pair indices of a cost-balanced split (module doc).

    Deterministic in (keys, world, thresh): every rank computes every rank's
    list, so the all-gather needs no index exchange.  Pair counts differ by at
    most one between ranks; the pairs with key > thresh are dealt in snake
    order of decreasing key (ties by index), so every rank gets the same
    number of them (+-1) and a similar mix of large and small turns."""
    keys = np.asarray(keys, dtype=np.float64).reshape(-1)
    B = len(keys)
    world = max(int(world), 1)
    heavy = np.flatnonzero(keys > thresh)
    heavy = heavy[np.lexsort((heavy, -keys[heavy]))]
    j = np.arange(len(heavy))
    lap, pos = j // world, j % world
    owner = np.where(lap % 2 == 0, pos, world - 1 - pos)
    h = np.bincount(owner, minlength=world)
    counts = np.full(world, B // world, dtype=np.int64)
    counts[:B % world] += 1
    quota = np.maximum(counts - h, 0)
    light = np.flatnonzero(~(keys > thresh))
    excess = int(quota.sum()) - len(light)   # > 0 only when a rank holds more turning pairs than its count
    while excess > 0:
        r = int(np.argmax(np.where(quota > 0, h + quota, -1)))
        quota[r] -= 1
        excess -= 1
    cut = np.r_[0, np.cumsum(quota)]
    return [np.sort(np.r_[heavy[owner == r], light[cut[r]:cut[r + 1]]]).astype(np.int64) for r in range(world)]


def contiguous_shards(n_items, world):
    """shard_range as index lists (the same interface as balanced_shards)."""
    return [np.arange(*shard_range(n_items, world, r)[:2], dtype=np.int64) for r in range(world)]


def unpack_shards(gathered, shards):
    """(world, rows, 11) gathered results of index-list shards -> host (tf
    (n,3,3), err (n,), iters (n,)) in pair order."""
    g = gathered.cpu().numpy() if hasattr(gathered, "cpu") else np.asarray(gathered)
    n = int(sum(len(s) for s in shards))
    out = np.zeros((n, RESULT_WIDTH))
    for r, idx in enumerate(shards):
        out[idx] = g[r, :len(idx)]
    return out[:, :9].reshape(-1, 3, 3), out[:, 9].copy(), out[:, 10].astype(np.int64)


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


def sharded_chain(odometry0, tf_local, n_items, group=None, iters_local=None, err_local=None, shards=None):
    """Every rank's ICP edges of its shard -> the full odometry chain
    (scripts/main.py:249-256) on every rank.  shards: every rank's pair
    indices (balanced_shards / contiguous_shards; default: contiguous
    shard_range slices), the local rows in the order of this rank's list.
    Returns (poses (n+1, 3), tf, err, iters)."""
    import torch
    import torch.distributed as dist
    from . import se2
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if shards is None:
        shards = contiguous_shards(n_items, world)
    B = len(shards[rank])
    rows = max(max(len(s) for s in shards), 1)
    tf = torch.as_tensor(np.asarray(tf_local, dtype=np.float64).reshape(B, 9))
    err = torch.as_tensor(np.zeros(B) if err_local is None else np.asarray(err_local, dtype=np.float64))
    its = torch.as_tensor(np.zeros(B, np.int64) if iters_local is None else np.asarray(iters_local))
    local = pack(tf, err, its, rows)
    if dist.get_backend(group) != "gloo":   # RCCL gathers device tensors only
        local = local.to(torch.device("cuda", torch.cuda.current_device()))
    g = all_gather_results(local, group)
    tf_all, err_all, it_all = unpack_shards(g, shards)
    return se2.compose_chain(np.asarray(odometry0, dtype=np.float64), tf_all), tf_all, err_all, it_all


def local_scans(scans, src, dst):
    """The scans a shard's pairs touch, once each: (scan list, local src,
    local dst) — a rank holds only its shard's scans in HBM."""
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    used, inv = np.unique(np.r_[src, dst], return_inverse=True)
    return [scans[i] for i in used], inv[:len(src)], inv[len(src):]


def unpack(gathered, n_items):
    """(world, rows, 11) -> host (tf (n,3,3), err (n,), iters (n,)) in pair order."""
    g = gathered.reshape(-1, RESULT_WIDTH)[:n_items].cpu().numpy()
    return g[:, :9].reshape(-1, 3, 3), g[:, 9].copy(), g[:, 10].astype(np.int64)
