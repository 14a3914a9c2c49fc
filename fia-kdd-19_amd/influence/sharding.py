"""Query sharding across the GPUs of one node and the final top-K gather.

FIA queries are independent (each reads only u's row, i's column and the
read-only parameters, matrix_factorization.py:315-322, 288-308), so a query
batch splits into contiguous per-rank ranges with no data-path collective.
The only exchange is the one the north star names: rank 0 collects every
rank's top-K influencer lists (a few bytes per query) with one all_gather over
RCCL (xGMI) -- or gloo on CPU in tests.
"""
import numpy as np


def shard_ranges(costs, world_size):
    """Contiguous [begin, end) query ranges, one per rank, balanced by the prefix
    sum of per-query costs (e.g. n_q, the related-set sizes)."""
    costs = np.asarray(costs, np.float64)
    n = costs.size
    if world_size <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(world_size - 1, 0)
    csum = np.concatenate([[0.0], np.cumsum(costs)])
    total = csum[-1]
    bounds = [0]
    for r in range(1, world_size):
        b = int(np.searchsorted(csum, total * r / world_size, side="left"))
        bounds.append(min(max(b, bounds[-1]), n))
    bounds.append(n)
    return [(bounds[r], bounds[r + 1]) for r in range(world_size)]


def gather_topk(topk_idx, topk_val, group=None):
    """All ranks' [Q_r, K] top-K lists, concatenated in rank order on every rank.

    topk_idx: int64 tensor [Q_r, K]; topk_val: float64 tensor [Q_r, K] (same device
    as the process group's backend expects: cuda for nccl/RCCL, cpu for gloo).
    Shards may differ in Q_r: rows are padded to the largest shard, gathered, and
    the padding is dropped."""
    import torch
    import torch.distributed as dist
    ws = dist.get_world_size(group)
    K = topk_idx.shape[1] if topk_idx.dim() == 2 else 1
    q_local = torch.tensor([topk_idx.shape[0]], dtype=torch.int64, device=topk_idx.device)
    sizes = [torch.zeros_like(q_local) for _ in range(ws)]
    dist.all_gather(sizes, q_local, group=group)
    sizes = [int(s.item()) for s in sizes]
    qmax = max(sizes) if sizes else 0
    # pack idx and value bits into one int64 [Q, 2K] buffer: one collective
    pack = torch.full((qmax, 2 * K), -1, dtype=torch.int64, device=topk_idx.device)
    if topk_idx.shape[0]:
        pack[:topk_idx.shape[0], :K] = topk_idx.reshape(-1, K)
        pack[:topk_idx.shape[0], K:] = topk_val.reshape(-1, K).contiguous().view(torch.int64)
    bufs = [torch.empty_like(pack) for _ in range(ws)]
    dist.all_gather(bufs, pack, group=group)
    parts = [b[:s] for b, s in zip(bufs, sizes)]
    allp = torch.cat(parts, 0) if parts else pack[:0]
    return allp[:, :K].contiguous(), allp[:, K:].contiguous().view(torch.float64)
