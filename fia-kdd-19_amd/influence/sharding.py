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


def gather_topk(topk_idx, topk_val, group=None, sizes=None):
    """All ranks' [Q_r, K] top-K lists, concatenated in rank order on every rank.

    topk_idx: int64 tensor [Q_r, K]; topk_val: float64 tensor [Q_r, K] (same device
    as the process group's backend expects: cuda for nccl/RCCL, cpu for gloo).
    Shards may differ in Q_r: rows are padded to the largest shard, gathered, and
    the padding is dropped.  sizes (every rank's Q_r) skips the size exchange."""
    import torch
    import torch.distributed as dist
    ws = dist.get_world_size(group)
    K = topk_idx.shape[1] if topk_idx.dim() == 2 else 1
    if sizes is None:
        q_local = torch.tensor([topk_idx.shape[0]], dtype=torch.int64, device=topk_idx.device)
        sz = [torch.zeros_like(q_local) for _ in range(ws)]
        dist.all_gather(sz, q_local, group=group)
        sizes = [int(s.item()) for s in sz]
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


class TopKGather(object):
    """The per-step top-K exchange of a multi-GPU job, asynchronous and double-buffered.

    Shard sizes are known up front (contiguous ranges from shard_ranges, or equal
    per-GPU batches), so there is no size exchange: start() packs this rank's
    [Q_r, K] lists (int64 index + float64 bits) into one of two persistent buffers
    and launches one all_gather with async_op=True, which overlaps the next step's
    kernels on the compute stream (RCCL runs on its own stream).  A buffer is
    reused only after its previous collective completed; wait() drains both and
    returns the gathered [sum Q_r, K] lists of the last start()."""

    def __init__(self, sizes, K, device, group=None):
        import torch
        self.sizes = [int(x) for x in sizes]
        self.K = int(K)
        self.group = group
        qmax = max(self.sizes) if self.sizes else 0
        self.pack = [torch.full((max(qmax, 1), 2 * self.K), -1, dtype=torch.int64, device=device) for _ in range(2)]
        self.bufs = [[torch.empty_like(self.pack[j]) for _ in self.sizes] for j in range(2)]
        self.work = [None, None]
        self.slot = 0
        self.last = None

    def start(self, topk_idx, topk_val):
        import torch.distributed as dist
        j = self.slot
        self.slot ^= 1
        if self.work[j] is not None:
            self.work[j].wait()
        n = topk_idx.shape[0]
        p = self.pack[j]
        if n:
            p[:n, :self.K] = topk_idx.reshape(-1, self.K)
            p[:n, self.K:] = topk_val.reshape(-1, self.K).contiguous().view(p.dtype)
        self.work[j] = dist.all_gather(self.bufs[j], p, group=self.group, async_op=True)
        self.last = j
        return j

    def wait(self):
        import torch
        for j in range(2):
            if self.work[j] is not None:
                self.work[j].wait()
                self.work[j] = None
        if self.last is None:
            return None, None
        parts = [b[:s] for b, s in zip(self.bufs[self.last], self.sizes)]
        allp = torch.cat(parts, 0)
        return allp[:, :self.K].contiguous(), allp[:, self.K:].contiguous().view(torch.float64)
