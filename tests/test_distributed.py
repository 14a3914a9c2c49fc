"""Multi-process (gloo, world size 2, CPU) tests of the query sharding and the
final top-K gather -- the only exchange of the multi-GPU path."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from influence.sharding import shard_ranges, gather_topk


def test_shard_ranges_balanced_and_contiguous():
    rng = np.random.default_rng(0)
    costs = rng.integers(1, 5000, 12074)
    for ws in (1, 2, 3, 8):
        rs = shard_ranges(costs, ws)
        assert len(rs) == ws and rs[0][0] == 0 and rs[-1][1] == costs.size
        assert all(rs[r][1] == rs[r + 1][0] for r in range(ws - 1))
        loads = [costs[b:e].sum() for b, e in rs]
        assert max(loads) <= costs.sum() / ws + costs.max()
    assert shard_ranges([], 4) == [(0, 0)] * 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, qs, K, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        rs = shard_ranges(np.ones(qs), ws)
        b, e = rs[rank]
        # stand-in per-rank results: deterministic functions of the global query id
        q = np.arange(b, e)
        idx = torch.tensor(np.stack([q * 10 + j for j in range(K)], 1), dtype=torch.int64).reshape(-1, K)
        val = torch.tensor(np.stack([np.sin(q + j) for j in range(K)], 1), dtype=torch.float64).reshape(-1, K)
        gi, gv = gather_topk(idx, val)
        # known sizes: no size exchange; and the async double-buffered form over 3 "steps"
        sizes = [e2 - b2 for b2, e2 in rs]
        gi2, gv2 = gather_topk(idx, val, sizes=sizes)
        from influence.sharding import TopKGather
        tg = TopKGather(sizes, K, "cpu")
        for step in range(3):
            tg.start(idx + 1000 * step, val + step)
        gi3, gv3 = tg.wait()
        assert np.array_equal(gi2.numpy(), gi.numpy()) and np.array_equal(gv2.numpy(), gv.numpy())
        out[rank] = (gi.numpy().copy(), gv.numpy().copy(), gi3.numpy().copy() - 2000, gv3.numpy().copy() - 2)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("qs", [9, 16])
def test_gather_topk_gloo_world2(qs):
    K = 3
    ws = 2
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(ws, _free_port(), qs, K, out), nprocs=ws, join=True)
        res = dict(out)
    q = np.arange(qs)
    want_i = np.stack([q * 10 + j for j in range(K)], 1)
    want_v = np.stack([np.sin(q + j) for j in range(K)], 1)
    for r in range(ws):
        gi, gv, gi3, gv3 = res[r]
        assert np.array_equal(gi, want_i)
        assert np.array_equal(gv, want_v)
        assert np.array_equal(gi3, want_i)          # the last async step's lists
        assert np.allclose(gv3, want_v, atol=1e-12)


def test_bench_rank_query_sets_are_distinct_and_same_shape():
    """bench.py weak scaling: rank r > 0 answers re-paired queries -- same users, same item
    multiset (so the same related-rating total), no pair in train, different from rank 0's."""
    import importlib
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    bench = importlib.import_module("bench")
    rng = np.random.default_rng(3)
    U, I, N, Q = 300, 120, 6000, 900
    key = rng.choice(U * I, N + Q, replace=False)
    tu, ti = (key[:N] // I).astype(np.int32), (key[:N] % I).astype(np.int32)
    qu, qi = (key[N:] // I).astype(np.int32), (key[N:] % I).astype(np.int32)
    train_key = set((tu.astype(np.int64) * I + ti).tolist())
    deg_u, deg_i = np.bincount(tu, minlength=U), np.bincount(ti, minlength=I)
    for rank in (1, 2, 7):
        q2 = bench.rank_query_items(qu, qi, (tu, ti, None), I, rank)
        assert np.array_equal(np.sort(q2), np.sort(qi))
        assert (q2 != qi).mean() > 0.9
        assert not any(int(u) * I + int(i) in train_key for u, i in zip(qu, q2))
        assert (deg_u[qu] + deg_i[q2]).sum() == (deg_u[qu] + deg_i[qi]).sum()


def test_bench_strong_split_with_query_cost():
    """bench.py strong scaling: every config balances n_q plus its per-query cost; the ranges
    are contiguous, cover every query once, and --shard-index picks one of them."""
    import importlib
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    bench = importlib.import_module("bench")
    rng = np.random.default_rng(5)
    n_q = rng.integers(20, 3000, 5000)
    for name, cfg in bench.CONFIGS.items():
        assert cfg["query_cost"] >= 0, name
        rs = shard_ranges(n_q + cfg["query_cost"], 8)
        assert rs[0][0] == 0 and rs[-1][1] == n_q.size
        assert all(rs[r][1] == rs[r + 1][0] for r in range(7))
        loads = [(n_q[b:e] + cfg["query_cost"]).sum() for b, e in rs]
        assert max(loads) <= (n_q + cfg["query_cost"]).sum() / 8 + n_q.max() + cfg["query_cost"]
    a = bench.parse(["--shard-of", "8", "--shard-index", "5", "--config", "20m-mf64"])
    assert a.shard_of == 8 and a.shard_index == 5
