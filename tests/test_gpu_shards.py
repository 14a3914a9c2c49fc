"""fia_prepare_for on the shards the 8-GPU job runs (bench.py --gpus 8, or --shard-of 8
--shard-index r on one GPU): each rank builds only its shard's Hessian caches, so the
marked Gram passes (small k: k_gram_mf_stream MARK + k_gram_combine) and the slot-mapped
large-k caches are what produce its results.

  * ml-1m-ex MF k=16 (the headline config): all 8 shards;
  * 20M MF k=64 (config 4): shards 0 and 7.

Each shard's outputs (related rows, influence, x, top-K) must equal, bit for bit, the same
queries' outputs after the full fia_prepare (the reference has one Hessian per query:
matrix_factorization.py:288-308, 315-322 -- which entities' caches exist must not change a
result), plus an fp64 oracle sample per shard including its heaviest query.  Config 5's
shards are in test_gpu_fullsize.py."""
import os

import numpy as np
import pytest

from influence import synth

pytestmark = pytest.mark.gpu

RTOL = 1e-5
BATCH_ROWS = 1 << 28


def _ctx(model, k, d, params):
    from test_gpu_fullsize import _ctx as mk
    return mk(model, k, d, params)


def shard_bounds(cfg_name, d, qu, qi, S=8):
    """bench.py's strong-scaling split (the per-query cost of the config)."""
    import bench
    from influence.sharding import shard_ranges
    deg_u = np.bincount(d["train"][0], minlength=d["U"])
    deg_i = np.bincount(d["train"][1], minlength=d["I"])
    return shard_ranges(deg_u[qu] + deg_i[qi] + bench.CONFIGS[cfg_name]["query_cost"], S)


def item_major(qu, qi):
    order = np.lexsort((qu, qi))
    return np.ascontiguousarray(qu[order]), np.ascontiguousarray(qi[order])


def batches(ctx, qu, qi, K):
    """bench.py's batching (<= BATCH_ROWS related ratings per fia_query_batch); yields the
    device outputs of each batch (buffers reused: consume before the next one)."""
    import torch
    dev = torch.device("cuda", 0)
    tqu, tqi = torch.from_numpy(qu).to(dev), torch.from_numpy(qi).to(dev)
    offs_all, _ = ctx.count_related(tqu, tqi)
    cum = np.concatenate([[0], np.cumsum(np.diff(offs_all.cpu().numpy()))])
    bounds = [0]
    while bounds[-1] < qu.size:
        b0 = bounds[-1]
        bounds.append(min(qu.size, max(int(np.searchsorted(cum, cum[b0] + BATCH_ROWS, side="right")) - 1, b0 + 1)))
    max_rows = int(max(cum[b1] - cum[b0] for b0, b1 in zip(bounds[:-1], bounds[1:])))
    D = ctx.num_params()
    rel = torch.empty(max(max_rows, 1), dtype=torch.int32, device=dev)
    infl = torch.empty(max(max_rows, 1), dtype=torch.float64, device=dev)
    for b0, b1 in zip(bounds[:-1], bounds[1:]):
        qb_u, qb_i = tqu[b0:b1].contiguous(), tqi[b0:b1].contiguous()
        offs, tot = ctx.count_related(qb_u, qb_i)
        xb = torch.empty((b1 - b0) * D, dtype=torch.float64, device=dev)
        tp = torch.empty((b1 - b0) * K, dtype=torch.int64, device=dev)
        tix = torch.empty_like(tp)
        tv = torch.empty((b1 - b0) * K, dtype=torch.float64, device=dev)
        ctx.query_batch(qb_u, qb_i, offs, tot, rel, infl, xb, K, tp, tix, tv)
        yield b0, b1, dict(offs=offs, rel=rel[:tot], infl=infl[:tot], x=xb, tp=tp, tix=tix, tv=tv)


def host(o):
    return {k: v.cpu().numpy() for k, v in o.items()}


def oracle_check(oracle, u, i, offs, rel, infl, x, j):
    from oracle import fia_oracle as fo
    o = oracle.query(int(u), int(i))
    b, e = int(offs[j]), int(offs[j + 1])
    assert np.array_equal(o["rel"], rel[b:e])
    s = max(np.abs(o["influence"]).max(initial=0.0), 1e-300)
    assert np.abs(infl[b:e] - o["influence"]).max(initial=0.0) / s < RTOL
    D = o["x"].size
    assert np.abs(x[j * D:(j + 1) * D] - o["x"]).max() / max(np.abs(o["x"]).max(), 1e-300) < RTOL
    return fo


@pytest.fixture(scope="module")
def ml1m_full():
    d = synth.make_dataset(synth.ML1M, seed=0)
    p = synth.mf_params(d["U"], d["I"], 16, 0)
    qu, qi = item_major(d["test"][0], d["test"][1])
    ctx = _ctx("MF", 16, d, p)
    ctx.prepare()
    (b0, b1, o), = list(batches(ctx, qu, qi, 1))
    full = host(o)
    assert (b0, b1) == (0, qu.size)
    return d, p, qu, qi, ctx, full


@pytest.mark.parametrize("shard", range(8))
def test_ml1m_shard_prepare_for_matches_full(ml1m_full, shard):
    """ml-1m-ex shard r of 8: fia_prepare_for (marked Gram stream) == full prepare, bitwise."""
    import torch
    from oracle import fia_oracle as fo
    d, p, qu, qi, ctx, full = ml1m_full
    r0, r1 = shard_bounds("ml1m-mf", d, qu, qi)[shard]
    su, si = qu[r0:r1], qi[r0:r1]
    assert su.size > 0
    dev = torch.device("cuda", 0)
    ctx.prepare_for(torch.from_numpy(su).to(dev), torch.from_numpy(si).to(dev))
    (b0, b1, o), = list(batches(ctx, su, si, 1))
    got = host(o)
    fb, fe = int(full["offs"][r0]), int(full["offs"][r1])
    assert np.array_equal(got["offs"], full["offs"][r0:r1 + 1] - fb)
    assert np.array_equal(got["rel"], full["rel"][fb:fe])
    assert np.array_equal(got["infl"].view(np.int64), full["infl"][fb:fe].view(np.int64))
    D = ctx.num_params()
    assert np.array_equal(got["x"].view(np.int64), full["x"][r0 * D:r1 * D].view(np.int64))
    for key in ("tp", "tix"):
        assert np.array_equal(got[key], full[key][r0:r1]), key
    assert np.array_equal(got["tv"].view(np.int64), full["tv"][r0:r1].view(np.int64))
    # oracle: the shard's heaviest query + 5 random ones
    n = np.diff(got["offs"])
    rng = np.random.default_rng(shard)
    oracle = fo.CsrExact("MF", p, 16, *d["train"], 1e-3, 1e-6)
    for j in [int(np.argmax(n))] + [int(q) for q in rng.choice(su.size, min(5, su.size), replace=False)]:
        oracle_check(oracle, su[j], si[j], got["offs"], got["rel"], got["infl"], got["x"], j)


@pytest.fixture(scope="module")
def data20m():
    os.environ.setdefault("FIA_SYNTH_CACHE", "/tmp/fia_synth")
    return synth.make_20m(seed=0)


@pytest.mark.parametrize("shard", [0, 7])
def test_config4_shard_prepare_for_matches_full(data20m, shard):
    """20M MF k=64 shard r of 8 (the north star's scaling config): a fia_prepare_for context
    and a full-prepare context answer the shard's queries batch by batch with identical bits
    (related rows, influence, x, top-1); oracle sample incl. the shard's heaviest query."""
    import torch
    from oracle import fia_oracle as fo
    d = data20m
    params = synth.mf_params(d["U"], d["I"], 64, 0)
    qu, qi = item_major(d["test"][0], d["test"][1])
    r0, r1 = shard_bounds("20m-mf64", d, qu, qi)[shard]
    su, si = qu[r0:r1], qi[r0:r1]
    dev = torch.device("cuda", 0)
    full_ctx = _ctx("MF", 64, d, params)
    full_ctx.prepare()
    part_ctx = _ctx("MF", 64, d, params)
    part_ctx.prepare_for(torch.from_numpy(su).to(dev), torch.from_numpy(si).to(dev))
    deg_u = np.bincount(d["train"][0], minlength=d["U"])
    deg_i = np.bincount(d["train"][1], minlength=d["I"])
    n_all = deg_u[su] + deg_i[si]
    heavy = int(np.argmax(n_all))
    rng = np.random.default_rng(10 + shard)
    keep = {heavy} | {int(q) for q in rng.choice(su.size, 7, replace=False)}
    oracle = fo.CsrExact("MF", params, 64, *d["train"], 1e-3, 1e-6)
    total = nb = 0
    for (b0, b1, a), (c0, c1, b) in zip(batches(full_ctx, su, si, 1), batches(part_ctx, su, si, 1)):
        assert (b0, b1) == (c0, c1)
        for key in ("offs", "rel", "tp", "tix"):
            assert torch.equal(a[key], b[key]), key
        for key in ("infl", "x", "tv"):
            assert torch.equal(a[key].view(torch.int64), b[key].view(torch.int64)), key
        total += int(b["offs"][-1])
        nb += 1
        mine = [q for q in keep if b0 <= q < b1]
        if mine:
            offs = b["offs"].cpu().numpy()
            D = part_ctx.num_params()
            for q in mine:
                j = q - b0
                s, e = int(offs[j]), int(offs[j + 1])
                sub = np.array([0, e - s])
                oracle_check(oracle, su[q], si[q], sub, b["rel"][s:e].cpu().numpy(), b["infl"][s:e].cpu().numpy(),
                             b["x"][j * D:(j + 1) * D].cpu().numpy(), 0)
    assert total == int(n_all.sum()) and su.size > 20000 and nb >= 1
    print("config 4 shard %d/8: %d queries, %d related ratings, %d batches, oracle sample of %d incl. n = %d"
          % (shard, su.size, total, nb, len(keep), int(n_all[heavy])))
    full_ctx.close()
    part_ctx.close()
    torch.cuda.empty_cache()
