"""GPU tests at the BASELINE configs' real sizes.

  * config 4 -- synthetic 20M ratings, MF k=64: all 276,986 held-out queries in
    fia_query_batch batches (as bench.py runs them), every batch checked on the GPU;
  * config 5 -- the same ratings, MF k=256 and NCF k=256: all 8 shards of the 8-GPU split
    bench.py runs, caches from fia_prepare_for;
  * config 3 -- yelp-ex NCF k=16: all 51,153 test ratings in one batch.

Size-independent properties, checked for EVERY query with torch on the GPU (the
outputs are too large to copy out): offsets = deg(u) + deg(i); the related list is
R_u's train rows ascending, then C_i's ascending (mf:315-322); influence finite; the
top-1 is the largest |influence| with the lowest related position among ties
(experiments.py:46-48 + the build's tie rule).  Plus an fp64 oracle sample (the
CPU restatement, tolerance 1e-5 relative to the query's max |influence|) that
includes the heaviest item's query and a query whose pair is a training row."""
import os

import numpy as np
import pytest

from influence import synth

pytestmark = pytest.mark.gpu

RTOL = 1e-5
BATCH_ROWS = 1 << 28


@pytest.fixture(scope="module")
def data20m():
    os.environ.setdefault("FIA_SYNTH_CACHE", "/tmp/fia_synth")
    return synth.make_20m(seed=0)


def _ctx(model, k, d, params):
    import torch
    from influence import _lib
    dev = torch.device("cuda", 0)
    ctx = _lib.Context(0)
    names = synth.MF_PARAM_NAMES if model == "MF" else synth.NCF_PARAM_NAMES
    tabs = [torch.from_numpy(np.ascontiguousarray(params[n], np.float32)).to(dev) for n in names]
    ctx.set_params(_lib.FIA_MODEL_MF if model == "MF" else _lib.FIA_MODEL_NCF, k, d["U"], d["I"], tabs, 1e-3, 1e-6)
    tu, ti, tr = d["train"]
    tt = [torch.from_numpy(a).to(dev) for a in (tu, ti, tr)]
    ctx.build_index(tt[0], tt[1], tt[2], d["U"], d["I"])
    ctx._keep_index = tt
    return ctx


class GpuChecker(object):
    """Property checks of one query batch's outputs, on the device."""

    def __init__(self, d):
        import torch
        self.dev = torch.device("cuda", 0)
        tu, ti, _ = d["train"]
        self.tu = torch.from_numpy(tu.astype(np.int64)).to(self.dev)
        self.ti = torch.from_numpy(ti.astype(np.int64)).to(self.dev)
        self.deg_u = torch.bincount(self.tu, minlength=d["U"])
        self.deg_i = torch.bincount(self.ti, minlength=d["I"])

    def check(self, offs, rel, infl, qu, qi, topk_pos, topk_val):
        import torch
        qu, qi = qu.long(), qi.long()
        Qb = qu.numel()
        n = offs[1:] - offs[:-1]
        assert int(offs[0]) == 0
        assert torch.equal(n, self.deg_u[qu] + self.deg_i[qi]), "offsets != deg(u) + deg(i)"
        total = int(offs[-1])
        seg = torch.repeat_interleave(torch.arange(Qb, device=self.dev), n)
        pos = torch.arange(total, device=self.dev) - offs[:-1][seg]
        user_part = pos < self.deg_u[qu][seg]
        r = rel[:total]
        assert bool(torch.all(torch.where(user_part, self.tu[r] == qu[seg], self.ti[r] == qi[seg]))), "foreign row"
        same = (seg[1:] == seg[:-1]) & (user_part[1:] == user_part[:-1])
        assert bool(torch.all((r[1:] > r[:-1]) | ~same)), "related list not ascending"
        v = infl[:total]
        assert bool(torch.isfinite(v).all())
        a = v.abs()
        amax = torch.full((Qb,), -1.0, dtype=torch.float64, device=self.dev).scatter_reduce(0, seg, a, "amax")
        big = torch.iinfo(torch.int64).max
        cand = torch.where(a == amax[seg], pos, torch.full_like(pos, big))
        first = torch.full((Qb,), big, dtype=torch.int64, device=self.dev).scatter_reduce(0, seg, cand, "amin")
        has = n > 0
        assert torch.equal(topk_pos[:, 0][has], first[has]), "top-1 position"
        assert torch.equal(topk_val[:, 0][has], v[offs[:-1][has] + first[has]]), "top-1 value"
        del seg, pos, user_part, same, a, cand
        return total


def run_batches(ctx, qu_np, qi_np, K, checker, keep=()):
    """bench.py's batching (<= BATCH_ROWS related ratings per call); every batch checked.
    Returns the host results of the queries in `keep` (global indices)."""
    import torch
    dev = torch.device("cuda", 0)
    qu = torch.from_numpy(qu_np).to(dev)
    qi = torch.from_numpy(qi_np).to(dev)
    offs_all, _ = ctx.count_related(qu, qi)
    n_q = np.diff(offs_all.cpu().numpy())
    cum = np.concatenate([[0], np.cumsum(n_q)])
    bounds = [0]
    while bounds[-1] < n_q.size:
        b0 = bounds[-1]
        b1 = int(np.searchsorted(cum, cum[b0] + BATCH_ROWS, side="right")) - 1
        bounds.append(min(n_q.size, max(b1, b0 + 1)))
    max_rows = int(max(cum[b1] - cum[b0] for b0, b1 in zip(bounds[:-1], bounds[1:])))
    D = ctx.num_params()
    rel = torch.empty(max_rows, dtype=torch.int32, device=dev)
    infl = torch.empty(max_rows, dtype=torch.float64, device=dev)
    out = {}
    total = 0
    for b0, b1 in zip(bounds[:-1], bounds[1:]):
        qb_u, qb_i = qu[b0:b1].contiguous(), qi[b0:b1].contiguous()
        offs, tot = ctx.count_related(qb_u, qb_i)
        xb = torch.empty((b1 - b0) * D, dtype=torch.float64, device=dev)
        tp = torch.empty((b1 - b0) * K, dtype=torch.int64, device=dev)
        tix = torch.empty_like(tp)
        tv = torch.empty((b1 - b0) * K, dtype=torch.float64, device=dev)
        ctx.query_batch(qb_u, qb_i, offs, tot, rel, infl, xb, K, tp, tix, tv)
        total += checker.check(offs, rel, infl, qb_u, qb_i, tp.view(-1, K), tv.view(-1, K))
        for q in keep:
            if b0 <= q < b1:
                j = q - b0
                s, e = int(offs[j]), int(offs[j + 1])
                out[q] = dict(rel=rel[s:e].cpu().numpy(), influence=infl[s:e].cpu().numpy(),
                              x=xb[j * D:(j + 1) * D].cpu().numpy(), topk_pos=tp[j * K:(j + 1) * K].cpu().numpy())
    assert total == int(cum[-1])
    return out, len(bounds) - 1, n_q


def compare_oracle(model, k, d, params, u, i, got, oracle=None):
    from oracle import fia_oracle as fo
    tu, ti, tr = d["train"]
    o = oracle.query(u, i) if oracle is not None else fo.query(model, params, k, tu, ti, tr, u, i, 1e-3, 1e-6)
    assert np.array_equal(o["rel"], got["rel"])
    s = max(np.abs(o["influence"]).max(initial=0.0), 1e-300)
    assert np.abs(got["influence"] - o["influence"]).max(initial=0.0) / s < RTOL
    sx = max(np.abs(o["x"]).max(), 1e-300)
    assert np.abs(got["x"] - o["x"]).max() / sx < RTOL
    want = fo.topk(o["influence"], 1)
    if want.size and got["topk_pos"][0] != want[0]:
        a = np.abs(o["influence"])     # near-tie: flagged, not failed
        assert abs(a[got["topk_pos"][0]] - a[want[0]]) <= 1e-12 * a.max()


def _train_pair_query(d):
    """A training pair (the heaviest user's first train row): its rel holds the pair twice
    and its Hessian couples the user and item blocks."""
    tu, ti, _ = d["train"]
    u = int(np.argmax(np.bincount(tu)))
    j = int(np.nonzero(tu == u)[0][0])
    return u, int(ti[j])


def test_config4_mf64_all_queries(data20m):
    """Config 4: MF k=64, all 276,986 held-out queries of the 20M set, every batch checked;
    oracle sample with the heaviest item's query, random queries and a train-pair query."""
    import torch
    from oracle import fia_oracle as fo
    d = data20m
    params = synth.mf_params(d["U"], d["I"], 64, 0)
    ctx = _ctx("MF", 64, d, params)
    ctx.prepare()
    qu, qi, _ = d["test"]
    order = np.lexsort((qu, qi))                       # bench.py's item-major batching
    qu, qi = np.ascontiguousarray(qu[order]), np.ascontiguousarray(qi[order])
    deg_i = np.bincount(d["train"][1], minlength=d["I"])
    deg_u = np.bincount(d["train"][0], minlength=d["U"])
    heavy = int(np.argmax(deg_i[qi]))
    # >= 200 oracle queries spread over every batch: 9 per batch of the bench's batching
    cum = np.concatenate([[0], np.cumsum(deg_u[qu] + deg_i[qi])])
    starts = [0]
    while starts[-1] < qu.size:
        b0 = starts[-1]
        starts.append(min(qu.size, max(int(np.searchsorted(cum, cum[b0] + BATCH_ROWS, side="right")) - 1, b0 + 1)))
    rng = np.random.default_rng(0)
    keep = [heavy] + [int(q) for b0, b1 in zip(starts[:-1], starts[1:])
                      for q in rng.choice(np.arange(b0, b1), min(9, b1 - b0), replace=False)]
    checker = GpuChecker(d)
    got, nb, n_q = run_batches(ctx, qu, qi, 1, checker, keep)
    assert qu.size == 276986 and nb > 1 and n_q.sum() > 1e10
    assert nb == len(starts) - 1 and len(set(keep)) >= 200, (nb, len(set(keep)))
    oracle = fo.CsrExact("MF", params, 64, *d["train"], 1e-3, 1e-6)
    for q in keep:
        compare_oracle("MF", 64, d, params, int(qu[q]), int(qi[q]), got[q], oracle)
    # a pair that is itself a train row (full-D coupled solve)
    u, i = _train_pair_query(d)
    g2, _, _ = run_batches(ctx, np.array([u, 0], np.int32), np.array([i, 0], np.int32), 1, checker, [0])
    compare_oracle("MF", 64, d, params, u, i, g2[0], oracle)
    ctx.close()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("shard", range(8))
@pytest.mark.parametrize("model", ["MF", "NCF"])
def test_config5_k256_shard(data20m, model, shard):
    """Config 5: k=256 (MF 2 x 257^2, NCF 2 x 512^2 blocks per query) on every shard of
    the 8-GPU split bench.py runs (n_q + the config's per-query cost, shard_ranges), caches from
    fia_prepare_for; every batch checked on the GPU; an fp64 oracle sample of >= 16 queries per
    shard: the shard's heaviest query (no size cap: the heaviest of any shard has ~122 k related
    ratings), its lightest, 13 random ones and a train-pair query of a shard user (coupled
    full-D system)."""
    import torch
    import bench
    from influence.sharding import shard_ranges
    from oracle import fia_oracle as fo
    d = data20m
    k = 256
    params = (synth.mf_params if model == "MF" else synth.ncf_params)(d["U"], d["I"], k, 0)
    ctx = _ctx(model, k, d, params)
    qu, qi, _ = d["test"]
    order = np.lexsort((qu, qi))
    qu, qi = np.ascontiguousarray(qu[order]), np.ascontiguousarray(qi[order])
    deg_u = np.bincount(d["train"][0], minlength=d["U"])
    deg_i = np.bincount(d["train"][1], minlength=d["I"])
    cost = bench.CONFIGS["20m-%s256" % model.lower()]["query_cost"]
    b0, b1 = shard_ranges(deg_u[qu] + deg_i[qi] + cost, 8)[shard]
    su, si = qu[b0:b1], qi[b0:b1]
    # a train-pair query of a shard user, appended (its item joins the cached set)
    tu, ti, _ = d["train"]
    j = int(np.nonzero(tu == su[0])[0][0])
    su = np.append(su, np.int32(tu[j]))
    si = np.append(si, np.int32(ti[j]))
    dev = torch.device("cuda", 0)
    ctx.prepare_for(torch.from_numpy(su).to(dev), torch.from_numpy(si).to(dev))
    n = deg_u[su] + deg_i[si]
    heavy, light = int(np.argmax(n[:-1])), int(np.argmin(n[:-1]))
    rng = np.random.default_rng(1 + shard)
    rest = np.setdiff1d(np.arange(su.size - 1), [heavy, light])
    keep = [heavy, light, su.size - 1] + [int(q) for q in rng.choice(rest, 13, replace=False)]
    got, nb, n_q = run_batches(ctx, su, si, 1, GpuChecker(d), keep)
    assert su.size > 12000 and n_q.sum() > 5e8 and len(set(keep)) == 16
    oracle = fo.CsrExact(model, params, k, *d["train"], 1e-3, 1e-6)
    for q in keep:
        compare_oracle(model, k, d, params, int(su[q]), int(si[q]), got[q], oracle)
    print("config 5 %s shard %d/8: %d queries, %d batches, oracle sample of %d incl. the heaviest (n = %d)"
          % (model, shard, su.size, nb, len(keep), int(n[heavy])))
    ctx.close()
    torch.cuda.empty_cache()


def test_config3_yelp_ncf_all_queries():
    """Config 3: NCF k=16 on yelp-ex, all 51,153 test ratings in one batch (the bench
    workload), properties for every query and an oracle sample incl. the heaviest item."""
    import torch
    d = synth.make_dataset(synth.YELP, seed=0)
    params = synth.ncf_params(d["U"], d["I"], 16, 0)
    ctx = _ctx("NCF", 16, d, params)
    ctx.prepare()
    qu, qi, _ = d["test"]
    assert qu.size == 51153
    deg_i = np.bincount(d["train"][1], minlength=d["I"])
    heavy = int(np.argmax(deg_i[qi]))
    rng = np.random.default_rng(2)
    keep = [heavy] + [int(q) for q in rng.choice(qu.size, 2000, replace=False)]
    got, nb, n_q = run_batches(ctx, qu, qi, 1, GpuChecker(d), keep)
    assert nb == 1 and len(set(keep)) >= 2000
    from oracle import fia_oracle as fo
    oracle = fo.CsrExact("NCF", params, 16, *d["train"], 1e-3, 1e-6)
    for q in keep:
        compare_oracle("NCF", 16, d, params, int(qu[q]), int(qi[q]), got[q], oracle)
    ctx.close()
    torch.cuda.empty_cache()
