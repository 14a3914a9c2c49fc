"""FIA influence-query throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config ml1m-mf|yelp-ncf|20m-mf64]

A step = one pass of the hot path over one batch: per-entity Hessian caches
(fia_prepare), related-set counts + offsets (fia_count_related), and the
batched query (fia_query_batch: exact solve, every related rating's influence
+ train row, top-1 influencer) over the workload's whole query set, all
resident in HBM.  With N > 1 (torchrun, one rank per GPU) every rank runs the
same-shaped per-GPU batch (weak scaling: rank r > 0 answers the workload's users and
items re-paired by a seeded permutation, so the node answers N distinct query sets) and the
step ends with the RCCL all_gather of the top-K influencer lists.

Rank 0 prints one JSON line.  `roofline` prices the dominant kernel (k_score:
gather + scoring) by SURVEY.md 8d's algorithmic bytes over its HIP-event
duration; `cpu_baseline` times the reference ALGORITHM (oracle/ncg_port.py:
O(N) scans, fmin_ncg with the reference arguments, per-rating gradient loop)
on a bounded sample on this host.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fia-kdd-19_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)

CONFIGS = {
    "ml1m-mf": dict(workload="MF k=16 ml-1m-ex, all 12,074 test ratings (config 2)", model="MF", k=16, data="ml1m"),
    "yelp-ncf": dict(workload="NCF k=16 yelp-ex, all 51,153 test ratings (config 3)", model="NCF", k=16, data="yelp"),
    "20m-mf64": dict(workload="MF k=64 synthetic 20M ratings, 276,986 held-out queries (config 4)", model="MF",
                     k=64, data="20m"),
    "20m-mf256": dict(workload="MF k=256 synthetic 20M ratings, 276,986 held-out queries (config 5, 2 x 257^2 "
                      "blocks per query)", model="MF", k=256, data="20m"),
    "20m-ncf256": dict(workload="NCF k=256 synthetic 20M ratings, 276,986 held-out queries (config 5, 2 x 512^2 "
                       "blocks per query)", model="NCF", k=256, data="20m"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="ml1m-mf", choices=sorted(CONFIGS))
    ap.add_argument("--query-order", default="item", choices=["item", "given"],
                    help="order in which the query set is batched (item-major or the data's order)")
    ap.add_argument("--topk", type=int, default=1)
    ap.add_argument("--batch-rows", type=int, default=1 << 29,
                    help="max related ratings per fia_query_batch call (output buffers are reused)")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="answer only this rank's 1/S share of the query set (contiguous, balanced by n_q): "
                         "with S=8 at N=1 this is one GPU's share of the 8-GPU strong-scaling job")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as one captured HIP graph (measured no faster on MI355X)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rank-set", type=int, default=0,
                    help="answer the query set weak-scaling rank R > 0 answers (check its cost on one GPU)")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="CPU-baseline worker processes (default: usable host cores, at most 16)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "score_traffic.json"))
    return ap.parse_args()


def load_data(cfg):
    from influence import synth
    if cfg["data"] == "ml1m":
        d = synth.make_dataset(synth.ML1M, seed=0)
    elif cfg["data"] == "yelp":
        d = synth.make_dataset(synth.YELP, seed=0)
    else:
        d = synth.make_20m(seed=0)
    k = cfg["k"]
    params = (synth.mf_params if cfg["model"] == "MF" else synth.ncf_params)(d["U"], d["I"], k, 0)
    return d, params


def score_kernel(cfg):
    """The library's scoring kernel for this config (models.hip / bigk.hip schedule choice)."""
    k, model = cfg["k"], cfg["model"]
    if k >= 128 or (model == "NCF" and k >= 64):
        return "k_big_score"
    if model == "NCF":
        return "k_score_ncf"
    return "k_score_mf" if k <= 16 else "k_score_grouped_mf"


def bytes_per_query(model, k, n):
    """SURVEY.md 8d algorithmic bytes per query: MF n(4k+32) + 8k+8; NCF n(8k+32)."""
    n = np.asarray(n, np.float64)
    if model == "MF":
        return n * (4 * k + 32) + 8 * k + 8
    return n * (8 * k + 32)


_CPU = {}     # state the forked CPU-baseline workers inherit


def _cpu_worker(w, P, seconds, barrier, out):
    from oracle import ncg_port
    try:
        from threadpoolctl import threadpool_limits
        threadpool_limits(1)                      # one BLAS thread per worker process
    except Exception:
        pass
    cfg, d, params, order = _CPU["cfg"], _CPU["d"], _CPU["params"], _CPU["order"]
    tu, ti, tr = d["train"]
    qu, qi, _ = d["test"]
    port = ncg_port.RefAlgorithm(cfg["model"], params, cfg["k"], tu, ti, tr, 1e-3, 1e-6)
    mine = order[w::P]
    barrier.wait()
    t0 = time.time()
    done = 0
    for t in mine:
        port.get_influence_on_test_loss(int(qu[t]), int(qi[t]))
        done += 1
        if time.time() - t0 > seconds and done >= 3:
            break
    out.put((done, time.time() - t0))


def rank_query_items(qu, qi, train, I, rank):
    """Weak scaling with distinct units: rank r > 0 answers its own query set of the same
    shape -- the workload's users and items re-paired by a seeded permutation (new (u, i)
    pairs, the same per-user and per-item query counts, so the same related-rating total).
    Like the real held-out pairs, the new pairs are distinct and avoid the training set (a
    pair that is a train row couples the two blocks of its system and takes the full-D
    solve): each offending entry swaps items with a random clean entry when both new pairs
    are clean, until none is left.  Returns the new items."""
    rng = np.random.default_rng(1000 + rank)
    n, I = qi.size, int(I)
    qi = np.ascontiguousarray(qi[rng.permutation(n)])
    tk = np.unique(train[0].astype(np.int64) * I + train[1])
    qu64 = qu.astype(np.int64)

    def in_train(keys):
        if tk.size == 0:
            return np.zeros(keys.shape, bool)
        pos = np.minimum(np.searchsorted(tk, keys), tk.size - 1)
        return tk[pos] == keys

    best, stall = n + 1, 0
    for _ in range(500):
        keys = qu64 * I + qi
        bad = in_train(keys)
        n_train = int(bad.sum())
        first = np.unique(keys, return_index=True)[1]
        dup = np.ones(n, bool)
        dup[first] = False
        bad |= dup
        B = np.nonzero(bad)[0]
        stall = stall + 1 if B.size >= best else 0
        best = min(best, B.size)
        # done when clean; a few duplicate pairs among heavy users may stay (harmless)
        if B.size == 0 or (n_train == 0 and stall >= 20):
            break
        O = rng.integers(0, n, B.size)
        ok = ~bad[O] & ~in_train(qu64[B] * I + qi[O]) & ~in_train(qu64[O] * I + qi[B])
        B, O = B[ok], O[ok]
        keep = np.unique(O, return_index=True)[1]          # one swap per partner
        B, O = B[keep], O[keep]
        qi[B], qi[O] = qi[O], qi[B]
    return qi


def cpu_cores():
    """Host cores this process may use, capped at the GPU box's CPU share (16 per GPU)."""
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(cfg, d, params, seconds, procs):
    """Reference algorithm on the host: `procs` query-parallel worker processes, one
    BLAS thread each, queries dealt round-robin in RQ1 order, time-bounded.  Runs before the
    process touches the GPU (the workers are forked)."""
    import multiprocessing as mp
    from influence import synth
    qu = d["test"][0]
    # the whole test set in RQ1 order (np.random.choice without replacement is prefix-stable,
    # so the first 100 are the RQ1 queries); random order for the synthetic sets
    order = synth.rq1_query_indices(qu.size, qu.size) if cfg["data"] == "ml1m" else \
        np.random.default_rng(0).permutation(qu.size)
    _CPU.update(cfg=cfg, d=d, params=params, order=order)
    ctx = mp.get_context("fork")
    barrier, out = ctx.Barrier(procs), ctx.Queue()
    ws = [ctx.Process(target=_cpu_worker, args=(w, procs, seconds, barrier, out)) for w in range(procs)]
    for p in ws:
        p.start()
    res = [out.get() for _ in ws]
    for p in ws:
        p.join()
    done = sum(r[0] for r in res)
    dt = max(r[1] for r in res)
    return dict(value=done / dt, unit="queries/s", cores=procs, kind="port",
                sample="%d %s queries in %.1f s on %d worker processes x 1 BLAS thread (reference algorithm: "
                       "np.where scans + scipy fmin_ncg avextol=1e-3 maxiter=100 with the verbose callback + "
                       "per-rating gradient loop); %.1f queries/s per core"
                       % (done, "RQ1-order" if cfg["data"] == "ml1m" else "random", dt, procs, done / dt / procs))


def main():
    args = parse()
    cfg = CONFIGS[args.config]
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    d, params = load_data(cfg)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # before anything touches the GPU: the baseline's workers are forked from this process
        cpu = cpu_baseline(cfg, d, params, args.cpu_baseline_seconds, args.cpu_procs or cpu_cores())
    torch.cuda.set_device(dev)

    from influence import _lib
    from influence.sharding import TopKGather, shard_ranges

    tu, ti, tr = d["train"]
    qu_np, qi_np, _ = d["test"]
    qset = rank if world > 1 else args.rank_set
    if qset > 0 and args.shard_of <= 1:
        qi_np = rank_query_items(qu_np, qi_np, d["train"], d["I"], qset)
    if args.query_order == "item":
        # item-major order (ties by user): queries of one item land in the same batch, so the
        # entity-shared scoring loads a long item list once per <= 8 of them.  Per-query
        # results do not depend on the order.
        order = np.lexsort((qu_np, qi_np))
        qu_np, qi_np = np.ascontiguousarray(qu_np[order]), np.ascontiguousarray(qi_np[order])
    U, I, k = d["U"], d["I"], cfg["k"]
    model_id = _lib.FIA_MODEL_MF if cfg["model"] == "MF" else _lib.FIA_MODEL_NCF

    ctx = _lib.Context(local)
    names = list(params)
    tables = [torch.from_numpy(np.ascontiguousarray(params[n], np.float32)).to(dev) for n in names]
    ctx.set_params(model_id, k, U, I, tables, 1e-3, 1e-6)
    t_u = torch.from_numpy(tu).to(dev)
    t_i = torch.from_numpy(ti).to(dev)
    t_r = torch.from_numpy(tr).to(dev)
    t0 = time.time()
    ctx.build_index(t_u, t_i, t_r, U, I)
    torch.cuda.synchronize(dev)
    index_s = time.time() - t0
    qu = torch.from_numpy(qu_np).to(dev)
    qi = torch.from_numpy(qi_np).to(dev)
    offsets_all, _ = ctx.count_related(qu, qi)
    n_q = np.diff(offsets_all.cpu().numpy())
    all_sizes = [int(n_q.size)] * world        # weak scaling: every rank answers one full-size set
    if args.shard_of > 1:
        rs = shard_ranges(n_q, args.shard_of)
        all_sizes = [rs[r % args.shard_of][1] - rs[r % args.shard_of][0] for r in range(world)]
        b0, b1 = rs[rank % args.shard_of]
        qu_np, qi_np, n_q = qu_np[b0:b1], qi_np[b0:b1], n_q[b0:b1]
        qu, qi = qu[b0:b1].contiguous(), qi[b0:b1].contiguous()
    Q = int(qu_np.size)
    total = int(n_q.sum())
    D = ctx.num_params()
    K = args.topk
    # query batches of <= --batch-rows related ratings (output buffers reused batch to batch;
    # ml-1m-ex / yelp-ex fit in one batch)
    cum = np.concatenate([[0], np.cumsum(n_q)])
    bounds = [0]
    while bounds[-1] < Q:
        b0 = bounds[-1]
        b1 = int(np.searchsorted(cum, cum[b0] + args.batch_rows, side="right")) - 1
        bounds.append(min(Q, max(b1, b0 + 1)))
    batches = []
    for b0, b1 in zip(bounds[:-1], bounds[1:]):
        qb_u, qb_i = qu[b0:b1], qi[b0:b1]
        off_b, tot_b = ctx.count_related(qb_u, qb_i)
        batches.append((b0, b1, qb_u, qb_i, off_b, tot_b))
    max_rows = max(b[5] for b in batches)
    max_q = max(b[1] - b[0] for b in batches)
    rel = torch.empty(max_rows, dtype=torch.int64, device=dev)
    infl = torch.empty(max_rows, dtype=torch.float64, device=dev)
    xbuf = torch.empty(max_q * D, dtype=torch.float64, device=dev)
    tp = torch.empty(Q * K, dtype=torch.int64, device=dev)
    tix = torch.empty(Q * K, dtype=torch.int64, device=dev)
    tv = torch.empty(Q * K, dtype=torch.float64, device=dev)

    big_k = k >= 128 or (cfg["model"] == "NCF" and k >= 64)

    # the top-K exchange: one async all_gather per step, overlapped with the next step
    tg = TopKGather(all_sizes, K, dev) if world > 1 else None

    def compute():
        if big_k:
            ctx.prepare_for(qu, qi)    # caches for this GPU's users/items only (fia_prepare_for)
        else:
            ctx.prepare()
        for b0, b1, qb_u, qb_i, off_b, tot_b in batches:
            ctx.count_related(qb_u, qb_i, off_b, want_total=False)
            ctx.query_batch(qb_u, qb_i, off_b, tot_b, rel, infl, xbuf, K, tp[b0 * K:b1 * K],
                            tix[b0 * K:b1 * K], tv[b0 * K:b1 * K])

    def step():
        compute()
        if tg is not None:
            tg.start(tix.view(Q, K), tv.view(Q, K))

    for _ in range(args.warmup):
        step()
    if tg is not None:
        tg.wait()
    torch.cuda.synchronize(dev)
    # per-phase breakdown (informational) from a few instrumented steps; the timed steps
    # below record only the scoring phase's event pair (the roofline kernel time)
    ctx.profile_read()
    ctx.set_profiling(True)
    for _ in range(min(args.steps, 5)):
        compute()
    torch.cuda.synchronize(dev)
    ctx.set_profiling(False)
    phases = ctx.profile_read()
    # the timed steps: the whole step (prepare + related counts + query batches) captured
    # once as a HIP graph and replayed -- every kernel still runs every step; the graph only
    # removes host launch cost and inter-kernel gaps.  fia_prepare_for (large k) decides
    # the cache size on the host, so those configs run eagerly.
    use_graph = args.graph and not big_k
    graph = None
    if use_graph:
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            compute()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            compute()
        torch.cuda.synchronize(dev)

    def timed_step():
        if graph is not None:
            graph.replay()
        else:
            compute()
        if tg is not None:
            tg.start(tix.view(Q, K), tv.view(Q, K))

    ctx.set_profiling(True, phases=("score",))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        timed_step()
    if tg is not None:
        tg.wait()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_profiling(False)
    timed = ctx.profile_read()          # scoring kernel duration over the timed region
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    ms_per_step = elapsed * 1e3 / args.steps
    value = world * Q * args.steps / elapsed
    score_ms = timed["score"][0] / max(timed["score"][1], 1)            # per launch, timed region
    if timed["score"][1] == 0:
        # graph replay: the library's events are not re-recorded by a replayed graph, so the
        # kernel time comes from the instrumented eager steps
        score_ms = phases["score"][0] / max(phases["score"][1], 1)
    bytes_launch = float(bytes_per_query(cfg["model"], k, n_q).sum()) / len(batches)   # mean per launch
    achieved = bytes_launch / (score_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            tj = tj.get(args.config, {}) if "config" not in tj else tj
            if tj.get("config") == args.config and tj.get("kernel", "").startswith(score_kernel(cfg)):
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    out = {
        "metric": "influence queries/sec (whole node) + % HBM roofline, MF k=16 ML-1M-ex"
        if args.config == "ml1m-mf" else "influence queries/sec (whole node), " + cfg["workload"],
        "value": value, "unit": "queries/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak" if args.shard_of <= 1 else "strong", "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic train ratings of the reference shape (train file not distributed) + the reference's "
                "real held-out test pairs; synthetic parameters",
        "config": {"workload": cfg["workload"], "model": cfg["model"], "k": k, "queries_per_gpu": Q,
                   "n_train": int(tu.size), "related_ratings_per_gpu_step": int(total), "topk": K,
                   "query_batches": len(batches), "query_order": args.query_order, "shard_of": args.shard_of,
                   "hip_graph": use_graph,
                   "parallelism": "dp%d (query shards, top-K all_gather)" % world},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": score_kernel(cfg), "kernel_ms": score_ms, "algorithmic_bytes_per_launch": bytes_launch},
        "phases_ms_per_step": {p: (v[0] / max(v[1], 1)) for p, v in phases.items()},
        "index_build_s": index_s,
    }
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
