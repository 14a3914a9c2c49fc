"""FIA influence-query throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config ml1m-mf|yelp-ncf|20m-mf64|20m-mf256|20m-ncf256]

A step = one pass of the hot path over one batch: per-entity Hessian caches
(fia_prepare / fia_prepare_for), related-set counts + offsets (fia_count_related),
and the batched query (fia_query_batch: exact solve, every related rating's
influence + train row, top-1 influencer) over the rank's whole query set, all
resident in HBM.

Multi-GPU (one process per GPU).  `--gpus N` without a launcher
re-launches this script under torch.distributed.run with N ranks before anything
touches the GPU; under torchrun (the driver) WORLD_SIZE/RANK/LOCAL_RANK are read
from the environment.  Scaling (`--scaling`; the sub-ms ml-1m-ex / yelp-ex steps default to
weak -- every rank answers a full-size query set, per-GPU work fixed as N grows -- and the
20M configs, whose test queries the north star shards across the GPUs, to strong):
  * strong: the config's fixed query set is split into N contiguous ranges balanced
    by n_q + query_cost (the related-set size plus a per-query fixed cost, CONFIGS;
    influence.sharding.shard_ranges); every rank answers its range.  On one GPU, `--shard-of S --shard-index r` answers range r
    of an S-way split (one rank's share of an S-GPU job);
  * weak: every rank answers one full-size query set -- rank 0 the workload's own
    pairs, rank r > 0 the same users and item multiset re-paired by a seeded
    permutation (distinct pairs, none a training row).  A 1/8 strong split of the
    0.1 ms ml-1m-ex step leaves each rank its fixed costs (the Gram pass is
    latency-bound: a shard's marked pass takes as long as the full one), so that
    split cannot scale (profiles/round6_shards.md).
The only exchange is the RCCL all_gather of the per-query top-K lists, overlapped
with the next step.

Batches in flight (`--inflight L`, default 2 for the sub-ms ml-1m-ex / yelp-ex steps): the
steps alternate over L library contexts, each with its own index, caches, scratch and output
buffers, each on its own HIP stream -- a serving pipeline's two query batches in flight, so
one step's kernel ramps and tails overlap the next step's kernels.  Every timed step still
runs the whole hot path over the whole batch; the timed region is still K steps between two
synchronisations.  `value` = queries answered by all ranks / the max-over-ranks
time of the timed steps.

Rank 0 prints one JSON line.  `roofline` prices the step's dominant phase (from a few
instrumented steps): the scoring phase against HBM -- `achieved` = its kernel's HBM
bytes per launch measured by rocprofv3 PMC (FETCH_SIZE x 2 + WRITE_SIZE,
MI355X_MICROARCH.md's gfx950 correction; profiles/traffic.json, tools/traffic_json.py)
over its HIP-event duration in this run, `frac` = achieved / 8 TB/s, with SURVEY 8d's
algorithmic byte count beside it under `algorithmic` -- or a solve / prepare phase
against the FP64 peak (algorithmic flops over its event time).
`cpu_baseline` times the reference ALGORITHM (oracle/ncg_port.py) on a bounded
sample on this host, with two more CPU figures under `variants`.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fia-kdd-19_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFS = 78.6       # MI355X dense FP64 (vector and matrix; tools/mb_f64.hip measures ~70)

# query_cost: a query's fixed work (its solve, chunk lists and share of the Gram pass) in units
# of one related rating's scoring time, for the strong-scaling split (n_q + query_cost per
# query); from the round-4 per-phase timings: e.g. 20M MF k=64 61 ns per
# query over 6.0 ps per scored rating; 20M MF k=64 refitted in round 6 from the 8 shards' steps at
# HEAD (step = 5.83 ps per related rating + 90.7 ns per query, fit residual < 0.1 ms)
CONFIGS = {
    "ml1m-mf": dict(workload="MF k=16 ml-1m-ex, all 12,074 test ratings (config 2)", model="MF", k=16, data="ml1m",
                    scaling="weak", query_cost=560, inflight=2),
    "yelp-ncf": dict(workload="NCF k=16 yelp-ex, all 51,153 test ratings (config 3)", model="NCF", k=16, data="yelp",
                     scaling="weak", query_cost=210, inflight=2),
    "20m-mf64": dict(workload="MF k=64 synthetic 20M ratings, 276,986 held-out queries (config 4)", model="MF",
                     k=64, data="20m", scaling="strong", query_cost=15600),
    "20m-mf256": dict(workload="MF k=256 synthetic 20M ratings, 276,986 held-out queries (config 5, 2 x 257^2 "
                      "blocks per query)", model="MF", k=256, data="20m", scaling="strong", query_cost=150000),
    "20m-ncf256": dict(workload="NCF k=256 synthetic 20M ratings, 276,986 held-out queries (config 5, 2 x 512^2 "
                       "blocks per query)", model="NCF", k=256, data="20m", scaling="strong", query_cost=310000),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="ml1m-mf", choices=sorted(CONFIGS))
    ap.add_argument("--scaling", default="auto", choices=["auto", "weak", "strong"],
                    help="N > 1: strong = split the config's query set over the ranks (auto, every config); "
                         "weak = a full-size set per rank, ranks > 0 answering SYNTHETIC re-paired queries")
    ap.add_argument("--query-order", default="item", choices=["item", "given"],
                    help="order in which the query set is batched (item-major or the data's order)")
    ap.add_argument("--topk", type=int, default=1)
    ap.add_argument("--batch-rows", type=int, default=1 << 29,
                    help="max related ratings per fia_query_batch call (output buffers are reused)")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="answer only one shard of S of the strong-scaling split (with S=8 at N=1: one GPU's share "
                         "of the 8-GPU job)")
    ap.add_argument("--shard-index", type=int, default=0,
                    help="with --shard-of S at N=1: which shard (0 .. S-1) to answer")
    ap.add_argument("--inflight", type=int, default=0,
                    help="query batches in flight: steps alternate over this many contexts, each on its own "
                         "stream with its own caches and outputs, so one step's kernel ramp and tail overlap "
                         "the next step's kernels (every step still runs the whole hot path); 0 = the config's "
                         "default (2 for the sub-ms ml-1m-ex / yelp-ex steps, else 1)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as one captured HIP graph (measured no faster on MI355X)")
    ap.add_argument("--no-timed-events", action="store_true",
                    help="A/B only: no HIP-event pair around the scoring kernel in the timed steps (the "
                         "roofline then falls back to the instrumented steps' kernel time); the pair costs "
                         "~4 us per ml-1m-ex step")
    ap.add_argument("--spinup-seconds", type=float, default=None,
                    help="untimed steps for at least this long before the warmup (default: 20 for the 20M configs, "
                         "6 otherwise): a fresh MI355X runs the HBM-heavy scoring kernels ~15 %% slower for its "
                         "first ~30 s of load, and the sub-ms ml-1m-ex / yelp-ex steps ~4 %% slower over the "
                         "driver's 5 + 20 steps than after 1 s of load (same-box A/B, tools/evt_ab.sh)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rank-set", type=int, default=0,
                    help="answer the query set weak-scaling rank R > 0 answers (check its cost on one GPU)")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="CPU-baseline worker processes (default: usable host cores, at most 16)")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="auto: nccl (RCCL) when every rank has a GPU of its own, gloo when ranks share one")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--rq2", action="store_true",
                    help="RQ2 single-query latency instead of the throughput line: ml-1m-ex test_idx 59 and "
                         "yelp-ex test_idx 1, MF and NCF k=16 (reference src/scripts/RQ2.py:53,57), GPU through "
                         "the facade beside the reference algorithm's CPU time for the same query")
    return ap.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args):
    """--gpus N > 1 outside a launcher: run this script under torch.distributed.run with N
    ranks (a child process, started before this process touches the GPU) and return its
    exit code; None when this process is already a rank (or N == 1)."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


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


def solve_kernel(cfg):
    """The library's side-system solve for this config (models.hip query_impl's use_quad_solve /
    use_tps / pair_layout / use_col_solve / use_tile_solve, bigk.hip query_big_impl)."""
    k, model = cfg["k"], cfg["model"]
    if k >= 128 or (model == "NCF" and k >= 64):
        return "k_bs_trail"              # batched blocked LDL^T panels (+ k_bs_dupd/dfac/back)
    if model == "MF" and k == 16:
        return "k_solve_quad"            # a quad of lanes per side system
    if model == "MF" and k <= 8:
        return "k_solve_tps"             # a thread per side system
    if model == "NCF" and k == 16:
        return "k_solve_rows"            # (+ k_ncf_query_pro, the thread-per-query MLP prologue)
    if model == "NCF" and k == 8:
        return "k_solve_col"
    return "k_solve_tile"


def prepare_kernel(cfg):
    """The library's Gram pass for this config (models.hip prepare_impl, bigk.hip prepare_big).
    MF k <= 16 is two kernels: the Gram stream and the combine of sliced lists' partial Grams
    (traffic.json holds their sum per step as the "prepare_phase" entry)."""
    k, model = cfg["k"], cfg["model"]
    if k >= 128 or (model == "NCF" and k >= 64):
        return "k_big_gram"
    if model == "NCF":
        return "k_ncf_gram_rows"
    # k in {32, 64}: the Gram pass also writes the list-ordered residuals k_score_mf_mfma reads
    return "k_gram_mf_stream + k_gram_combine" if k <= 16 else "k_gram_mf_mfma"


def side_dim(model, k):
    """Coordinates of one side block of H_t: MF k + 1, NCF 2k."""
    return k + 1 if model == "MF" else 2 * k


def solve_flops(model, k, Q):
    """Algorithmic FP64 flops of the exact solve of Q queries: two side systems of D_s
    coordinates each, LDL^T (D^3/3 multiply-adds) + forward and backward solves (D^2)."""
    Dd = float(side_dim(model, k))
    return 2.0 * Q * (2.0 * Dd ** 3 / 3.0 + 2.0 * Dd * Dd)


def prepare_flops(model, k, rows):
    """Entity Gram caches: per list entry (a rating in its user's or its item's list) a
    symmetric rank-1 update, D_s(D_s+1)/2 multiply-adds (+ for NCF the ~12 k^2 flops of the
    per-rating MLP).  rows = the list entries of the cached entities: 2N for the
    full prepare, the marked users' and items' list lengths for a shard's fia_prepare_for."""
    Dd = float(side_dim(model, k))
    per = Dd * (Dd + 1.0) + (12.0 * k * k if model == "NCF" else 0.0)
    return float(rows) * per


def score_kernel(cfg, K=1):
    """The library's scoring kernel for this config (the dispatch in models.hip query_impl /
    bigk.hip query_big_impl: one kernel per (model, k, top-K))."""
    k, model = cfg["k"], cfg["model"]
    if k >= 128 or (model == "NCF" and k >= 64):
        return "k_big_score_mfma"
    if model == "NCF":
        return "k_score_ncf_runs" if k <= 16 else "k_score_ncf"
    if k <= 16:
        return "k_score_mf_runs"
    if K <= 1:
        return "k_score_mf_mfma"
    return "k_score_grouped_mf"


def bytes_per_query(model, k, n):
    """SURVEY.md 8d algorithmic bytes per query, with the train-row output as int32 (4 B, not
    the survey's 8 B): MF n(4k+28) + 8k+8; NCF n(8k+28).  Counts the gathered rows once per
    query (the entity-shared kernels load them once per query block)."""
    n = np.asarray(n, np.float64)
    if model == "MF":
        return n * (4 * k + 28) + 8 * k + 8
    return n * (8 * k + 28)


_CPU = {}     # state the forked CPU-baseline workers inherit


def _cpu_worker(kind, w, P, seconds, barrier, out, blas_threads):
    try:
        from threadpoolctl import threadpool_limits
        threadpool_limits(blas_threads)
    except Exception:
        pass
    qu, qi, _ = _CPU["d"]["test"]
    algo = _CPU["port"] if kind == "port" else _CPU["exact"]
    mine = _CPU["order"][w::P]
    barrier.wait()
    t0 = time.time()
    done = 0
    for t in mine:
        if kind == "port":
            algo.get_influence_on_test_loss(int(qu[t]), int(qi[t]))
        else:
            algo.query(int(qu[t]), int(qi[t]))
        done += 1
        if time.time() - t0 > seconds:
            break
    out.put((done, time.time() - t0))


def _cpu_run(kind, procs, seconds, blas_threads):
    import multiprocessing as mp
    ctx = mp.get_context("fork")
    barrier, out = ctx.Barrier(procs), ctx.Queue()
    ws = [ctx.Process(target=_cpu_worker, args=(kind, w, procs, seconds, barrier, out, blas_threads))
          for w in range(procs)]
    for p in ws:
        p.start()
    res = [out.get() for _ in ws]
    for p in ws:
        p.join()
    done = sum(r[0] for r in res)
    dt = max(r[1] for r in res)
    return done, dt


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def cpu_cores():
    """Host cores this process may use, capped at the GPU box's CPU share (16 per GPU)."""
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(cfg, d, params, seconds, procs):
    """CPU figures on this host, all forked before the
    process touches the GPU, each time-bounded (at least one query per worker):
      headline -- the reference ALGORITHM (np.where scans, scipy fmin_ncg with the reference
                  arguments and verbose callback, per-rating gradient loop; oracle/ncg_port.py)
                  on `procs` query-parallel processes x 1 BLAS thread;
      variants -- the same algorithm in ONE process with `procs` BLAS threads, and the
                  vectorized exact fp64 solve over a CSR index (oracle.CsrExact) on `procs`
                  processes."""
    from influence import synth
    from oracle import ncg_port, fia_oracle
    tu, ti, tr = d["train"]
    qu = d["test"][0]
    # the whole test set in RQ1 order (np.random.choice without replacement is prefix-stable,
    # so the first 100 are the RQ1 queries); random order for the synthetic sets
    order = synth.rq1_query_indices(qu.size, qu.size) if cfg["data"] == "ml1m" else \
        np.random.default_rng(0).permutation(qu.size)
    _CPU.update(d=d, order=order,
                port=ncg_port.RefAlgorithm(cfg["model"], params, cfg["k"], tu, ti, tr, 1e-3, 1e-6),
                exact=fia_oracle.CsrExact(cfg["model"], params, cfg["k"], tu, ti, tr, 1e-3, 1e-6))
    sample = "RQ1-order" if cfg["data"] == "ml1m" else "random"
    done, dt = _cpu_run("port", procs, seconds, 1)
    head = dict(value=done / dt, unit="queries/s", cores=procs, kind="port", cpu=cpu_model(),
                sample="%d %s queries in %.1f s on %d worker processes x 1 BLAS thread (reference algorithm: "
                       "np.where scans + scipy fmin_ncg avextol=1e-3 maxiter=100 with the verbose callback + "
                       "per-rating gradient loop, oracle/ncg_port.py); %.2f queries/s per core"
                       % (done, sample, dt, procs, done / dt / procs))
    var = []
    s2 = max(3.0, seconds / 2)
    done, dt = _cpu_run("port", 1, s2, procs)
    var.append(dict(name="reference algorithm, 1 process x %d BLAS threads" % procs, value=done / dt,
                    unit="queries/s", cores=procs, sample="%d %s queries in %.1f s" % (done, sample, dt)))
    done, dt = _cpu_run("exact", procs, s2, 1)
    var.append(dict(name="exact fp64 solve + vectorized scoring over a CSR index (oracle.CsrExact), "
                         "%d processes x 1 BLAS thread" % procs, value=done / dt, unit="queries/s", cores=procs,
                    sample="%d %s queries in %.1f s" % (done, sample, dt)))
    head["variants"] = var
    return head


def rank_query_items(qu, qi, train, I, rank, stats=None):
    """Weak scaling with distinct units: rank r > 0 answers its own query set of the same
    shape -- the workload's users and items re-paired by a seeded permutation (new (u, i)
    pairs, the same per-user and per-item query counts, so the same related-rating total).
    Like the real held-out pairs, the new pairs are distinct and avoid the training set (a
    pair that is a train row couples the two blocks of its system and takes the full-D
    solve): each offending entry swaps items with a random clean entry when both new pairs
    are clean, until none is left.  Returns the new items; `stats` (a dict) receives the
    pairs still in train / duplicated if the swaps could not remove them all."""
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

    def duplicated(keys):
        first = np.unique(keys, return_index=True)[1]
        dup = np.ones(n, bool)
        dup[first] = False
        return dup

    best, stall = n + 1, 0
    for _ in range(500):
        keys = qu64 * I + qi
        bad = in_train(keys)
        n_train = int(bad.sum())
        bad |= duplicated(keys)
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
    keys = qu64 * I + qi
    left_train, left_dup = int(in_train(keys).sum()), int(duplicated(keys).sum())
    if left_train:
        print("bench: rank %d query set keeps %d training pairs (full-D coupled solves)" % (rank, left_train),
              file=sys.stderr)
    if stats is not None:
        stats.update(train_pairs=left_train, duplicate_pairs=left_dup)
    return qi


def load_traffic(path, config, kernel):
    """PMC HBM bytes per launch of `kernel` for `config`, or None.  profiles/traffic.json:
    {config: {kernel: entry}} (tools/traffic_json.py); the round-2 layout {config: entry}
    is read too."""
    if not os.path.exists(path):
        return None
    try:
        tj = json.load(open(path)).get(config, {})
        if tj.get("kernel") == kernel:
            return tj
        e = tj.get(kernel)
        return e if isinstance(e, dict) and e.get("kernel") == kernel else None
    except Exception:
        return None


def compulsory_bytes(cfg, qu, qi, deg_u, deg_i, bounds):
    """Bytes the scoring kernel cannot avoid, per launch (mean over the batches): its outputs
    (8 B influence + 4 B train row per related rating) and every list entry of the batch's
    users and items read once (4 B row + 4 B other id + 4 B rating; MF k in {32, 64}: the 8 B
    list-ordered residual k_score_mf_mfma reads instead of the rating)."""
    ent = 16.0 if cfg["model"] == "MF" and cfg["k"] in (32, 64) else 12.0
    tot = 0.0
    for b0, b1 in zip(bounds[:-1], bounds[1:]):
        u, i = qu[b0:b1], qi[b0:b1]
        out = 12.0 * float(deg_u[u].sum() + deg_i[i].sum())
        lists = ent * float(deg_u[np.unique(u)].sum() + deg_i[np.unique(i)].sum())
        tot += out + lists
    return tot / max(len(bounds) - 1, 1)


def rq2_main(args):
    """RQ2 (reference src/scripts/RQ2.py, experiments.record_time_cost): the latency of ONE
    query -- ml-1m-ex test_idx 59, yelp-ex test_idx 1, MF and NCF k=16 -- as the reference times
    it (get_influence_on_test_loss: related set, inverse HVP, per-rating influence), GPU through
    the facade (fia-kdd-19_amd/scripts/RQ2.py: median of 5 calls after a warm-up; the three stage
    timers from the call's HIP events and the call's host wall time), beside the reference
    ALGORITHM on this host's CPU for the same query (oracle/ncg_port.py: np.where scans + scipy
    fmin_ncg with the reference arguments + the per-rating gradient loop; one process, BLAS
    threads = the usable cores; median of 3).  The CPU runs first, before the GPU is touched."""
    from influence import synth
    from oracle import ncg_port
    cases = []
    for data, test_idx in (("ml1m", 59), ("yelp", 1)):
        d = synth.make_dataset(synth.ML1M if data == "ml1m" else synth.YELP, seed=0)
        tu, ti, tr = d["train"]
        u, i = int(d["test"][0][test_idx]), int(d["test"][1][test_idx])
        for model in ("MF", "NCF"):
            params = (synth.mf_params if model == "MF" else synth.ncf_params)(d["U"], d["I"], 16, 0)
            ref = ncg_port.RefAlgorithm(model, params, 16, tu, ti, tr, 1e-3, 1e-6)
            from threadpoolctl import threadpool_limits
            ts = []
            with threadpool_limits(cpu_cores()):
                for _ in range(3):
                    t0 = time.perf_counter()
                    ref.get_influence_on_test_loss(u, i)
                    ts.append(time.perf_counter() - t0)
            cases.append(dict(dataset="ml-1m-ex" if data == "ml1m" else "yelp-ex", model=model, test_idx=test_idx,
                              user=u, item=i, cpu_reference_algorithm_s=float(np.median(ts)), cpu_cores=cpu_cores()))
    import torch
    torch.cuda.set_device(0)
    from scripts import RQ2
    from scripts.load_movielens import load_movielens_synthetic
    from scripts.load_yelp import load_yelp_synthetic
    import tempfile
    tmp = tempfile.mkdtemp(prefix="rq2_")
    cfg = dict(RQ2.configs)
    for c in cases:
        ds = load_movielens_synthetic(0) if c["dataset"] == "ml-1m-ex" else load_yelp_synthetic(0)
        m = RQ2.build("movielens" if c["dataset"] == "ml-1m-ex" else "yelp", c["model"], cfg, ds, train_dir=tmp)
        g = RQ2.time_query(m, c["test_idx"], cfg["repeat"])
        m.ctx.close()
        c.update(n_related=g["n"], gpu_inverse_hvp_s=g["inverse_hvp_s"], gpu_multiply_s=g["multiply_s"],
                 gpu_total_s=g["total_s"], gpu_wall_s=g["wall_s"],
                 speedup_wall=c["cpu_reference_algorithm_s"] / g["wall_s"])
    print(json.dumps({"metric": "RQ2 single-query latency (seconds), reference src/scripts/RQ2.py",
                      "higher_is_better": False, "cpu": cpu_model(), "cases": cases}), flush=True)


def main():
    args = parse()
    if args.rq2:
        return rq2_main(args)
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    cfg = CONFIGS[args.config]
    scaling = cfg["scaling"] if args.scaling == "auto" else args.scaling
    if args.shard_of > 1 and args.scaling == "auto":
        scaling = "strong"      # one rank's share of an S-way split of the query set
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus not in (1, world):
        print("bench: --gpus %d but WORLD_SIZE=%d; using WORLD_SIZE" % (args.gpus, world), file=sys.stderr)

    d, params = load_data(cfg)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # before anything touches the GPU: the baseline's workers are forked from this process
        cpu = cpu_baseline(cfg, d, params, args.cpu_baseline_seconds, args.cpu_procs or cpu_cores())

    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))
    backend = args.dist_backend
    if backend == "auto":
        backend = "nccl" if world <= ndev else "gloo"
    if world > 1:
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(dev)

    from influence import _lib
    from influence.sharding import TopKGather, shard_ranges

    tu, ti, tr = d["train"]
    qu_np, qi_np, _ = d["test"]
    repair = {}
    qset = rank if (world > 1 and scaling == "weak") else args.rank_set
    if qset > 0 and args.shard_of <= 1:
        qi_np = rank_query_items(qu_np, qi_np, d["train"], d["I"], qset, repair)
    if args.query_order == "item":
        # item-major order (ties by user): queries of one item land in the same batch, so the
        # entity-shared scoring loads a long item list once per query block.  Per-query
        # results do not depend on the order.
        order = np.lexsort((qu_np, qi_np))
        qu_np, qi_np = np.ascontiguousarray(qu_np[order]), np.ascontiguousarray(qi_np[order])
    U, I, k = d["U"], d["I"], cfg["k"]
    model_id = _lib.FIA_MODEL_MF if cfg["model"] == "MF" else _lib.FIA_MODEL_NCF

    ctx = _lib.Context(dev.index)
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
    # this rank's queries and every rank's count
    if scaling == "strong" and (world > 1 or args.shard_of > 1):
        S = world if world > 1 else args.shard_of
        rs = shard_ranges(n_q + cfg["query_cost"], S)
        all_sizes = [b - a for a, b in rs][:world] if world > 1 else [rs[0][1] - rs[0][0]]
        if world == 1 and not 0 <= args.shard_index < S:
            raise SystemExit("bench: --shard-index %d outside 0 .. %d" % (args.shard_index, S - 1))
        b0, b1 = rs[rank if world > 1 else args.shard_index]
        if world == 1:
            all_sizes = [b1 - b0]
        qu_np, qi_np, n_q = qu_np[b0:b1], qi_np[b0:b1], n_q[b0:b1]
        qu, qi = qu[b0:b1].contiguous(), qi[b0:b1].contiguous()
        shard_of = S
    else:
        all_sizes = [int(n_q.size)] * world
        shard_of = 1
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
    max_rows = max([b[5] for b in batches] + [1])
    max_q = max([b[1] - b[0] for b in batches] + [1])

    def lane_state(c, bat):
        return dict(ctx=c, batches=bat,
                    rel=torch.empty(max_rows, dtype=torch.int32, device=dev),
                    infl=torch.empty(max_rows, dtype=torch.float64, device=dev),
                    xbuf=torch.empty(max_q * D, dtype=torch.float64, device=dev),
                    tp=torch.empty(max(Q * K, 1), dtype=torch.int64, device=dev),
                    tix=torch.empty(max(Q * K, 1), dtype=torch.int64, device=dev),
                    tv=torch.empty(max(Q * K, 1), dtype=torch.float64, device=dev))

    # --inflight L: L contexts (own index, caches, scratch and outputs) on L streams
    lanes = [lane_state(ctx, batches)]
    streams = [torch.cuda.current_stream(dev)]
    n_inflight = args.inflight if args.inflight > 0 else cfg.get("inflight", 1)
    for _ in range(1, max(1, n_inflight)):
        c2 = _lib.Context(dev.index)
        c2.set_params(model_id, k, U, I, tables, 1e-3, 1e-6)
        c2.build_index(t_u, t_i, t_r, U, I)
        bat2 = [(b0, b1, qb_u, qb_i, c2.count_related(qb_u, qb_i)[0], tot_b)
                for b0, b1, qb_u, qb_i, _, tot_b in batches]
        lanes.append(lane_state(c2, bat2))
        streams.append(torch.cuda.Stream(device=dev))
    torch.cuda.synchronize(dev)
    rel, infl, xbuf, tp, tix, tv = (lanes[0][n] for n in ("rel", "infl", "xbuf", "tp", "tix", "tv"))

    big_k = k >= 128 or (cfg["model"] == "NCF" and k >= 64)

    # the top-K exchange: one async all_gather per step, overlapped with the next step (gloo:
    # host copies of the lists, for rehearsals with several ranks on one GPU)
    gdev = dev if backend == "nccl" else torch.device("cpu")
    tg = TopKGather(all_sizes, K, gdev) if world > 1 else None

    # a rank answering a shard of the query set builds only its users'/items' caches
    # (fia_prepare_for; small k: marked on the device, no host round trip); the full set
    # builds every cache
    sharded = shard_of > 1
    step_no = [0]

    def compute_lane(L):
        c = L["ctx"]
        if big_k or sharded:
            c.prepare_for(qu, qi)
        else:
            c.prepare()
        for b0, b1, qb_u, qb_i, off_b, tot_b in L["batches"]:
            c.count_related(qb_u, qb_i, off_b, want_total=False)
            c.query_batch(qb_u, qb_i, off_b, tot_b, L["rel"], L["infl"], L["xbuf"], K, L["tp"][b0 * K:b1 * K],
                          L["tix"][b0 * K:b1 * K], L["tv"][b0 * K:b1 * K])

    def compute():
        j = step_no[0] % len(lanes)
        step_no[0] += 1
        if j == 0:
            compute_lane(lanes[0])
        else:
            with torch.cuda.stream(streams[j]):
                compute_lane(lanes[j])
        return j

    def exchange(j=0):
        if tg is None:
            return
        # on the lane's own stream: the pack (and, with RCCL, the collective's enqueue) is
        # ordered after that lane's kernels, without making the other lane's stream wait
        with torch.cuda.stream(streams[j]):
            a, b = lanes[j]["tix"][:Q * K].view(Q, K), lanes[j]["tv"][:Q * K].view(Q, K)
            if gdev.type == "cpu":
                a, b = a.cpu(), b.cpu()
            tg.start(a, b)

    # sub-ms configs: 6 s (the GPU part of a default run is then long enough for an outside
    # utilisation sampler to see the card busy; the timed steps are unchanged)
    spinup = args.spinup_seconds if args.spinup_seconds is not None else (20.0 if cfg["data"] == "20m" else 6.0)
    t_spin = time.time()
    n_spin = 0
    while time.time() - t_spin < spinup:
        compute()
        torch.cuda.synchronize(dev)
        n_spin += 1
    for _ in range(args.warmup):
        exchange(compute())
    if tg is not None:
        tg.wait()
    torch.cuda.synchronize(dev)
    # per-phase breakdown (informational) from a few instrumented steps; the timed steps
    # below record only the scoring phase's event pair (the roofline kernel time)
    def read_all():
        tot = {}
        for L in lanes:
            for p, v in L["ctx"].profile_read().items():
                a = tot.get(p, (0.0, 0))
                tot[p] = (a[0] + v[0], a[1] + v[1])
        return tot

    read_all()
    for L in lanes:
        L["ctx"].set_profiling(True)
    # (instrumented steps one at a time: the per-phase breakdown of an un-overlapped step)
    n_instr = max(1, min(args.steps, 5))
    for _ in range(n_instr):
        compute()
        torch.cuda.synchronize(dev)
    for L in lanes:
        L["ctx"].set_profiling(False)
    phases = read_all()
    # optional: the whole step captured once as a HIP graph and replayed (every kernel still
    # runs every step; the graph only removes host launch cost).  fia_prepare_for (large k)
    # decides the cache size on the host, so those configs run eagerly.
    use_graph = args.graph and not big_k and len(lanes) == 1
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

    # the step's dominant phase (instrumented steps above) is priced by the roofline; its
    # launches and the scoring kernel's are timed by HIP events over the timed region
    per_step = {p: v[0] / n_instr for p, v in phases.items()}
    dom = max(("prepare", "solve", "score"), key=lambda p: per_step.get(p, 0.0))
    if not args.no_timed_events:
        for L in lanes:
            L["ctx"].set_profiling(True, phases=tuple(sorted({"score", dom})))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if graph is not None:
            graph.replay()
            exchange()
        else:
            exchange(compute())
    if tg is not None:
        tg.wait()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    for L in lanes:
        L["ctx"].set_profiling(False)
    timed = read_all()          # scoring kernel duration over the timed region
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=gdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    ms_per_step = elapsed * 1e3 / args.steps
    node_queries = int(sum(all_sizes))
    value = node_queries * args.steps / elapsed

    def timed_ms(phase):
        # per launch over the timed region (graph replay: events are not re-recorded, so the
        # instrumented eager steps stand in)
        t = timed.get(phase, (0.0, 0))
        if t[1] == 0:
            t = phases.get(phase, (0.0, 0))
        return t[0] / max(t[1], 1)

    # the scoring kernel against HBM: PMC bytes per launch (profiles/traffic.json) over its
    # event time; compulsory bytes = its outputs + every list entry of the batch read once
    score_ms = timed_ms("score")
    kern = score_kernel(cfg, K)
    alg_bytes = float(bytes_per_query(cfg["model"], k, n_q).sum()) / len(batches)   # mean per launch
    # a shard's kernels move the shard's bytes: its own traffic.json key (none: traffic null)
    tkey = args.config if shard_of == 1 else "%s/shard%dof%d" % (
        args.config, rank if world > 1 else args.shard_index, shard_of)
    tj = load_traffic(args.traffic_json, tkey, kern)
    traffic = tj.get("hbm_bytes_per_launch") if tj else None
    deg_u = np.bincount(tu, minlength=U).astype(np.float64)
    deg_i = np.bincount(ti, minlength=I).astype(np.float64)
    comp = compulsory_bytes(cfg, qu_np, qi_np, deg_u, deg_i, bounds)
    achieved = traffic / (score_ms * 1e-3) / 1e9 if traffic else None
    score_hbm = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": achieved / HBM_PEAK_GBS if achieved is not None else None, "traffic": traffic,
                 "compulsory_bytes": comp, "traffic_over_compulsory": traffic / comp if traffic else None,
                 "kernel": kern, "kernel_ms": score_ms,
                 "source": ("rocprofv3 PMC (FETCH_SIZE x 2 + WRITE_SIZE) per launch, %s" % os.path.relpath(
                     args.traffic_json, ROOT)) if traffic else "no PMC traffic recorded for this config/kernel",
                 "algorithmic": {"model": "SURVEY.md 8d (gathered rows counted once per query)",
                                 "bytes_per_launch": alg_bytes, "gbs": alg_bytes / (score_ms * 1e-3) / 1e9}}
    if len(lanes) > 1:
        # batches in flight share the GPU, so the timed-region launch is longer than the
        # kernel alone: the same bytes over the instrumented (one step at a time) launches too
        iso = phases.get("score", (0.0, 0))
        iso_ms = iso[0] / max(iso[1], 1)
        score_hbm["isolated"] = {"kernel_ms": iso_ms,
                                 "achieved": traffic / (iso_ms * 1e-3) / 1e9 if traffic and iso_ms > 0 else None,
                                 "frac": traffic / (iso_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if traffic and iso_ms > 0
                                 else None,
                                 "note": "instrumented steps run one at a time (no overlap with another batch)"}
    if dom == "score":
        roofline = dict(score_hbm, phase="score")
    else:
        # a compute phase: algorithmic FP64 flops per launch over its event time
        ph_ms = timed_ms(dom)
        if dom == "solve":
            dk = solve_kernel(cfg)
            flops = solve_flops(cfg["model"], k, Q) / len(batches)
            fmodel = "2 side systems per query of D_s = %d: LDL^T 2D^3/3 + solves 2D^2 flops" % side_dim(cfg["model"], k)
        else:
            dk = prepare_kernel(cfg)
            # the list entries of the cached entities (a shard caches only its queries' users
            # and items)
            rows = float(deg_u[np.unique(qu_np)].sum() + deg_i[np.unique(qi_np)].sum()) if sharded \
                else 2.0 * tu.size
            flops = prepare_flops(cfg["model"], k, rows)
            fmodel = ("per list entry of the %s entities (%d entries): Gram rank-1 update D_s(D_s+1) flops "
                      "(+ NCF MLP 12 k^2)" % ("shard's cached" if sharded else "cached", rows))
        # PMC bytes of the whole phase per launch when recorded (the solve phase is several
        # kernels, dispatched many times per batch: "<phase>_phase" entries sum them), else the
        # dominant kernel's own entry
        dtj = load_traffic(args.traffic_json, tkey, dom + "_phase") or \
            load_traffic(args.traffic_json, tkey, dk)
        dtraffic = dtj.get("hbm_bytes_per_launch") if dtj else None
        tfs = flops / (ph_ms * 1e-3) / 1e12
        roofline = {"bound": "mfma", "achieved": tfs, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                    "frac": tfs / FP64_PEAK_TFS, "traffic": dtraffic, "phase": dom, "kernel": dk, "kernel_ms": ph_ms,
                    "dtype": "f64", "flops_per_launch": flops, "flop_model": fmodel,
                    "peak_note": "MI355X dense FP64; f64 MFMA and f64 VALU issue to the same DP units (DESIGN.md "
                                 "section 6), so this one peak bounds both",
                    "traffic_gbs": dtraffic / (ph_ms * 1e-3) / 1e9 if dtraffic else None,
                    "traffic_scope": dtj.get("scope", "kernel " + dk + ", per dispatch") if dtj else None,
                    "score_hbm": score_hbm}
        if len(lanes) > 1:
            iso = phases.get(dom, (0.0, 0))
            iso_ms = iso[0] / max(iso[1], 1)
            roofline["isolated"] = {"kernel_ms": iso_ms,
                                    "achieved": flops / (iso_ms * 1e-3) / 1e12 if iso_ms > 0 else None,
                                    "frac": flops / (iso_ms * 1e-3) / 1e12 / FP64_PEAK_TFS if iso_ms > 0 else None,
                                    "note": "instrumented steps run one at a time (no overlap with another batch)"}
    workload = cfg["workload"]
    if world > 1 and scaling == "weak":
        workload += " -- WEAK scaling: ranks > 0 answer synthetic re-paired queries of the same shape"
    out = {
        "metric": "influence queries/sec (whole node) + % HBM roofline, MF k=16 ML-1M-ex"
        if args.config == "ml1m-mf" else "influence queries/sec (whole node), " + cfg["workload"],
        "value": value, "unit": "queries/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": scaling, "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic train ratings of the reference shape (train file not distributed) + the reference's "
                "real held-out test pairs (20M: synthetic held-out pairs); synthetic parameters",
        "config": {"workload": workload, "scope": "%d GPU%s (value = all ranks' queries / max-over-ranks time)" % (
                       world, "" if world == 1 else "s"),
                   "model": cfg["model"], "k": k, "queries_per_rank": all_sizes,
                   "node_queries_per_step": node_queries, "n_train": int(tu.size),
                   "related_ratings_rank0_step": int(total), "topk": K, "query_batches": len(batches),
                   "query_order": args.query_order, "shard_of": shard_of,
                   "shard_index": (rank if world > 1 else args.shard_index) if shard_of > 1 else None,
                   "hip_graph": use_graph,
                   "batches_in_flight": len(lanes),
                   "spinup_steps": n_spin,
                   "dist_backend": backend if world > 1 else None,
                   "parallelism": "dp%d (query shards, top-K all_gather)" % world},
        "roofline": roofline,
        "phases_ms_per_step": {p: v[0] / n_instr for p, v in phases.items()},
        "phases_ms_per_launch": {p: (v[0] / max(v[1], 1)) for p, v in phases.items()},
        "index_build_s": index_s,
    }
    if repair:
        out["config"]["rank0_requery"] = repair
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(out), flush=True)
    for L in lanes:
        L["ctx"].close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
