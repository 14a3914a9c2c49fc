"""Multi-process sharded FIA on the GPU (layer 4; 8e).

Two processes share cuda:0 under a gloo process group (the RCCL path needs one GPU
per rank; the exchange is the same all_gather).  Each rank answers its contiguous,
n_q-balanced query range through libfia; the gathered top-K lists and each rank's
influence vectors must be bitwise equal to a single-process run of the whole set
(queries are independent, mf:315-322).  And bench.py's own multi-rank path
(`--gpus 2`: it re-launches itself under torch.distributed.run) runs end to end."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem(model, k):
    from influence import synth
    rng = np.random.default_rng(21 + k)
    U, I, N, Q = 3000, 400, 60000, 4000
    key = np.sort(rng.choice(U * I, N, replace=False))
    tu, ti = (key // I).astype(np.int32), (key % I).astype(np.int32)
    tr = rng.integers(1, 6, N).astype(np.float32)
    qu = rng.integers(0, U, Q).astype(np.int32)
    qi = rng.integers(0, I, Q).astype(np.int32)
    qu[5], qi[5] = tu[9], ti[9]          # one pair that is a train row
    p = synth.mf_params(U, I, k, 2) if model == "MF" else synth.ncf_params(U, I, k, 2)
    names = synth.MF_PARAM_NAMES if model == "MF" else synth.NCF_PARAM_NAMES
    return U, I, (tu, ti, tr), (qu, qi), [p[n] for n in names]


def _answer(model, k, U, I, train, qu_np, qi_np, tables_np, K):
    import torch
    from influence import _lib
    dev = torch.device("cuda", 0)
    ctx = _lib.Context(0)
    tabs = [torch.from_numpy(np.ascontiguousarray(t, np.float32)).to(dev) for t in tables_np]
    ctx.set_params(_lib.FIA_MODEL_MF if model == "MF" else _lib.FIA_MODEL_NCF, k, U, I, tabs, 1e-3, 1e-6)
    tt = [torch.from_numpy(a).to(dev) for a in train]
    ctx.build_index(tt[0], tt[1], tt[2], U, I)
    qu = torch.from_numpy(qu_np).to(dev)
    qi = torch.from_numpy(qi_np).to(dev)
    if k >= 128 or (model == "NCF" and k >= 64):
        ctx.prepare_for(qu, qi)
    else:
        ctx.prepare()
    offs, tot = ctx.count_related(qu, qi)
    Q = qu.numel()
    rel = torch.empty(max(tot, 1), dtype=torch.int32, device=dev)
    infl = torch.empty(max(tot, 1), dtype=torch.float64, device=dev)
    tp = torch.empty(Q * K, dtype=torch.int64, device=dev)
    tix = torch.empty_like(tp)
    tv = torch.empty(Q * K, dtype=torch.float64, device=dev)
    ctx.query_batch(qu, qi, offs, tot, rel, infl, None, K, tp, tix, tv)
    out = (infl[:tot].cpu(), tix.view(Q, K).cpu(), tv.view(Q, K).cpu(), offs.cpu())
    ctx.close()
    return out


def _rank(rank, ws, port, model, k, K, res):
    import torch.distributed as dist
    from influence.sharding import shard_ranges, gather_topk
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        U, I, train, (qu, qi), tables = _problem(model, k)
        deg_u = np.bincount(train[0], minlength=U)
        deg_i = np.bincount(train[1], minlength=I)
        b, e = shard_ranges(deg_u[qu] + deg_i[qi], ws)[rank]
        infl, tix, tv, _ = _answer(model, k, U, I, train, qu[b:e].copy(), qi[b:e].copy(), tables, K)
        gi, gv = gather_topk(tix, tv)
        res[rank] = (b, e, infl.numpy().copy(), gi.numpy().copy(), gv.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model,k", [("MF", 16), ("MF", 64), ("NCF", 16), ("NCF", 64)])
def test_two_ranks_on_one_gpu_equal_single_process(model, k):
    import torch.multiprocessing as mp
    K = 3
    with mp.Manager() as mgr:
        res = mgr.dict()
        mp.spawn(_rank, args=(2, _free_port(), model, k, K, res), nprocs=2, join=True)
        res = dict(res)
    U, I, train, (qu, qi), tables = _problem(model, k)
    infl, tix, tv, offs = _answer(model, k, U, I, train, qu, qi, tables, K)
    offs = offs.numpy()
    for r in range(2):
        b, e, rinfl, gi, gv = res[r]
        assert np.array_equal(gi, tix.numpy()), "gathered top-K rows differ from the single-process run"
        assert np.array_equal(gv.view(np.int64), tv.numpy().view(np.int64)), "gathered top-K values differ"
        assert np.array_equal(rinfl.view(np.int64), infl.numpy()[offs[b]:offs[e]].view(np.int64))
    assert res[0][1] == res[1][0] and res[1][1] == qu.size


@pytest.mark.parametrize("scaling", ["default", "weak", "strong"])
def test_bench_two_ranks(scaling, tmp_path):
    """bench.py --gpus 2 (self-launched under torch.distributed.run; both ranks on cuda:0, so
    gloo carries the top-K exchange): one JSON line with n_gpus 2 and the node's total.  The
    ml-1m-ex default is weak scaling (rank 1's synthetic re-paired queries are labelled in
    config.workload); strong scaling splits the real test set."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline"] + ([] if scaling == "default" else ["--scaling", scaling])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    want = "weak" if scaling == "default" else scaling
    assert out["n_gpus"] == 2 and out["scaling"] == want and out["value"] > 0
    sizes = out["config"]["queries_per_rank"]
    if want == "weak":
        assert sizes == [12074, 12074]
        assert "synthetic re-paired" in out["config"]["workload"]
    else:
        assert sum(sizes) == 12074 and min(sizes) > 0
        assert "re-paired" not in out["config"]["workload"]
    assert out["config"]["node_queries_per_step"] == sum(sizes)
