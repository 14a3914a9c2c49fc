"""GPU parity of the HIP path (through the C ABI, via the reference-shaped
facade) against the fp64 oracle's golden fixtures and, at full size, against
size-independent properties.

Tolerances (north star): related sets and top-K ordering bit-exact; influence
and x within 1e-5 relative, normalised by the query's max |influence| / |x|
(the kernels compute in fp64, so the observed error is ~1e-13)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from influence import synth
from influence.dataset import DataSet

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def load(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def params_of(f):
    return {k[3:].replace("__", "/"): f[k] for k in f if k.startswith("p__")}


def make_model(model, U, I, k, train, test_pairs, params, wd=1e-3, damping=1e-6, tmpdir="output"):
    from influence.matrix_factorization import MF
    from influence.NCF import NCF
    tu, ti, tr = train
    qu, qi = test_pairs
    data_sets = {"train": DataSet(np.stack([tu, ti], 1), np.asarray(tr, np.float64)),
                 "validation": None,
                 "test": DataSet(np.stack([qu, qi], 1), np.zeros(len(qu)))}
    cls = MF if model == "MF" else NCF
    return cls(num_users=int(U), num_items=int(I), embedding_size=int(k), weight_decay=wd, num_classes=1,
               batch_size=3020, data_sets=data_sets, initial_learning_rate=1e-3, damping=damping,
               decay_epochs=[10000, 20000], mini_batch=True, train_dir=str(tmpdir), log_dir="log",
               avextol=1e-3, model_name="test_%s" % model, params=params, verbose=False)


def rel_err(a, b):
    s = np.abs(b).max(initial=0.0)
    return np.abs(a - b).max(initial=0.0) / (s if s > 0 else 1.0)


NEAR_TIE = 1e-12


def check_topk(got, gpu_vals, oracle_vals, K):
    """Top-K positions: (1) bit-exact selection on the kernel's own fp64 values;
    (2) bit-exact against the oracle's ranking, except that two entries whose
    |oracle value| differ by < 1e-12 * max may swap (near-ties are flagged, not
    failed: SURVEY.md 8c).  Returns the number of near-tie swaps."""
    from oracle import fia_oracle as fo
    want_gpu = fo.topk(gpu_vals, K)
    assert np.array_equal(got[:want_gpu.size], want_gpu)
    assert (got[want_gpu.size:] == -1).all()
    want = fo.topk(oracle_vals, K)
    assert want.size == want_gpu.size
    a = np.abs(oracle_vals)
    tol = NEAR_TIE * a.max(initial=0.0)
    swaps = 0
    for t in np.nonzero(got[:want.size] != want)[0]:
        assert abs(a[got[t]] - a[want[t]]) <= tol, (t, got[t], want[t], a[got[t]], a[want[t]])
        swaps += 1
    return swaps


@pytest.mark.parametrize("name", ["small_mf_k16.npz", "small_ncf_k16.npz", "small_mf_k8.npz", "small_ncf_k8.npz"])
def test_small_golden_single_query_api(name, tmp_path):
    f = load(name)
    model = "MF" if "_mf_" in name else "NCF"
    m = make_model(model, f["U"], f["I"], f["k"], (f["train_user"], f["train_item"], f["train_rating"]),
                   (f["q_user"], f["q_item"]), params_of(f), tmpdir=tmp_path)
    N = f["train_user"].size
    for q in range(f["q_user"].size):
        b, e = f["offsets"][q], f["offsets"][q + 1]
        rel = m.get_train_indices_of_test_case([q])
        assert rel.dtype == np.int64 and np.array_equal(rel, f["rel"][b:e])
        infl = m.get_influence_on_test_loss([q], np.arange(N))
        assert np.array_equal(m.train_indices_of_test_case, f["rel"][b:e])
        assert infl.dtype == np.float64 and infl.shape == (e - b,)
        if e > b:
            assert rel_err(infl, f["influence"][b:e]) < RTOL
            assert rel_err(np.concatenate(m.inverse_hvp), f["x"][q]) < RTOL
        else:
            assert np.isnan(np.concatenate(m.inverse_hvp)).all()


@pytest.mark.parametrize("name", ["small_mf_k16.npz", "small_ncf_k16.npz"])
@pytest.mark.parametrize("K", [1, 3, 5, 64])
def test_small_golden_batch_and_topk(name, K, tmp_path):
    from oracle import fia_oracle as fo
    f = load(name)
    model = "MF" if "_mf_" in name else "NCF"
    m = make_model(model, f["U"], f["I"], f["k"], (f["train_user"], f["train_item"], f["train_rating"]),
                   (f["q_user"], f["q_item"]), params_of(f), tmpdir=tmp_path)
    Q = f["q_user"].size
    res = m.get_influence_batch(list(range(Q)), K=K)
    assert np.array_equal(res["offsets"], f["offsets"])
    assert np.array_equal(res["rel_idx"], f["rel"])
    for q in range(Q):
        b, e = f["offsets"][q], f["offsets"][q + 1]
        if e > b:
            assert rel_err(res["influence"][b:e], f["influence"][b:e]) < RTOL
        got = res["topk_pos"][q]
        check_topk(got, res["influence"][b:e], f["influence"][b:e], K)
        want = got[got >= 0]
        assert np.isnan(res["topk_val"][q][want.size:]).all()
        assert np.array_equal(res["topk_idx"][q][:want.size], f["rel"][b:e][want])
        np.testing.assert_array_equal(res["topk_val"][q][:want.size], res["influence"][b:e][want])


def test_duplicate_rows_tie_by_position(tmp_path):
    """The test pair present twice in train appears 4 times in rel with equal
    influence per copy: top-K must list equal values by related position."""
    f = load("small_mf_k16.npz")
    m = make_model("MF", f["U"], f["I"], f["k"], (f["train_user"], f["train_item"], f["train_rating"]),
                   (f["q_user"], f["q_item"]), params_of(f), tmpdir=tmp_path)
    q = 2   # (tu[7], ti[7]) duplicated in train
    res = m.get_influence_batch([q], K=8)
    infl = res["influence"]
    rel = res["rel_idx"]
    for row in np.unique(rel):
        copies = infl[rel == row]
        assert (copies == copies[0]).all()          # each copy of a train row: identical bits
    assert (np.bincount(rel) == 2).sum() == 2       # both (u,i) rows appear twice
    order = np.lexsort((np.arange(infl.size), -np.abs(infl)))[:8]
    assert np.array_equal(res["topk_pos"][0], order)


@pytest.mark.parametrize("model", ["MF", "NCF"])
def test_ml1m_rq1_golden(model, tmp_path):
    f = load("ml1m_rq1_%s_k16.npz" % model.lower())
    d = synth.make_dataset(synth.ML1M, seed=0)
    p = synth.mf_params(d["U"], d["I"], 16, 0) if model == "MF" else synth.ncf_params(d["U"], d["I"], 16, 0)
    m = make_model(model, d["U"], d["I"], 16, d["train"], (f["q_user"], f["q_item"]), p, tmpdir=tmp_path)
    res = m.get_influence_batch(list(range(f["q_user"].size)), K=5)
    assert np.array_equal(res["offsets"], f["offsets"])
    assert np.array_equal(res["rel_idx"], f["rel"])
    for q in range(f["q_user"].size):
        b, e = f["offsets"][q], f["offsets"][q + 1]
        assert rel_err(res["influence"][b:e], f["influence"][b:e]) < RTOL
        assert rel_err(res["x"][q], f["x"][q]) < RTOL
        check_topk(res["topk_pos"][q], res["influence"][b:e], f["influence"][b:e], 5)
        assert np.array_equal(res["topk_pos"][q], f["topk_pos"][q])


@pytest.fixture(scope="module")
def ml1m_full(tmp_path_factory):
    d = synth.make_dataset(synth.ML1M, seed=0)
    p = synth.mf_params(d["U"], d["I"], 16, 0)
    qu, qi, _ = d["test"]
    m = make_model("MF", d["U"], d["I"], 16, d["train"], (qu, qi), p, tmpdir=tmp_path_factory.mktemp("ml"))
    res = m.get_influence_batch(list(range(qu.size)), K=4)
    return d, p, m, res


def test_ml1m_all_12074_queries_match_oracle(ml1m_full):
    """Config 2 (all 12,074 ml-1m-ex test ratings), EVERY query against the fp64 oracle
    (oracle.CsrExact: the closed form over CSR/CSC lists, mf:315-322, 237-246): related set
    bit-exact, influence and x within 1e-5 relative, top-4 bit-exact under the tie rule on the
    kernel's values and against the oracle's ranking up to flagged near-ties (< 1e-12 max);
    offsets = deg(u) + deg(i)."""
    from oracle import fia_oracle as fo
    d, p, m, res = ml1m_full
    tu, ti, tr = d["train"]
    qu, qi, _ = d["test"]
    assert qu.size == 12074
    deg_u = np.bincount(tu, minlength=d["U"])
    deg_i = np.bincount(ti, minlength=d["I"])
    n = deg_u[qu] + deg_i[qi]
    assert np.array_equal(np.diff(res["offsets"]), n)
    rel, infl, offs = res["rel_idx"], res["influence"], res["offsets"]
    assert np.isfinite(infl).all()
    oracle = fo.CsrExact("MF", p, 16, tu, ti, tr, 1e-3, 1e-6)
    worst_i = worst_x = 0.0
    near_ties = checked = 0
    for q in range(qu.size):
        o = oracle.query(int(qu[q]), int(qi[q]))
        b, e = offs[q], offs[q + 1]
        assert np.array_equal(o["rel"], rel[b:e]), q
        ei, ex = rel_err(infl[b:e], o["influence"]), rel_err(res["x"][q], o["x"])
        assert ei < RTOL and ex < RTOL, (q, ei, ex)
        worst_i, worst_x = max(worst_i, ei), max(worst_x, ex)
        near_ties += check_topk(res["topk_pos"][q], infl[b:e], o["influence"], 4)
        checked += 1
    assert checked == 12074
    print("ml-1m-ex: %d queries vs oracle, worst influence %.2e, worst x %.2e, %d near-tie swaps"
          % (checked, worst_i, worst_x, near_ties))


def test_ml1m_deterministic(ml1m_full):
    d, p, m, res = ml1m_full
    again = m.get_influence_batch(list(range(d["test"][0].size)), K=4)
    for key in ("rel_idx", "influence", "x", "topk_pos", "topk_val"):
        assert np.array_equal(again[key], res[key], equal_nan=True), key


def test_yelp_ncf_sample_matches_oracle(tmp_path):
    """Config 3 shape (yelp-ex, NCF k=16): a query sample against the oracle."""
    from oracle import fia_oracle as fo
    d = synth.make_dataset(synth.YELP, seed=0)
    p = synth.ncf_params(d["U"], d["I"], 16, 0)
    qu, qi, _ = d["test"]
    sel = np.random.default_rng(1).choice(qu.size, 16, replace=False)
    m = make_model("NCF", d["U"], d["I"], 16, d["train"], (qu[sel], qi[sel]), p, tmpdir=tmp_path)
    res = m.get_influence_batch(list(range(sel.size)), K=2)
    tu, ti, tr = d["train"]
    for q in range(sel.size):
        o = fo.ncf_query(p, 16, tu, ti, tr, int(qu[sel[q]]), int(qi[sel[q]]), 1e-3, 1e-6)
        b, e = res["offsets"][q], res["offsets"][q + 1]
        assert np.array_equal(o["rel"], res["rel_idx"][b:e])
        assert rel_err(res["influence"][b:e], o["influence"]) < RTOL
        check_topk(res["topk_pos"][q], res["influence"][b:e], o["influence"], 2)


@pytest.mark.parametrize("model,k", [("MF", 8), ("MF", 16), ("MF", 32), ("MF", 64), ("NCF", 8), ("NCF", 16),
                                     ("NCF", 32)])
def test_every_built_size_matches_oracle(model, k, tmp_path):
    """Every (model, k) the library is built for, on a small random problem with
    long lists (Gram work items split and recombined), a held-out pair, the pair
    itself in train and an empty side."""
    from oracle import fia_oracle as fo
    rng = np.random.default_rng(k + (100 if model == "NCF" else 0))
    U, I, N = 700, 30, 3000
    key = np.sort(rng.choice((U - 1) * I, N - 1, replace=False))
    tu, ti = (key // I).astype(np.int32), (key % I).astype(np.int32)
    # one very long item list: item 0 rated by every user (forces split Gram items at 512/list)
    extra_u = np.arange(U - 1, dtype=np.int32)
    tu = np.concatenate([tu, extra_u, [tu[5]]]).astype(np.int32)
    ti = np.concatenate([ti, np.full(U - 1, I - 1, np.int32), [ti[5]]]).astype(np.int32)
    tr = rng.integers(1, 6, tu.size).astype(np.float32)
    p = synth.mf_params(U, I, k, 3) if model == "MF" else synth.ncf_params(U, I, k, 3)
    qs = [(1, 2), (int(tu[5]), int(ti[5])), (U - 1, 3), (7, I - 1), (int(tu[50]), int(ti[50]))]
    qu = np.array([q[0] for q in qs], np.int32)
    qi = np.array([q[1] for q in qs], np.int32)
    m = make_model(model, U, I, k, (tu, ti, tr), (qu, qi), p, tmpdir=tmp_path)
    res = m.get_influence_batch(list(range(len(qs))), K=3)
    for q, (u, i) in enumerate(qs):
        o = fo.query(model, p, k, tu, ti, tr, u, i, 1e-3, 1e-6)
        b, e = res["offsets"][q], res["offsets"][q + 1]
        assert np.array_equal(o["rel"], res["rel_idx"][b:e])
        if o["n"]:
            assert rel_err(res["influence"][b:e], o["influence"]) < RTOL, (model, k, q)
            assert rel_err(res["x"][q], o["x"]) < RTOL, (model, k, q)
            check_topk(res["topk_pos"][q], res["influence"][b:e], o["influence"], 3)


def test_invalid_queries_raise(tmp_path):
    from influence._lib import FIAError
    f = load("small_mf_k16.npz")
    qu = np.array([0, 1000], np.int32)
    qi = np.array([0, 0], np.int32)
    m = make_model("MF", f["U"], f["I"], f["k"], (f["train_user"], f["train_item"], f["train_rating"]),
                   (qu, qi), params_of(f), tmpdir=tmp_path)
    with pytest.raises(FIAError):
        m.get_influence_batch([1], K=1)
    with pytest.raises(FIAError):
        m.get_influence_batch([0], K=65)


@pytest.mark.parametrize("model,k", [("MF", 128), ("MF", 256), ("NCF", 64), ("NCF", 128), ("NCF", 256)])
def test_large_k_matches_oracle(model, k, tmp_path):
    """The large-k path (tile-packed Gram caches, blocked MFMA LDL^T, entity-shared
    scoring): a long item list (Gram slices + partial combine, 3 scoring chunks), a
    query group of > 8 queries on that item (several query blocks), the pair in
    train twice (coupled full-D solve), an empty user side."""
    from oracle import fia_oracle as fo
    rng = np.random.default_rng(k + (100 if model == "NCF" else 0))
    U, I, N = 2600, 30, 6000
    key = np.sort(rng.choice((U - 1) * (I - 1), N, replace=False))
    tu, ti = (key // (I - 1)).astype(np.int32), (key % (I - 1)).astype(np.int32)
    # item I-1 rated by 2200 users (two Gram slices, 9 scoring chunks); pair (tu[5], ti[5]) twice more
    ex = rng.choice(U - 1, 2200, replace=False).astype(np.int32)
    tu = np.concatenate([tu, ex, [tu[5], tu[5]]]).astype(np.int32)
    ti = np.concatenate([ti, np.full(ex.size, I - 1, np.int32), [ti[5], ti[5]]]).astype(np.int32)
    tr = rng.integers(1, 6, tu.size).astype(np.float32)
    p = synth.mf_params(U, I, k, 3) if model == "MF" else synth.ncf_params(U, I, k, 3)
    shared = [(int(u), I - 1) for u in rng.choice(U - 1, 11, replace=False)]
    qs = [(1, 2), (int(tu[5]), int(ti[5])), (U - 1, 3), (7, I - 1), (U - 1, I - 1), (int(ex[0]), I - 1)] + shared
    qu = np.array([q[0] for q in qs], np.int32)
    qi = np.array([q[1] for q in qs], np.int32)
    m = make_model(model, U, I, k, (tu, ti, tr), (qu, qi), p, tmpdir=tmp_path)
    res = m.get_influence_batch(list(range(len(qs))), K=3)
    for q, (u, i) in enumerate(qs):
        o = fo.query(model, p, k, tu, ti, tr, u, i, 1e-3, 1e-6)
        b, e = res["offsets"][q], res["offsets"][q + 1]
        assert np.array_equal(o["rel"], res["rel_idx"][b:e])
        if o["n"]:
            assert rel_err(res["influence"][b:e], o["influence"]) < RTOL, (model, k, q)
            assert rel_err(res["x"][q], o["x"]) < RTOL, (model, k, q)
            check_topk(res["topk_pos"][q], res["influence"][b:e], o["influence"], 3)
        else:
            assert np.isnan(res["x"][q]).all()
    # the two copies of a train row in rel carry identical bits
    b, e = res["offsets"][1], res["offsets"][2]
    rel, infl = res["rel_idx"][b:e], res["influence"][b:e]
    for row in np.unique(rel[np.bincount(rel)[rel] > 1]):
        assert (infl[rel == row] == infl[rel == row][0]).all()


@pytest.mark.parametrize("model,k", [("MF", 128), ("NCF", 64), ("MF", 16), ("MF", 64), ("NCF", 16), ("NCF", 8),
                                     ("MF", 32), ("NCF", 32)])
def test_prepare_for_subset(model, k, tmp_path):
    """fia_prepare_for: caches for only the queried users/items give the same
    results as the full prepare (bitwise), and a query outside the set is rejected
    until the next full prepare.  Large k: compacted slot caches; small k: dense caches
    of the marked entities only."""
    from influence._lib import FIAError
    rng = np.random.default_rng(5)
    U, I, N = 300, 40, 4000
    key = np.sort(rng.choice(U * I, N, replace=False))
    tu, ti = (key // I).astype(np.int32), (key % I).astype(np.int32)
    tr = rng.integers(1, 6, N).astype(np.float32)
    p = synth.mf_params(U, I, k, 1) if model == "MF" else synth.ncf_params(U, I, k, 1)
    qu = rng.integers(0, U, 12).astype(np.int32)
    qi = rng.integers(0, I, 12).astype(np.int32)
    qu[11], qi[11] = U - 1, I - 1
    m = make_model(model, U, I, k, (tu, ti, tr), (qu, qi), p, tmpdir=tmp_path)
    full = m.get_influence_batch(list(range(12)), K=2)
    subset = [q for q in range(11) if qu[q] != U - 1 and qi[q] != I - 1]
    m.prepare_for(subset)
    part = m.get_influence_batch(subset, K=2)
    for j, q in enumerate(subset):
        b, e = full["offsets"][q], full["offsets"][q + 1]
        pb, pe = part["offsets"][j], part["offsets"][j + 1]
        assert np.array_equal(part["rel_idx"][pb:pe], full["rel_idx"][b:e])
        assert np.array_equal(part["influence"][pb:pe], full["influence"][b:e])   # same kernels, same bits
        assert np.array_equal(part["x"][j], full["x"][q])
    with pytest.raises(FIAError):
        m.get_influence_batch([11], K=1)
    m.ctx.prepare()                              # every cache again: the query is answered
    again = m.get_influence_batch([11], K=2)
    b, e = full["offsets"][11], full["offsets"][12]
    assert np.array_equal(again["influence"], full["influence"][b:e])


@pytest.mark.parametrize("model,k", [("MF", 16), ("NCF", 8), ("MF", 32), ("MF", 64)])
def test_many_queries_scan_windows(model, k, tmp_path):
    """40,000 queries (157 scan tiles of 256: the decoupled look-back walks more than one
    64-tile window) with repeated users and items: offsets = deg(u) + deg(i) exactly, the
    related lists and top-K are consistent, and a sample matches the oracle."""
    from oracle import fia_oracle as fo
    rng = np.random.default_rng(7 + k)
    U, I, N = 2000, 300, 30000
    key = np.sort(rng.choice(U * I, N, replace=False))
    tu, ti = (key // I).astype(np.int32), (key % I).astype(np.int32)
    tr = rng.integers(1, 6, N).astype(np.float32)
    p = synth.mf_params(U, I, k, 5) if model == "MF" else synth.ncf_params(U, I, k, 5)
    Q = 40000
    qu = rng.integers(0, U, Q).astype(np.int32)
    qi = rng.integers(0, I, Q).astype(np.int32)
    m = make_model(model, U, I, k, (tu, ti, tr), (qu, qi), p, tmpdir=tmp_path)
    res = m.get_influence_batch(list(range(Q)), K=2)
    deg_u = np.bincount(tu, minlength=U)
    deg_i = np.bincount(ti, minlength=I)
    assert np.array_equal(np.diff(res["offsets"]), deg_u[qu] + deg_i[qi])
    assert res["offsets"][0] == 0
    offs, rel, infl = res["offsets"], res["rel_idx"], res["influence"]
    for q in rng.choice(Q, 30, replace=False):
        b, e = offs[q], offs[q + 1]
        du = deg_u[qu[q]]
        assert (tu[rel[b:b + du]] == qu[q]).all() and (ti[rel[b + du:e]] == qi[q]).all()
        assert np.array_equal(res["topk_pos"][q], fo.topk(infl[b:e], 2))
    for q in rng.choice(Q, 6, replace=False):
        o = fo.query(model, p, k, tu, ti, tr, int(qu[q]), int(qi[q]), 1e-3, 1e-6)
        b, e = offs[q], offs[q + 1]
        assert np.array_equal(o["rel"], rel[b:e])
        if o["n"]:
            assert rel_err(infl[b:e], o["influence"]) < RTOL, (model, k, q)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [32, 64])
@pytest.mark.parametrize("K", [1, 4, 6])
def test_mf_entity_shared_topk_paths(k, K, tmp_path):
    """MF k >= 32 entity-shared scoring (k_score_grouped_mf) at K = 1, 4, 6: many queries
    per entity (query blocks split), a query whose pair is a train row; every query's
    related set, influence and top-K against the fp64 oracle."""
    from oracle import fia_oracle as fo
    rng = np.random.default_rng(11 * k + K)
    U, I, N = 400, 12, 2500
    key = np.sort(rng.choice(U * I, N, replace=False))
    tu, ti = (key // I).astype(np.int32), (key % I).astype(np.int32)
    tr = rng.integers(1, 6, N).astype(np.float32)
    p = synth.mf_params(U, I, k, 9)
    Q = 300
    qu = rng.integers(0, U, Q).astype(np.int32)
    qi = rng.integers(0, I, Q).astype(np.int32)
    qu[0], qi[0] = tu[17], ti[17]          # pair in train (dup path)
    m = make_model("MF", U, I, k, (tu, ti, tr), (qu, qi), p, tmpdir=tmp_path)
    res = m.get_influence_batch(list(range(Q)), K=K)
    offs = res["offsets"]
    for q in range(Q):
        o = fo.query("MF", p, k, tu, ti, tr, int(qu[q]), int(qi[q]), 1e-3, 1e-6)
        b, e = offs[q], offs[q + 1]
        assert np.array_equal(o["rel"], res["rel_idx"][b:e])
        assert rel_err(res["influence"][b:e], o["influence"]) < RTOL, (k, K, q)
        assert np.array_equal(res["topk_pos"][q][:min(K, e - b)], fo.topk(res["influence"][b:e], K)), (k, K, q)
        check_topk(res["topk_pos"][q], res["influence"][b:e], o["influence"], K)


@pytest.mark.parametrize("name", ["small_mf_k16.npz", "small_ncf_k16.npz"])
def test_cached_inverse_hvp_force_refresh_false(name, tmp_path):
    """get_influence_on_test_loss(force_refresh=False) with the reference's cached
    <model>-cg-normal_loss-test-[t].npz present scores with the cached vector
    (matrix_factorization.py:210-214) on the GPU (fia_query_batch_x): the cache the first
    call wrote gives the same influence up to the rounding of the record's x . theta and
    x . v sums (k_record_x sums them in another order than the solve kernels: 1e-12
    relative), and a doubled vector exactly doubled influence (same kernel; influence is
    linear in x, a power-of-two scale is exact in fp64)."""
    f = load(name)
    model = "MF" if "mf" in name else "NCF"
    k, U, I = int(f["k"]), int(f["U"]), int(f["I"])
    m = make_model(model, U, I, k, (f["train_user"], f["train_item"], f["train_rating"]),
                   (f["q_user"], f["q_item"]), params_of(f), tmpdir=tmp_path)
    t = 0
    n_tr = f["train_user"].size
    first = m.get_influence_on_test_loss([t], np.arange(n_tr), force_refresh=True)
    x0 = np.concatenate([np.ravel(a) for a in m.inverse_hvp])
    again = m.get_influence_on_test_loss([t], np.arange(n_tr), force_refresh=False)
    assert np.abs(again - first).max() <= 1e-12 * np.abs(first).max()
    fname = os.path.join(str(tmp_path), "test_%s-cg-normal_loss-test-[%d].npz" % (model, t))
    with np.load(fname, allow_pickle=False) as z:
        cached = z["inverse_hvp"]
    np.savez(fname, inverse_hvp=2.0 * cached)
    twice = m.get_influence_on_test_loss([t], np.arange(n_tr), force_refresh=False)
    assert np.array_equal(twice, 2.0 * again)
    x1 = np.concatenate([np.ravel(a) for a in m.inverse_hvp])
    assert np.array_equal(x1, 2.0 * x0)
    # force_refresh=True ignores (and rewrites) the cache
    fresh = m.get_influence_on_test_loss([t], np.arange(n_tr), force_refresh=True)
    assert np.array_equal(fresh.view(np.int64), first.view(np.int64))


@pytest.mark.parametrize("model,k", [("MF", 128), ("NCF", 64)])
def test_cached_inverse_hvp_force_refresh_false_large_k(model, k, tmp_path):
    """force_refresh=False at large k (matrix_factorization.py:210-214, experiments.py:4,17):
    the cached vector replaces the batched LDL^T (k_big_record_x) for a plain query and for
    one whose test pair is a train row (the coupled full-D system); the second call matches
    the first to 1e-12 relative, a doubled vector gives exactly doubled influence, and a file
    holding the reference's own ragged per-block list (an object array, refused without
    pickle) is ignored -- the solve runs instead, and the file is not overwritten."""
    rng = np.random.default_rng(11)
    U, I, N = 300, 40, 4000
    key = np.sort(rng.choice(U * I, N, replace=False))
    tu, ti = (key // I).astype(np.int32), (key % I).astype(np.int32)
    tr = rng.integers(1, 6, N).astype(np.float32)
    p = synth.mf_params(U, I, k, 2) if model == "MF" else synth.ncf_params(U, I, k, 2)
    qu = np.array([3, int(tu[7])], np.int32)          # query 1: its pair is a train row
    qi = np.array([5, int(ti[7])], np.int32)
    m = make_model(model, U, I, k, (tu, ti, tr), (qu, qi), p, tmpdir=tmp_path)
    for t in (0, 1):
        first = m.get_influence_on_test_loss([t], np.arange(N), force_refresh=True)
        x0 = np.concatenate([np.ravel(a) for a in m.inverse_hvp])
        again = m.get_influence_on_test_loss([t], np.arange(N), force_refresh=False)
        assert np.abs(again - first).max() <= 1e-12 * np.abs(first).max(), (t, rel_err(again, first))
        fname = os.path.join(str(tmp_path), "test_%s-cg-normal_loss-test-[%d].npz" % (model, t))
        np.savez(fname, inverse_hvp=2.0 * x0)
        twice = m.get_influence_on_test_loss([t], np.arange(N), force_refresh=False)
        assert np.array_equal(twice, 2.0 * again)
        # the reference's ragged list [k, k, 1, 1] (mf:221): an object array -> ignored
        ragged = np.empty(4, dtype=object)
        ragged[:] = [x0[:2], x0[2:5], x0[5:6], x0[6:]]
        np.savez(fname, inverse_hvp=ragged)
        with open(fname, "rb") as fh:
            ref_bytes = fh.read()
        solved = m.get_influence_on_test_loss([t], np.arange(N), force_refresh=False)
        assert np.array_equal(solved.view(np.int64), first.view(np.int64))
        with open(fname, "rb") as fh:           # the reference-format file is left as it was
            assert fh.read() == ref_bytes


@pytest.mark.parametrize("model", ["MF", "NCF"])
@pytest.mark.parametrize("k", [8, 16])
@pytest.mark.parametrize("K", [1, 4])
def test_small_k_topk_only_no_outputs(model, k, K, tmp_path):
    """fia_query_batch with rel_idx = influence = NULL (get_influence_batch(full=False)): the
    k <= 16 item-run kernels (k_score_mf_runs, k_score_ncf_runs) drop every per-rating store
    (zero-length buffer ranges) and the top-K lists equal the full run's."""
    rng = np.random.default_rng(40 + k)
    U, I, N = 500, 60, 6000
    key = np.sort(rng.choice(U * I, N, replace=False))
    tu, ti = (key // I).astype(np.int32), (key % I).astype(np.int32)
    tr = rng.integers(1, 6, N).astype(np.float32)
    p = (synth.mf_params if model == "MF" else synth.ncf_params)(U, I, k, 4)
    qi = np.sort(rng.integers(0, I, 200)).astype(np.int32)      # item runs
    qu = rng.integers(0, U, 200).astype(np.int32)
    m = make_model(model, U, I, k, (tu, ti, tr), (qu, qi), p, tmpdir=tmp_path)
    full = m.get_influence_batch(list(range(qu.size)), K=K)
    lean = m.get_influence_batch(list(range(qu.size)), K=K, full=False, return_x=False)
    assert "influence" not in lean and "rel_idx" not in lean
    for key_ in ("topk_pos", "topk_idx"):
        assert np.array_equal(lean[key_], full[key_]), key_
    assert np.array_equal(lean["topk_val"], full["topk_val"], equal_nan=True)


@pytest.mark.parametrize("model", ["MF", "NCF"])
def test_graph_capture_matches_eager(model):
    """fia_prepare + fia_count_related + fia_query_batch captured into one HIP graph after an
    eager warm-up on another stream (as `bench.py --graph` does: the capture starts on a new
    stream, which the ABI must not synchronise against) and replayed: every output equals the
    eager run's bit for bit."""
    import torch
    from influence import _lib
    rng = np.random.default_rng(77)
    U, I, N, k = 400, 80, 8000, 16
    key = np.sort(rng.choice(U * I, N, replace=False))
    tu, ti = (key // I).astype(np.int32), (key % I).astype(np.int32)
    tr = rng.integers(1, 6, N).astype(np.float32)
    p = (synth.mf_params if model == "MF" else synth.ncf_params)(U, I, k, 7)
    qi_np = np.sort(rng.integers(0, I, 300)).astype(np.int32)
    qu_np = rng.integers(0, U, 300).astype(np.int32)
    dev = torch.device("cuda:0")
    ctx = _lib.Context(0)
    tables = [torch.from_numpy(np.ascontiguousarray(p[n], np.float32)).to(dev) for n in p]
    ctx.set_params(_lib.FIA_MODEL_MF if model == "MF" else _lib.FIA_MODEL_NCF, k, U, I, tables, 1e-3, 1e-6)
    ctx.build_index(torch.from_numpy(tu).to(dev), torch.from_numpy(ti).to(dev), torch.from_numpy(tr).to(dev), U, I)
    qu, qi = torch.from_numpy(qu_np).to(dev), torch.from_numpy(qi_np).to(dev)
    off, tot = ctx.count_related(qu, qi)
    D, K, Q = ctx.num_params(), 3, qu_np.size

    def bufs():
        return dict(rel=torch.full((tot,), -7, dtype=torch.int32, device=dev),
                    infl=torch.full((tot,), float("nan"), dtype=torch.float64, device=dev),
                    x=torch.zeros(Q * D, dtype=torch.float64, device=dev),
                    tp=torch.zeros(Q * K, dtype=torch.int64, device=dev),
                    tix=torch.zeros(Q * K, dtype=torch.int64, device=dev),
                    tv=torch.zeros(Q * K, dtype=torch.float64, device=dev))

    def step(b):
        ctx.prepare()
        ctx.count_related(qu, qi, off, want_total=False)
        ctx.query_batch(qu, qi, off, tot, b["rel"], b["infl"], b["x"], K, b["tp"], b["tix"], b["tv"])

    eager = bufs()
    step(eager)
    torch.cuda.synchronize(dev)
    rep = bufs()
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        step(rep)
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    for v in rep.values():
        v.zero_()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step(rep)
    graph.replay()
    torch.cuda.synchronize(dev)
    for name in eager:
        a, b = eager[name].cpu().numpy(), rep[name].cpu().numpy()
        assert np.array_equal(a, b, equal_nan=True), name


def test_graph_capture_refused_after_unjoined_prepare():
    """An eager fia_prepare that forks its Gram pass onto the context's aux stream (NCF k=16)
    followed directly by a capture: the captured kernels could not depend on that pass, so the
    first call inside the capture fails with FIA_ERR_STATE (no host wait is legal there); after
    a joining eager query the same capture succeeds and replays bit-identical to eager."""
    import torch
    from influence import _lib
    rng = np.random.default_rng(78)
    U, I, N, k = 300, 60, 5000, 16
    key = np.sort(rng.choice(U * I, N, replace=False))
    tu, ti = (key // I).astype(np.int32), (key % I).astype(np.int32)
    tr = rng.integers(1, 6, N).astype(np.float32)
    p = synth.ncf_params(U, I, k, 8)
    qi_np = np.sort(rng.integers(0, I, 200)).astype(np.int32)
    qu_np = rng.integers(0, U, 200).astype(np.int32)
    dev = torch.device("cuda:0")
    ctx = _lib.Context(0)
    tables = [torch.from_numpy(np.ascontiguousarray(p[n], np.float32)).to(dev) for n in p]
    ctx.set_params(_lib.FIA_MODEL_NCF, k, U, I, tables, 1e-3, 1e-6)
    ctx.build_index(torch.from_numpy(tu).to(dev), torch.from_numpy(ti).to(dev), torch.from_numpy(tr).to(dev), U, I)
    qu, qi = torch.from_numpy(qu_np).to(dev), torch.from_numpy(qi_np).to(dev)
    off, tot = ctx.count_related(qu, qi)
    D, K, Q = ctx.num_params(), 2, qu_np.size

    def bufs():
        return dict(rel=torch.full((tot,), -7, dtype=torch.int32, device=dev),
                    infl=torch.full((tot,), float("nan"), dtype=torch.float64, device=dev),
                    x=torch.zeros(Q * D, dtype=torch.float64, device=dev),
                    tp=torch.zeros(Q * K, dtype=torch.int64, device=dev),
                    tix=torch.zeros(Q * K, dtype=torch.int64, device=dev),
                    tv=torch.zeros(Q * K, dtype=torch.float64, device=dev))

    def step(b):
        ctx.prepare()
        ctx.count_related(qu, qi, off, want_total=False)
        ctx.query_batch(qu, qi, off, tot, b["rel"], b["infl"], b["x"], K, b["tp"], b["tix"], b["tv"])

    eager = bufs()
    step(eager)
    torch.cuda.synchronize(dev)
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        ctx.prepare()                        # forked, not joined by any query
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    refused = torch.cuda.CUDAGraph()
    with pytest.raises(_lib.FIAError, match="not joined"):
        with torch.cuda.graph(refused):
            ctx.prepare()
    del refused
    rep = bufs()
    with torch.cuda.stream(side):
        step(rep)                            # the query joins the pending pass
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    for v in rep.values():
        v.zero_()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step(rep)
    graph.replay()
    torch.cuda.synchronize(dev)
    for name in eager:
        a, b = eager[name].cpu().numpy(), rep[name].cpu().numpy()
        assert np.array_equal(a, b, equal_nan=True), name
    ctx.close()


@pytest.mark.parametrize("k", [8, 16])
def test_prepare_for_sliced_item_lists(k, tmp_path):
    """MF k <= 16 fia_prepare_for with item lists longer than a Gram-stream slice (256
    ratings): the marked entities' partial Grams of several slices are summed by
    k_gram_combine; results equal the full prepare's bit for bit (matrix_factorization.py:
    315-322: one Hessian per query whichever caches exist)."""
    rng = np.random.default_rng(90 + k)
    U, I, N = 3000, 24, 20000
    # skewed items: a few hold > 1000 ratings (several 256-rating slices), most fewer
    w = 1.0 / np.arange(1, I + 1) ** 1.2
    items = rng.choice(I, N, p=w / w.sum())
    users = rng.integers(0, U, N)
    key = np.unique(users.astype(np.int64) * I + items)
    tu, ti = (key // I).astype(np.int32), (key % I).astype(np.int32)
    tr = rng.integers(1, 6, tu.size).astype(np.float32)
    assert np.bincount(ti, minlength=I).max() > 1000
    p = synth.mf_params(U, I, k, 6)
    qu = rng.integers(0, U, 40).astype(np.int32)
    qi = rng.integers(0, I, 40).astype(np.int32)
    qi[:4] = np.argsort(-np.bincount(ti, minlength=I))[:4]      # the longest lists
    m = make_model("MF", U, I, k, (tu, ti, tr), (qu, qi), p, tmpdir=tmp_path)
    full = m.get_influence_batch(list(range(40)), K=2)
    subset = list(range(0, 40, 2))
    m.prepare_for(subset)
    part = m.get_influence_batch(subset, K=2)
    for j, q in enumerate(subset):
        b, e = full["offsets"][q], full["offsets"][q + 1]
        pb, pe = part["offsets"][j], part["offsets"][j + 1]
        assert np.array_equal(part["rel_idx"][pb:pe], full["rel_idx"][b:e])
        assert np.array_equal(part["influence"][pb:pe], full["influence"][b:e])
        assert np.array_equal(part["x"][j], full["x"][q])
    from oracle import fia_oracle as fo
    for q in subset[:3]:
        o = fo.query("MF", p, k, tu, ti, tr, int(qu[q]), int(qi[q]), 1e-3, 1e-6)
        b, e = full["offsets"][q], full["offsets"][q + 1]
        assert rel_err(full["influence"][b:e], o["influence"]) < RTOL


@pytest.mark.parametrize("model", ["MF", "NCF"])
def test_single_query_path_matches_batch(model, tmp_path):
    """get_influence_on_test_loss's one-sync single-query path (host degree counts, persistent
    pinned buffers) returns the batch path's bits for ml-1m-ex queries -- RQ2's test_idx 59,
    the heaviest query, a train-pair query, growing related-set sizes (buffer regrowth) -- and
    after prepare_for it takes the checked path (an uncovered query raises)."""
    from influence._lib import FIAError
    d = synth.make_dataset(synth.ML1M, seed=0)
    tu, ti, tr = d["train"]
    qu, qi, _ = d["test"]
    p = (synth.mf_params if model == "MF" else synth.ncf_params)(d["U"], d["I"], 16, 0)
    qu = np.append(qu, np.int32(tu[5]))           # a train pair (coupled system)
    qi = np.append(qi, np.int32(ti[5]))
    m = make_model(model, d["U"], d["I"], 16, d["train"], (qu, qi), p, tmpdir=tmp_path)
    m.save_inverse_hvp = False
    n = np.bincount(tu, minlength=d["U"])[qu] + np.bincount(ti, minlength=d["I"])[qi]
    order = [int(j) for j in np.argsort(n)[::1200]]
    qs = [59, int(np.argmax(n)), qu.size - 1] + order
    for t in qs:
        one = m.get_influence_on_test_loss([t], np.arange(tu.size))
        ref = m.get_influence_batch([t], K=0)
        assert np.array_equal(m.train_indices_of_test_case, ref["rel_idx"])
        assert np.array_equal(one.view(np.int64), ref["influence"].view(np.int64)), t
        x = np.concatenate([np.ravel(a) for a in m.inverse_hvp])
        assert np.array_equal(x.view(np.int64), ref["x"][0].view(np.int64)), t
    m.prepare_for([0, 1])
    far = next(t for t in range(qu.size) if qu[t] not in qu[:2] and qi[t] not in qi[:2])
    with pytest.raises(FIAError):
        m.get_influence_on_test_loss([far], np.arange(tu.size))
    m.ctx.prepare()
    again = m.get_influence_on_test_loss([far], np.arange(tu.size))
    assert np.array_equal(again.view(np.int64), m.get_influence_batch([far], K=0)["influence"].view(np.int64))
