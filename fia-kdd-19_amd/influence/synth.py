"""Synthetic training ratings and parameters shaped like the reference's configs.

The reference's training files are absent (/root/reference/.MISSING_LARGE_BLOBS
lists data/ml-1m-ex.train.rating and data/yelp-ex.train.rating) and there is no
trained checkpoint, so the FIA path is exercised on synthetic train ratings
with the cardinalities the reference loaders hard-code, plus the REAL held-out
test pairs (fia-kdd-19_amd/data/*.npz, re-encoded from the reference's data/).

Shapes:
  ml-1m-ex : U=6040,   I=3706,   N=975,460   (load_movielens.py:12, train[:975460])
  yelp-ex  : U=25,677, I=25,815, N=628,881   (load_yelp.py:12, train[:628881])
  20M      : U=138,493, I=26,744, N=20,000,000 (ML-20M shape, Zipf(1.0) items)

Train rows are grouped by user (as in the NCF-format *.train.rating files), in
draw order inside a user; held-out pairs never appear in train.  Every
generator is deterministic in its seed (numpy Generator / PCG64).
"""
import os
import numpy as np

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "data")

ML1M = dict(name="ml-1m-ex", U=6040, I=3706, N=975460, mean_deg=161.5, min_deg=16, sigma=0.95,
            test_keep=slice(0, -6))          # load_movielens.py:16 test[:-6]
YELP = dict(name="yelp-ex", U=25677, I=25815, N=628881, mean_deg=24.5, min_deg=6, sigma=0.8,
            test_keep=slice(0, 51153))       # load_yelp.py:16 test[:51153]
ML20M = dict(name="synthetic-20m", U=138493, I=26744, N=20000000, mean_deg=144.4, min_deg=16, sigma=0.9)


def load_heldout(name):
    """Real held-out pairs of the reference: dict with test_/valid_ user,item,rating."""
    path = os.path.join(DATA_DIR, name.replace("-", "_") + ".npz")
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_queries(cfg):
    """(users, items, ratings) of the test split after the loader truncation."""
    h = load_heldout(cfg["name"])
    s = cfg["test_keep"]
    return (h["test_user"][s].astype(np.int32), h["test_item"][s].astype(np.int32),
            h["test_rating"][s].astype(np.float64))


def rq1_query_indices(num_test, test_size=12074):
    """RQ1 query choice: np.random.seed(0) (genericNeuralNet.py:83) then
    np.random.choice(test_size, num_test, replace=False) (RQ1.py:132)."""
    st = np.random.get_state()
    try:
        np.random.seed(0)
        return np.random.choice(test_size, num_test, replace=False)
    finally:
        np.random.set_state(st)


def _degrees(rng, U, N, mean_deg, min_deg, sigma, cap):
    mu = np.log(mean_deg) - 0.5 * sigma * sigma
    d = rng.lognormal(mu, sigma, U)
    for _ in range(50):
        d = np.clip(d, min_deg, cap)
        d *= N / d.sum()
        if d.min() >= min_deg - 1e-9 and np.all(d <= cap + 1e-9):
            break
    d = np.clip(d, min_deg, cap)
    base = np.floor(d).astype(np.int64)
    rem = int(N - base.sum())
    frac = d - base
    order = np.argsort(-frac, kind="stable")
    i = 0
    while rem != 0:
        u = order[i % U]
        if rem > 0 and base[u] < cap[u]:
            base[u] += 1
            rem -= 1
        elif rem < 0 and base[u] > min_deg:
            base[u] -= 1
            rem += 1
        i += 1
    return base


def synth_train(U, I, N, heldout_u, heldout_i, item_weight, mean_deg, min_deg, sigma, rating_p, seed):
    """Sample N distinct (user, item) train pairs avoiding the held-out pairs."""
    rng = np.random.default_rng(seed)
    heldout_key = np.unique(heldout_u.astype(np.int64) * I + heldout_i.astype(np.int64))
    held_per_user = np.bincount((heldout_key // I).astype(np.int64), minlength=U)
    cap = (I - held_per_user).astype(np.float64)
    need = _degrees(rng, U, N, mean_deg, min_deg, sigma, cap)
    cdf = np.cumsum(np.asarray(item_weight, np.float64))
    cdf /= cdf[-1]

    taken_keys = np.zeros(0, np.int64)      # accepted pairs (any order)
    chunks_u, chunks_i = [], []
    remaining = need.copy()
    for rnd in range(64):
        users = np.nonzero(remaining > 0)[0]
        if users.size == 0:
            break
        draws = np.ceil(remaining[users] * 1.25).astype(np.int64) + 4
        uu = np.repeat(users, draws)
        if rnd < 48:
            ii = np.searchsorted(cdf, rng.random(uu.size), side="right")
        else:  # stragglers whose popular-item budget is exhausted: uniform items
            ii = rng.integers(0, I, uu.size)
        ii = np.minimum(ii, I - 1)
        key = uu.astype(np.int64) * I + ii
        # first occurrence in draw order, not held out, not already taken
        _, first = np.unique(key, return_index=True)
        first.sort()
        key, uu, ii = key[first], uu[first], ii[first]
        ok = ~np.isin(key, heldout_key) & ~np.isin(key, taken_keys)
        key, uu, ii = key[ok], uu[ok], ii[ok]
        # keep the first remaining[u] per user, in draw order
        order = np.argsort(uu, kind="stable")
        uu, ii, key = uu[order], ii[order], key[order]
        starts = np.searchsorted(uu, users)
        rank = np.arange(uu.size) - np.repeat(starts, np.diff(np.append(starts, uu.size)))
        keep = rank < remaining[uu]
        uu, ii, key = uu[keep], ii[keep], key[keep]
        chunks_u.append(uu)
        chunks_i.append(ii)
        taken_keys = np.union1d(taken_keys, key)
        remaining -= np.bincount(uu, minlength=U)
    if np.any(remaining > 0):
        raise RuntimeError("synthetic sampler could not place every rating")
    users = np.concatenate(chunks_u)
    items = np.concatenate(chunks_i)
    order = np.argsort(users, kind="stable")     # group by user, draw order inside
    users = users[order].astype(np.int32)
    items = items[order].astype(np.int32)
    ratings = (rng.choice(len(rating_p), size=N, p=np.asarray(rating_p) / np.sum(rating_p)) + 1).astype(np.float32)
    assert users.size == N
    return users, items, ratings


def _rating_p(r):
    c = np.bincount(r.astype(np.int64), minlength=6)[1:6].astype(np.float64)
    return c / c.sum()


def make_dataset(cfg, seed=0):
    """Synthetic train + real held-out pairs for ml-1m-ex / yelp-ex.

    Returns dict(train=(u,i,r), test=(u,i,r), valid=(u,i,r), U, I)."""
    h = load_heldout(cfg["name"])
    U, I = cfg["U"], cfg["I"]
    hu = np.concatenate([h["test_user"], h["valid_user"]])
    hi = np.concatenate([h["test_item"], h["valid_item"]])
    pop = np.bincount(hi.astype(np.int64), minlength=I).astype(np.float64) + 1.0
    rp = _rating_p(h["test_rating"])
    tr = synth_train(U, I, cfg["N"], hu, hi, pop, cfg["mean_deg"], cfg["min_deg"], cfg["sigma"], rp, seed)
    s = cfg["test_keep"]
    test = (h["test_user"][s].astype(np.int32), h["test_item"][s].astype(np.int32),
            h["test_rating"][s].astype(np.float64))
    valid = (h["valid_user"].astype(np.int32), h["valid_item"].astype(np.int32),
             h["valid_rating"].astype(np.float64))
    return dict(train=tr, test=test, valid=valid, U=U, I=I)


def make_20m(seed=0, N=None, U=None, I=None):
    """ML-20M-shaped synthetic set: Zipf(1.0) item popularity, log-normal user
    degrees, 2 held-out query pairs per user.

    Generation takes about a minute; with FIA_SYNTH_CACHE=<dir> the arrays are kept
    there as an npz (written by this function, reloaded with allow_pickle=False), so
    several runs inside one job share one draw."""
    cache = os.environ.get("FIA_SYNTH_CACHE")
    if cache:
        path = os.path.join(cache, "synth20m_s%d_%s_%s_%s.npz" % (seed, N, U, I))
        if os.path.exists(path):
            with np.load(path, allow_pickle=False) as z:
                return dict(train=(z["tu"], z["ti"], z["tr"]), test=(z["qu"], z["qi"], z["qr"]), valid=None,
                            U=int(z["U"]), I=int(z["I"]))
        d = _make_20m(seed, N, U, I)
        os.makedirs(cache, exist_ok=True)
        tmp = path + ".%d.tmp.npz" % os.getpid()
        np.savez(tmp, tu=d["train"][0], ti=d["train"][1], tr=d["train"][2], qu=d["test"][0], qi=d["test"][1],
                 qr=d["test"][2], U=d["U"], I=d["I"])
        os.replace(tmp, path)
        return d
    return _make_20m(seed, N, U, I)


def _make_20m(seed, N, U, I):
    cfg = dict(ML20M)
    U = U or cfg["U"]
    I = I or cfg["I"]
    N = N or cfg["N"]
    rng = np.random.default_rng(seed + 1000)
    perm = rng.permutation(I)
    pop = np.empty(I)
    pop[perm] = 1.0 / np.arange(1, I + 1)     # Zipf(1.0) over a random item order
    cdf = np.cumsum(pop) / pop.sum()
    qu = np.repeat(np.arange(U, dtype=np.int32), 2)
    qi = np.empty(2 * U, np.int64)
    a = np.minimum(np.searchsorted(cdf, rng.random(U), side="right"), I - 1)
    b = np.minimum(np.searchsorted(cdf, rng.random(U), side="right"), I - 1)
    b = np.where(b == a, (a + 1 + rng.integers(0, I - 1, U)) % I, b)
    qi[0::2], qi[1::2] = a, b
    qi = qi.astype(np.int32)
    mean_deg = N / U
    rp = (0.06, 0.11, 0.26, 0.34, 0.23)
    tr = synth_train(U, I, N, qu, qi, pop, mean_deg, min(16, int(mean_deg)), cfg["sigma"], rp, seed)
    test = (qu, qi, np.full(qu.shape, 4.0))
    return dict(train=tr, test=test, valid=None, U=U, I=I)


def _truncated_normal(rng, shape, stddev):
    """tf.truncated_normal_initializer: N(0, stddev) redrawn beyond 2 stddev
    (genericNeuralNet.py:57)."""
    out = rng.standard_normal(shape)
    bad = np.abs(out) > 2.0
    while bad.any():
        out[bad] = rng.standard_normal(int(bad.sum()))
        bad = np.abs(out) > 2.0
    return (out * stddev).astype(np.float32)


def mf_params(U, I, k, seed=0, bias_std=0.1, global_bias=3.60):
    """Parameter dict keyed by the reference variable names (matrix_factorization.py:30-36)."""
    rng = np.random.default_rng(seed + 7)
    s = 1.0 / np.sqrt(k)
    return {
        "embedding_layer/embedding_users": _truncated_normal(rng, (U * k,), s),
        "embedding_layer/embedding_items": _truncated_normal(rng, (I * k,), s),
        "embedding_layer/bias_users": (rng.standard_normal(U) * bias_std).astype(np.float32),
        "embedding_layer/bias_items": (rng.standard_normal(I) * bias_std).astype(np.float32),
        "embedding_layer/global_bias": np.array([global_bias], np.float32),
    }


def ncf_params(U, I, k, seed=0, bias_std=0.1):
    """NCF parameter dict keyed by the reference names (NCF.py:29-41, 85-145)."""
    if k % 2:
        raise ValueError("NCF needs an even embedding size (h2 has k/2 units, NCF.py:141)")
    rng = np.random.default_rng(seed + 11)
    s = 1.0 / np.sqrt(k)
    h = k // 2
    return {
        "embedding_layer/mlp/embedding_users": _truncated_normal(rng, (U * k,), s),
        "embedding_layer/mlp/embedding_items": _truncated_normal(rng, (I * k,), s),
        "embedding_layer/gmf/embedding_users": _truncated_normal(rng, (U * k,), s),
        "embedding_layer/gmf/embedding_items": _truncated_normal(rng, (I * k,), s),
        "h1/weights": _truncated_normal(rng, (2 * k * k,), 1.0 / np.sqrt(2 * k)),
        "h1/biases": (rng.standard_normal(k) * bias_std).astype(np.float32),
        "h2/weights": _truncated_normal(rng, (k * h,), 1.0 / np.sqrt(k)),
        "h2/biases": (rng.standard_normal(h) * bias_std).astype(np.float32),
        "h3/weights": _truncated_normal(rng, (3 * h,), 1.0 / np.sqrt(3 * h)),
        "h3/biases": np.array([3.6], np.float32),
    }


MF_PARAM_NAMES = ["embedding_layer/embedding_users", "embedding_layer/embedding_items",
                  "embedding_layer/bias_users", "embedding_layer/bias_items",
                  "embedding_layer/global_bias"]
NCF_PARAM_NAMES = ["embedding_layer/mlp/embedding_users", "embedding_layer/mlp/embedding_items",
                   "embedding_layer/gmf/embedding_users", "embedding_layer/gmf/embedding_items",
                   "h1/weights", "h1/biases", "h2/weights", "h2/biases", "h3/weights", "h3/biases"]
