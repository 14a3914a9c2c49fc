"""Generate the committed golden fixtures (run in the build container).

    python tests/golden/make_golden.py

Each fixture holds inputs (params, train ratings, queries) and the expected
outputs of the fp64 closed-form oracle (oracle/fia_oracle.py): related set,
x = H^-1 v (reference theta order), influence vector, top-K positions.  Every
expected output is cross-checked here against the torch double-backward
restatement of the TF graph (oracle/autograd_oracle.py) before it is written,
and the reference-solver result (scipy fmin_ncg with the reference arguments,
oracle/ncg_port.py, fp32 HVPs as TF computes them) is stored beside it to
record the documented CG-vs-exact gap.

Also pins the pieces of the reference that CAN run here: the reference's own
DataSet class (/root/reference/src/influence/dataset.py, numpy-only) is imported
to build the float32 x arrays the related-set scans compare against
(matrix_factorization.py:318-321), and the RQ1 query choice is checked against
the known answer listed in SURVEY.md 8d.
"""
import hashlib
import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fia-kdd-19_amd"))

from influence import synth  # noqa: E402
from oracle import fia_oracle as fo, autograd_oracle as ao, ncg_port  # noqa: E402

WD, DAMP, K_TOP = 1e-3, 1e-6, 5


def reference_dataset_cls():
    path = "/root/reference/src/influence/dataset.py"
    if not os.path.exists(path):
        return None
    spec = importlib.util.spec_from_file_location("ref_dataset", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.DataSet


def small_problem(seed=1, U=50, I=40, N=800):
    """Random distinct pairs; user U-1 and item I-1 have no train ratings; one pair
    is duplicated (same (u,i) twice) to exercise the multi-dup Hessian terms."""
    rng = np.random.default_rng(seed)
    key = rng.choice((U - 1) * (I - 1), N - 1, replace=False)
    key.sort()
    tu = (key // (I - 1)).astype(np.int32)
    ti = (key % (I - 1)).astype(np.int32)
    tu = np.append(tu, tu[7])                 # duplicate of row 7 at the end
    ti = np.append(ti, ti[7])
    tr = rng.integers(1, 6, N).astype(np.float32)
    in_train = set(zip(tu.tolist(), ti.tolist()))
    plain = []
    for c in rng.permutation((U - 1) * (I - 1)):
        pair = (int(c // (I - 1)), int(c % (I - 1)))
        if pair not in in_train:
            plain.append(pair)
        if len(plain) == 3:
            break
    # plain (held out, as real test pairs are), the pair itself in train (indefinite
    # H possible), the pair twice in train, empty user side, empty item side, n = 0
    queries = [plain[0], (int(tu[10]), int(ti[10])), (int(tu[7]), int(ti[7])),
               (U - 1, 6), (12, I - 1), (U - 1, I - 1), plain[1], plain[2]]
    return U, I, tu, ti, tr, queries


def run_queries(model, params, k, U, I, tu, ti, tr, queries, autograd=True, ncg=True):
    out = {"q_user": np.array([q[0] for q in queries], np.int32),
           "q_item": np.array([q[1] for q in queries], np.int32)}
    rel_all, infl_all, x_all, topk_all, offs = [], [], [], [], [0]
    x_ncg_all, infl_ncg_all = [], []
    port = ncg_port.RefAlgorithm(model, params, k, tu, ti, tr, WD, DAMP) if ncg else None
    for (u, i) in queries:
        o = fo.query(model, params, k, tu, ti, tr, u, i, WD, DAMP)
        if autograd:
            a = ao.query(model, params, k, U, I, tu, ti, tr, u, i, WD, DAMP)
            assert np.array_equal(a["rel"], o["rel"])
            if o["n"] > 0:
                sx = np.abs(o["x"]).max()
                si = np.abs(o["influence"]).max()
                assert np.abs(a["x"] - o["x"]).max() <= 1e-10 * sx, (model, u, i)
                assert np.abs(a["influence"] - o["influence"]).max() <= 1e-10 * si, (model, u, i)
        rel_all.append(o["rel"])
        infl_all.append(o["influence"])
        x_all.append(o["x"])
        tk = fo.topk(o["influence"], K_TOP)
        topk_all.append(np.concatenate([tk, -np.ones(K_TOP - tk.size, np.int64)]))
        offs.append(offs[-1] + o["rel"].size)
        if port is not None:
            _, infl_n, x_n, _ = port.get_influence_on_test_loss(u, i)
            x_ncg_all.append(x_n)
            infl_ncg_all.append(infl_n)
    out.update(offsets=np.array(offs, np.int64), rel=np.concatenate(rel_all).astype(np.int64),
               influence=np.concatenate(infl_all), x=np.stack(x_all), topk_pos=np.stack(topk_all))
    if port is not None:
        out.update(x_ncg=np.stack(x_ncg_all), influence_ncg=np.concatenate(infl_ncg_all))
    return out


def save(name, **arrs):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrs)
    print("wrote", path, os.path.getsize(path), "bytes")


def params_arrays(prefix, params):
    return {prefix + n.replace("/", "__"): v for n, v in params.items()}


def main():
    RefDataSet = reference_dataset_cls()
    assert list(synth.rq1_query_indices(10)) == [2712, 2168, 4934, 5235, 7786, 9434, 5490, 9180, 11139, 10884]

    U, I, tu, ti, tr, queries = small_problem()
    if RefDataSet is not None:
        # related-set semantics through the reference's own DataSet (x -> float32)
        ds = RefDataSet(np.stack([tu, ti], 1), tr.astype(np.float64))
        for (u, i) in queries:
            want = np.concatenate((np.where(ds.x[:, 0] == u)[0], np.where(ds.x[:, 1] == i)[0]))
            assert np.array_equal(want, fo.related_indices(ds.x, u, i))
    for model, k in (("MF", 16), ("NCF", 16), ("MF", 8), ("NCF", 8)):
        params = synth.mf_params(U, I, k, seed=3) if model == "MF" else synth.ncf_params(U, I, k, seed=3)
        res = run_queries(model, params, k, U, I, tu, ti, tr, queries)
        save("small_%s_k%d.npz" % (model.lower(), k), U=U, I=I, k=k, wd=WD, damping=DAMP, K_top=K_TOP,
             train_user=tu, train_item=ti, train_rating=tr, **params_arrays("p__", params), **res)

    # ML-1M-ex shaped: 5 RQ1 queries (real test pairs) over the synthetic train set
    d = synth.make_dataset(synth.ML1M, seed=0)
    tu, ti, tr = d["train"]
    digest = hashlib.sha256(tu.tobytes() + ti.tobytes() + tr.tobytes()).hexdigest()
    qu, qi, _ = d["test"]
    idx = synth.rq1_query_indices(5)
    qs = [(int(qu[t]), int(qi[t])) for t in idx]
    for model, k in (("MF", 16), ("NCF", 16)):
        params = synth.mf_params(d["U"], d["I"], k, 0) if model == "MF" else synth.ncf_params(d["U"], d["I"], k, 0)
        res = run_queries(model, params, k, d["U"], d["I"], tu, ti, tr, qs, autograd=False, ncg=True)
        save("ml1m_rq1_%s_k%d.npz" % (model.lower(), k), U=d["U"], I=d["I"], k=k, wd=WD, damping=DAMP,
             K_top=K_TOP, test_indices=idx, train_sha256=np.array(digest), **res)


if __name__ == "__main__":
    main()
