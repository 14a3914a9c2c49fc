"""Trainer (influence/train.py) on the CPU: the reference's
mini-batch order, the TF-Adam update, the loss, and full-batch retraining."""
import os

import numpy as np
import pytest

from conftest import GOLDEN


def test_next_batch_matches_reference_order():
    """influence.dataset.DataSet.next_batch == the reference DataSet (golden file made by
    tests/golden/make_batch_golden.py from /root/reference/src/influence/dataset.py)."""
    from influence.dataset import DataSet
    with np.load(os.path.join(GOLDEN, "batch_order.npz"), allow_pickle=False) as z:
        for c in range(2):
            n, bs, calls = z["case%d_shape" % c]
            np.random.seed(0)
            ds = DataSet(np.stack([np.arange(n), np.arange(n) % 7], 1), np.arange(n, dtype=np.float64))
            got = [ds.next_batch(int(bs))[1] for _ in range(int(calls))]
            assert np.array_equal([g.size for g in got], z["case%d_lens" % c])
            assert np.array_equal(np.concatenate(got), z["case%d_labels" % c])


def _numpy_tf_adam(p, grads, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8):
    """tf.train.AdamOptimizer, written out: m, v, lr_t = lr sqrt(1-b2^t)/(1-b1^t)."""
    p = p.astype(np.float64).copy()
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    for t, g in enumerate(grads, 1):
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        lr_t = lr * np.sqrt(1 - b2 ** t) / (1 - b1 ** t)
        p = p - lr_t * m / (np.sqrt(v) + eps)
    return p


def test_tf_adam_update():
    import torch
    from influence.train import TFAdam
    rng = np.random.default_rng(0)
    p0 = rng.standard_normal(7).astype(np.float32)
    grads = [rng.standard_normal(7).astype(np.float32) for _ in range(4)]
    p = torch.tensor(p0)
    opt = TFAdam([p], lr=1e-2)
    for g in grads:
        opt.step([torch.tensor(g)])
    want = _numpy_tf_adam(p0, grads, lr=1e-2)
    assert np.allclose(p.numpy(), want, rtol=1e-5, atol=1e-6)
    st = opt.state()
    assert np.isclose(st["b1p"], 0.9 ** 5) and np.isclose(st["b2p"], 0.999 ** 5, rtol=1e-6)


@pytest.mark.parametrize("model", ["MF", "NCF"])
def test_loss_matches_oracle_and_training_descends(model):
    """total_loss = mean squared error + wd/2 * (decayed norms) (mf:122-132, gnn:40-65),
    checked against the fp64 oracle's prediction; then Adam steps lower the loss and
    full_batch(n) == n eager steps."""
    from influence import synth
    from influence.train import Trainer, DECAYED
    from influence.matrix_factorization import MF
    from influence.NCF import NCF
    from oracle import fia_oracle as fo
    rng = np.random.default_rng(3)
    U, I, N, k, wd = 30, 20, 300, 8, 1e-3
    tu = rng.integers(0, U, N)
    ti = rng.integers(0, I, N)
    y = rng.integers(1, 6, N).astype(np.float32)
    p = synth.mf_params(U, I, k, 1) if model == "MF" else synth.ncf_params(U, I, k, 1)
    names = (MF if model == "MF" else NCF).PARAM_NAMES
    tr = Trainer(model, k, wd, 1e-2, p, names, "cpu")
    pred = fo.mf_predict(p, k, tu, ti) if model == "MF" else fo.ncf_predict(p, k, tu, ti)
    want = np.mean((pred - y) ** 2) + 0.5 * wd * sum(float(np.sum(p[n].astype(np.float64) ** 2))
                                                     for n in DECAYED[model])
    assert abs(tr.loss(tu, ti, y) - want) < 1e-5 * max(1.0, want)
    l0 = tr.loss(tu, ti, y)
    for _ in range(30):
        tr.step(tu, ti, y)
    assert tr.loss(tu, ti, y) < l0
    a = Trainer(model, k, wd, 1e-2, p, names, "cpu")
    b = Trainer(model, k, wd, 1e-2, p, names, "cpu")
    for _ in range(5):
        a.step(tu, ti, y)
    b.full_batch(tu, ti, y, 5)
    pa, pb = a.params_numpy(), b.params_numpy()
    for n in names:
        assert np.array_equal(pa[n], pb[n])
