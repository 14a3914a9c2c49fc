"""GPU: trainer (HIP-graph retrain), RQ1 leave-one-out harness, checkpoints
(SURVEY.md 8f rows 1-3)."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _model(kind, data, k=8, tmp="output", batch=500, lr=1e-2):
    from influence.matrix_factorization import MF
    from influence.NCF import NCF
    x = data["train"].x
    cls = MF if kind == "MF" else NCF
    return cls(num_users=int(x[:, 0].max()) + 1, num_items=int(x[:, 1].max()) + 1, embedding_size=k,
               weight_decay=1e-3, num_classes=1, batch_size=batch, data_sets=data, initial_learning_rate=lr,
               damping=1e-6, decay_epochs=[10000, 20000], train_dir=str(tmp), avextol=1e-3,
               model_name="t_%s" % kind, verbose=False, save_inverse_hvp=False)


@pytest.mark.parametrize("kind", ["MF", "NCF"])
def test_graph_retrain_matches_eager(kind, tmp_path):
    """retrain_full_batch() replays one captured HIP graph per full-batch step; it must follow
    the eager steps (embedding-gradient atomics reorder fp32 sums: tolerance, not bits)."""
    from rq1_small import small_data
    m = _model(kind, small_data(), tmp=tmp_path)
    tr = m.trainer()
    f = m.fill_feed_dict_with_all_ex(m.data_sets["train"])
    p0, s0 = tr.params_numpy(), tr.opt.state()
    for _ in range(40):
        tr.step(f["users"], f["items"], f["labels"])
    eager = tr.params_numpy()
    tr.set_params(p0)
    tr.opt.load_state(s0)
    m.retrain_full_batch(40, f)
    graph = tr.params_numpy()
    for n in m.PARAM_NAMES:
        assert np.allclose(graph[n], eager[n], rtol=1e-4, atol=1e-6), n
    assert abs(tr.opt.state()["b1p"] - 0.9 ** 41) < 1e-6


def test_rq1_harness_mf(tmp_path):
    """Train, maxinf, leave-one-out retraining: FIA's predicted change of r-hat(test)
    tracks the retrained change (the reference's RQ1 Pearson check, RQ1.py:139-165)."""
    from rq1_small import small_data
    from scripts.RQ1 import run, configs
    cfg = dict(configs, model="MF", embed_size=8, num_steps_train=3000, num_steps_retrain=1000, num_test=6,
               retrain_times=1, batch_size=500, lr=1e-2, dataset="small")
    out = run(cfg, data_sets=small_data(), train_dir=str(tmp_path), verbose=False)
    a, p = out["actual"], out["predicted"]
    assert np.isfinite(a).all() and np.isfinite(p).all()
    assert out["corr"] > 0.7, (a, p)
    assert (np.sign(a) == np.sign(p)).sum() >= 5
    # the predicted diff is FIA's top-1 |influence| of the query, from the trained model
    m = out["model"]
    for j, t in enumerate(out["test_indices"]):
        res = m.get_influence_batch([int(t)], K=1)
        want = res["topk_val"][0][0]
        assert p[j] == (want if abs(want) <= 1 else 0.0)
        assert out["removed"][j] == res["topk_pos"][0][0]
    assert os.path.exists(os.path.join(str(tmp_path), "RQ1-MF-small.npz"))


@pytest.mark.parametrize("kind", ["MF", "NCF"])
def test_tf_checkpoint_into_model(kind, tmp_path):
    """A TF checkpoint-V2 bundle under the reference names loads into the model and gives
    bit-identical influence to the same parameters passed directly; Adam slots restore."""
    from rq1_small import small_data
    from influence import synth
    data = small_data()
    m = _model(kind, data, tmp=tmp_path)
    U, I, k = m.num_users, m.num_items, m.embedding_size
    p = synth.mf_params(U, I, k, 9) if kind == "MF" else synth.ncf_params(U, I, k, 9)
    m.load_params(p)
    want = m.get_influence_batch([0, 1, 2], K=2)
    m.trainer()
    m.train(num_steps=30, verbose=False, save_checkpoints=False)
    prefix = m.save_tf_checkpoint(str(tmp_path / "tf" / ("t_%s-checkpoint-29" % kind)))
    st = m.trainer().opt.state()
    trained = m.get_influence_batch([0, 1, 2], K=2)
    m.load_params(p)
    assert np.array_equal(m.get_influence_batch([0, 1, 2], K=2)["influence"], want["influence"])
    m.trainer().opt.reset()
    m.load_tf_checkpoint(prefix)
    again = m.get_influence_batch([0, 1, 2], K=2)
    for key in ("influence", "rel_idx", "x", "topk_pos"):
        assert np.array_equal(again[key], trained[key]), key
    st2 = m.trainer().opt.state()
    assert st2["b1p"] == st["b1p"] and all(np.array_equal(a, b) for a, b in zip(st["m"], st2["m"]))
