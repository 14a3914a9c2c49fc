"""ml-1m-ex loader (reference src/scripts/load_movielens.py:6-25).

load_movielens(train_dir) reads <train_dir>/ml-1m-ex.{train,valid,test}.rating
with the reference's truncations (train[:975460], valid/test[:-6]).  The
reference's train file is not distributed, so load_movielens_synthetic() pairs a
synthetic train set of the same shape with the real held-out pairs.
"""
import numpy as np

from influence.dataset import DataSet
from influence import synth


def load_movielens(train_dir, validation_size=5000):
    train = np.loadtxt("%s/ml-1m-ex.train.rating" % train_dir, delimiter="\t")
    valid = np.loadtxt("%s/ml-1m-ex.valid.rating" % train_dir, delimiter="\t")
    test = np.loadtxt("%s/ml-1m-ex.test.rating" % train_dir, delimiter="\t")
    return {"train": DataSet(train[:975460, :2].astype(np.int32), train[:975460, 2]),
            "validation": DataSet(valid[:-6, :2].astype(np.int32), valid[:-6, 2]),
            "test": DataSet(test[:-6, :2].astype(np.int32), test[:-6, 2])}


def load_movielens_synthetic(seed=0):
    d = synth.make_dataset(synth.ML1M, seed)
    return _to_datasets(d)


def _to_datasets(d):
    (tu, ti, tr), (su, si, sr) = d["train"], d["test"]
    out = {"train": DataSet(np.stack([tu, ti], 1), tr.astype(np.float64)),
           "test": DataSet(np.stack([su, si], 1), sr)}
    if d.get("valid") is not None:
        vu, vi, vr = d["valid"]
        out["validation"] = DataSet(np.stack([vu, vi], 1), vr)
    else:
        out["validation"] = None
    return out
