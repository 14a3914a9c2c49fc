"""yelp-ex loader (reference src/scripts/load_yelp.py:6-25): train[:628881],
test[:51153]; load_yelp_synthetic() pairs a synthetic train set of that shape
with the real held-out pairs."""
import numpy as np

from influence.dataset import DataSet
from influence import synth
from scripts.load_movielens import _to_datasets


def load_yelp(train_dir):
    train = np.loadtxt("%s/yelp-ex.train.rating" % train_dir, delimiter="\t")
    valid = np.loadtxt("%s/yelp-ex.valid.rating" % train_dir, delimiter="\t")
    test = np.loadtxt("%s/yelp-ex.test.rating" % train_dir, delimiter="\t")
    return {"train": DataSet(train[:628881, :2].astype(np.int32), train[:628881, 2]),
            "validation": DataSet(valid[:, :2].astype(np.int32), valid[:, 2]),
            "test": DataSet(test[:51153, :2].astype(np.int32), test[:51153, 2])}


def load_yelp_synthetic(seed=0):
    return _to_datasets(synth.make_dataset(synth.YELP, seed))
