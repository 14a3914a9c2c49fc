"""Rating container with the reference's x/labels semantics.

Mirrors the parts of the reference ``DataSet`` (src/influence/dataset.py:5-33)
that the FIA path reads: ``x`` is stored as float32 (dataset.py:14), labels
keep the loader's dtype (float64 from np.loadtxt, load_movielens.py:12-13),
and ``num_examples`` is the row count.  ``next_batch`` / ``reset_batch`` keep the
reference's mini-batch order exactly (dataset.py:36-70): sequential batches, a
short final batch, then a global-``np.random`` shuffle of the batch copy.

Added for the device path: ``users`` / ``items`` int32 views of the id
columns (ids are exact in float32 below 2**24, which the reference relies on
when it compares ``x[:, 0] == test_u`` at matrix_factorization.py:320).
"""
import numpy as np


class DataSet(object):
    def __init__(self, x, labels):
        x = np.asarray(x)
        labels = np.asarray(labels)
        if x.ndim > 2:
            x = x.reshape(x.shape[0], -1)
        if x.shape[0] != labels.shape[0]:
            raise ValueError("x has %d rows but labels has %d" % (x.shape[0], labels.shape[0]))
        ids = np.asarray(x[:, :2])
        if ids.size and (ids.min() < 0 or ids.max() >= 2 ** 24):
            raise ValueError("user/item ids must lie in [0, 2**24) to stay exact in float32")
        self._x = x.astype(np.float32)
        self._labels = labels
        self._users = np.ascontiguousarray(ids[:, 0].astype(np.int32)) if ids.size else np.zeros(0, np.int32)
        self._items = np.ascontiguousarray(ids[:, 1].astype(np.int32)) if ids.size else np.zeros(0, np.int32)
        self._num_examples = x.shape[0]
        self._x_batch = np.copy(self._x)
        self._labels_batch = np.copy(self._labels)
        self._index_in_epoch = 0

    def reset_batch(self):
        self._index_in_epoch = 0
        self._x_batch = np.copy(self._x)
        self._labels_batch = np.copy(self._labels)

    def next_batch(self, batch_size):
        """Reference mini-batch order (dataset.py:49-70)."""
        start = self._index_in_epoch
        self._index_in_epoch += batch_size
        if self._index_in_epoch > self._num_examples:
            if self._index_in_epoch < self._num_examples + batch_size:
                self._index_in_epoch = self._num_examples
            else:
                perm = np.arange(self._num_examples)
                np.random.shuffle(perm)
                self._x_batch = self._x_batch[perm, :]
                self._labels_batch = self._labels_batch[perm]
                start = 0
                self._index_in_epoch = batch_size
        end = self._index_in_epoch
        return self._x_batch[start:end], self._labels_batch[start:end]

    @property
    def x(self):
        return self._x

    @property
    def labels(self):
        return self._labels

    @property
    def num_examples(self):
        return self._num_examples

    @property
    def users(self):
        return self._users

    @property
    def items(self):
        return self._items
