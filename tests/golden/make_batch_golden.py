"""Golden mini-batch order of the reference DataSet (run in the build container).

    python tests/golden/make_batch_golden.py

Imports the reference's numpy-only DataSet (/root/reference/src/influence/
dataset.py:49-70) by path, seeds np.random, and records the label order of a
sequence of next_batch calls (sequential batches, short last batch, shuffle of
the batch copy at the wrap) for two shapes.  tests/test_train.py replays the same
calls on influence.dataset.DataSet and requires the identical order -- the
trainer's mini-batches are the reference's.
"""
import importlib.util
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = [(10, 4, 9), (3020 * 2 + 7, 3020, 7)]     # (num_examples, batch_size, calls)


def main():
    spec = importlib.util.spec_from_file_location("ref_dataset", "/root/reference/src/influence/dataset.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = {}
    for c, (n, bs, calls) in enumerate(CASES):
        np.random.seed(0)
        ds = mod.DataSet(np.stack([np.arange(n), np.arange(n) % 7], 1), np.arange(n, dtype=np.float64))
        order = [ds.next_batch(bs)[1] for _ in range(calls)]
        out["case%d_lens" % c] = np.array([o.size for o in order])
        out["case%d_labels" % c] = np.concatenate(order)
        out["case%d_shape" % c] = np.array([n, bs, calls])
    np.savez_compressed(os.path.join(HERE, "batch_order.npz"), **out)
    print("wrote batch_order.npz")


if __name__ == "__main__":
    main()
