"""Re-encode the reference's held-out rating files as compact npz data.

Run ONLY in the build container (reads /root/reference/data, which does not
exist on the GPU box).  The outputs are data (user, item, rating triples of
the reference's own valid/test files), stored under fia-kdd-19_amd/data/ so
the loaders, tests and bench can use the real test queries anywhere.

Sources: /root/reference/data/ml-1m-ex.{valid,test}.rating and
yelp-ex.{valid,test}.rating (tab separated "u i r", read by
src/scripts/load_movielens.py:9-10 and load_yelp.py:9-10 with np.loadtxt).
"""
import os
import numpy as np

REF = "/root/reference/data"
OUT = os.path.join(os.path.dirname(__file__), "..", "fia-kdd-19_amd", "data")


def main():
    os.makedirs(OUT, exist_ok=True)
    for name in ("ml-1m-ex", "yelp-ex"):
        arrs = {}
        for split in ("valid", "test"):
            a = np.loadtxt(os.path.join(REF, "%s.%s.rating" % (name, split)), delimiter="\t")
            assert np.all(a == np.round(a))
            arrs[split + "_user"] = a[:, 0].astype(np.int32)
            arrs[split + "_item"] = a[:, 1].astype(np.int32)
            arrs[split + "_rating"] = a[:, 2].astype(np.int8)
        path = os.path.join(OUT, name.replace("-", "_") + ".npz")
        np.savez_compressed(path, **arrs)
        print(path, {k: v.shape for k, v in arrs.items()}, os.path.getsize(path))


if __name__ == "__main__":
    main()
