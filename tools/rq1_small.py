"""Small RQ1 run on the GPU (trainer + FIA maxinf + leave-one-out retraining):
    python tools/rq1_small.py [MF|NCF] [train_steps] [retrain_steps] [num_test]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fia-kdd-19_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from influence.dataset import DataSet  # noqa: E402


def small_data(U=300, I=150, N=6000, seed=0):
    rng = np.random.default_rng(seed)
    key = np.sort(rng.choice(U * I, N + 40, replace=False))
    u, i = (key // I).astype(np.int32), (key % I).astype(np.int32)
    P = rng.standard_normal((U, 4)) * 0.7
    Q = rng.standard_normal((I, 4)) * 0.7
    r = np.clip(np.round(3.5 + (P[u] * Q[i]).sum(1) + rng.standard_normal(u.size) * 0.3), 1, 5)
    te = rng.choice(u.size, 40, replace=False)
    tr_mask = np.ones(u.size, bool)
    tr_mask[te] = False
    return {"train": DataSet(np.stack([u[tr_mask], i[tr_mask]], 1), r[tr_mask]),
            "validation": None, "test": DataSet(np.stack([u[te], i[te]], 1), r[te])}


if __name__ == "__main__":
    from scripts.RQ1 import run, configs
    model = sys.argv[1] if len(sys.argv) > 1 else "MF"
    cfg = dict(configs, model=model, embed_size=8, num_steps_train=int(sys.argv[2]) if len(sys.argv) > 2 else 3000,
               num_steps_retrain=int(sys.argv[3]) if len(sys.argv) > 3 else 1000,
               num_test=int(sys.argv[4]) if len(sys.argv) > 4 else 8, retrain_times=1, batch_size=500,
               lr=1e-2, dataset="small")
    t0 = time.time()
    out = run(cfg, data_sets=small_data(), train_dir=os.path.join(ROOT, "gpurun_out", "rq1"), verbose=False)
    print("model", model, "corr %.4f" % out["corr"], "time %.1f s" % (time.time() - t0))
    print("actual   ", np.round(out["actual"], 5))
    print("predicted", np.round(out["predicted"], 5))
