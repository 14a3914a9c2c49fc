"""RQ1: does FIA predict the effect of removing a training rating?  (reference
src/scripts/RQ1.py)

Train MF/NCF (influence/train.py, TF-Adam), then for num_test test ratings
remove the most influential related training rating (maxinf), retrain from
the checkpoint without it retrain_times times, and correlate the actual change
of r-hat(test) with FIA's prediction (pearsonr, RQ1.py:165).

The reference hard-codes its configs (RQ1.py:18-34; its argparse is
commented out, RQ1.py:36-64); this script keeps the same dict and accepts
--key value overrides.  Its train file is not distributed (.MISSING_LARGE_BLOBS),
so the train set is the synthetic one of the same shape (scripts/load_*.py)
with the reference's real held-out test pairs.

    python fia-kdd-19_amd/scripts/RQ1.py --num_steps_train 20000 --num_steps_retrain 2000
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

configs = {
    "avextol": 1e-3,
    "damping": 1e-6,
    "weight_decay": 1e-3,
    "lr": 1e-3,
    "embed_size": 16,
    "maxinf": 1,
    "dataset": "movielens",
    "model": "MF",
    "num_test": 5,
    "num_steps_train": 180000,
    "num_steps_retrain": 27000,
    "reset_adam": 0,
    "load_checkpoint": 1,
    "retrain_times": 4,
    "sort_test_case": 0,
}


def run(cfg, data_sets=None, train_dir="output", verbose=True, device=0):
    from scipy.stats import pearsonr
    import influence.experiments as experiments
    from influence.matrix_factorization import MF
    from influence.NCF import NCF
    if data_sets is None:
        if cfg["dataset"] == "movielens":
            from scripts.load_movielens import load_movielens_synthetic
            data_sets = load_movielens_synthetic(0)
        elif cfg["dataset"] == "yelp":
            from scripts.load_yelp import load_yelp_synthetic
            data_sets = load_yelp_synthetic(0)
        else:
            raise NotImplementedError(cfg["dataset"])
    batch_size = cfg.get("batch_size", 3020 if cfg["dataset"] == "movielens" else 3009)   # RQ1.py:67-72
    train_x = data_sets["train"].x
    num_users = int(cfg.get("num_users", int(np.max(train_x[:, 0])) + 1))
    num_items = int(cfg.get("num_items", int(np.max(train_x[:, 1])) + 1))
    Model = MF if cfg["model"] == "MF" else NCF
    model = Model(num_users=num_users, num_items=num_items, embedding_size=cfg["embed_size"],
                  weight_decay=cfg["weight_decay"], num_classes=1, batch_size=batch_size, data_sets=data_sets,
                  initial_learning_rate=cfg["lr"], damping=cfg["damping"], decay_epochs=[10000, 20000],
                  mini_batch=True, train_dir=train_dir, log_dir="log", avextol=cfg["avextol"],
                  model_name="%s_%s_explicit_damping%.0e_avextol%.0e_embed%d_maxinf%d_wd%.0e" % (
                      cfg["dataset"], cfg["model"], cfg["damping"], cfg["avextol"], cfg["embed_size"],
                      cfg["maxinf"], cfg["weight_decay"]),
                  device=device, verbose=verbose, save_inverse_hvp=False)
    num_steps = cfg["num_steps_train"]
    iter_to_load = num_steps - 1
    model.train(num_steps=num_steps, verbose=verbose)
    test_size = data_sets["test"].num_examples
    num_test = cfg["num_test"]
    test_indices = np.random.choice(test_size, num_test, replace=False)
    if cfg["sort_test_case"]:
        n_rel = [model.get_train_indices_of_test_case([t]).shape[0] for t in range(test_size)]
        test_indices = np.argsort(np.array(n_rel))[:num_test]
    actual = np.zeros(num_test)
    predicted = np.zeros(num_test)
    removed = np.zeros(num_test)
    for j, t in enumerate(test_indices):
        a, p, idx = experiments.test_retraining(
            model, test_idx=int(t), iter_to_load=iter_to_load, retrain_times=cfg["retrain_times"], num_to_remove=1,
            num_steps=cfg["num_steps_retrain"], remove_type="maxinf" if cfg["maxinf"] else "random",
            force_refresh=True, reset_adam=cfg["reset_adam"], load_checkpoint=cfg["load_checkpoint"],
            verbose=verbose)
        actual[j], predicted[j], removed[j] = a[0], p[0], idx[0]
    os.makedirs(train_dir, exist_ok=True)
    np.savez(os.path.join(train_dir, "RQ1-%s-%s.npz" % (cfg["model"], cfg["dataset"])),
             actual_loss_diffs=actual, predicted_loss_diffs=predicted, indices_to_remove=removed)
    corr = pearsonr(actual, predicted)[0] if num_test > 1 else float("nan")
    if verbose:
        print("Correlation is %s" % corr)
    return dict(actual=actual, predicted=predicted, removed=removed, test_indices=test_indices, corr=corr,
                model=model)


def main():
    ap = argparse.ArgumentParser()
    for k, v in configs.items():
        ap.add_argument("--" + k, type=type(v), default=v)
    ap.add_argument("--train_dir", default="output")
    args = vars(ap.parse_args())
    train_dir = args.pop("train_dir")
    run(args, train_dir=train_dir)


if __name__ == "__main__":
    main()
