"""Experiment callers of the FIA path (reference src/influence/experiments.py).

record_time_cost mirrors experiments.py:4-15 (RQ2 timing of one query).
maxinf mirrors the top-K selection of test_retraining (experiments.py:36-53):
argsort(|predicted|)[-K:][::-1] mapped back through train_indices_of_test_case,
with ties broken by related position (the reference's quicksort leaves them
unspecified).  Leave-one-out retraining (experiments.py:55-150) is training
and is not part of this build.
"""
import numpy as np


def record_time_cost(model, test_idx, iter_to_load=None, force_refresh=False, random_seed=17):
    np.random.seed(random_seed)
    if iter_to_load is not None:
        model.load_checkpoint(iter_to_load)
    approx_params = {"batch_size": model.batch_size, "damping": model.damping}
    model.get_influence_on_test_loss([test_idx], np.arange(len(model.data_sets["train"].labels)),
                                     force_refresh=force_refresh, approx_params=approx_params)
    return 0


def maxinf(model, test_idx, num_to_remove=1):
    """(predicted_y_diffs[top], indices_to_remove (related positions), train rows), computed
    on the GPU by the fused top-K of fia_query_batch."""
    res = model.get_influence_batch([test_idx], K=num_to_remove, full=True, return_x=False)
    pos = res["topk_pos"][0]
    keep = pos >= 0
    model.train_indices_of_test_case = res["rel_idx"]
    return res["topk_val"][0][keep], pos[keep], res["topk_idx"][0][keep]
