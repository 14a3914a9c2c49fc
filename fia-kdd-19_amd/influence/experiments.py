"""Experiment callers of the FIA path (reference src/influence/experiments.py).

record_time_cost mirrors experiments.py:4-15 (RQ2 timing of one query).
maxinf mirrors the top-K selection of test_retraining (experiments.py:36-53):
argsort(|predicted|)[-K:][::-1] mapped back through train_indices_of_test_case,
with ties broken by related position (the reference's quicksort leaves them
unspecified); the selection is the fused top-K of fia_query_batch.
test_retraining is the RQ1 validation harness (experiments.py:17-150,
SURVEY.md 8f row 2): predicted influence of the top training ratings vs the
change of r-hat(test) after leave-one-out retraining (influence/train.py).
"""
import os

import numpy as np


def record_time_cost(model, test_idx, iter_to_load=None, force_refresh=False, random_seed=17):
    """experiments.py:4-15: one FIA query, timed.  The reference returns 0 and prints the
    three stage timers; this returns them too (model.last_timing: inverse_hvp_s,
    multiply_s, total_s, wall_s, n)."""
    np.random.seed(random_seed)
    if iter_to_load is not None:
        model.load_checkpoint(iter_to_load)
    approx_params = {"batch_size": model.batch_size, "damping": model.damping}
    model.get_influence_on_test_loss([test_idx], np.arange(len(model.data_sets["train"].labels)),
                                     force_refresh=force_refresh, approx_params=approx_params)
    return model.last_timing


def total_y_diffs_path(model, test_idx):
    """experiments.py:43: np.save("output/%s-[%s]-_total_y_diffs" % (model_name, test_idx)) --
    under the model's train_dir (the reference hard-codes output/, its default train_dir)."""
    return os.path.join(model.train_dir, "%s-[%s]-_total_y_diffs.npy" % (model.model_name, test_idx))


def maxinf(model, test_idx, num_to_remove=1, save=True):
    """(predicted_y_diffs[top], indices_to_remove (related positions), train rows), computed
    on the GPU by the fused top-K of fia_query_batch.  Like the reference's maxinf branch
    (experiments.py:36-48) the full predicted vector is saved first (save=True)."""
    res = model.get_influence_batch([test_idx], K=num_to_remove, full=True, return_x=False)
    if save:
        np.save(total_y_diffs_path(model, test_idx), res["influence"])
    pos = res["topk_pos"][0]
    keep = pos >= 0
    model.train_indices_of_test_case = res["rel_idx"]
    return res["topk_val"][0][keep], pos[keep], res["topk_idx"][0][keep]


def test_retraining(model, test_idx, iter_to_load, retrain_times, force_refresh=False, num_to_remove=50,
                    num_steps=1000, random_seed=17, remove_type="random", reset_adam=0, load_checkpoint=True,
                    verbose=True):
    """Leave-one-out retraining against predicted influence (experiments.py:17-150).

    Returns (actual_y_diffs, predicted_y_diffs, indices_to_remove) like the reference:
    indices are related positions (into model.train_indices_of_test_case); actual diffs
    are mean r-hat(test) over retrain_times retrains without the row, minus the original
    prediction, minus the mean drift of retraining with nothing removed (bias_retrain);
    |predicted| > 1 is clamped to 0 and NaN retrains are dropped (experiments.py:136-140)."""
    log = print if verbose else (lambda *a, **k: None)
    np.random.seed(random_seed)
    model.load_checkpoint(iter_to_load)
    train = model.data_sets["train"]
    if remove_type == "random":
        idx = np.random.choice(model.num_train_examples, size=num_to_remove, replace=False)
        infl = model.get_influence_on_test_loss([test_idx], idx, force_refresh=force_refresh)
        # the reference indexes the related list with train-row draws (experiments.py:33-37);
        # keep only draws that are valid related positions
        indices_to_remove = idx[idx < infl.size]
        predicted_y_diffs = infl[indices_to_remove]
    elif remove_type == "maxinf":
        predicted_y_diffs, indices_to_remove, _ = maxinf(model, test_idx, num_to_remove)
    else:
        raise ValueError("remove_type not well specified")
    num_to_remove = len(indices_to_remove)
    predicted_y_diffs = np.array(predicted_y_diffs, np.float64)
    actual_y_diffs = np.zeros([num_to_remove])
    rows = model.train_indices_of_test_case[indices_to_remove]
    log("Indices to remove are:", rows)

    test_y_val = model.predict_test(test_idx)
    train_loss_val = model.train_loss()
    log("Prediction for the test case is:", test_y_val)
    all_rows = model.fill_feed_dict_with_all_ex(train)
    retrained_test_y_val, retrained_train_loss_val = [], []
    if not load_checkpoint:
        retrained_test_y_val.append(model.predict_test(test_idx))
        retrained_train_loss_val.append(model.train_loss())
    else:
        for _ in range(retrain_times):
            if reset_adam:
                model.reset_optimizer()
            model.retrain(num_steps=num_steps, feed_dict=all_rows)
            retrained_test_y_val.append(model.predict_test(test_idx))
            retrained_train_loss_val.append(model.train_loss())
            model.load_checkpoint(iter_to_load, do_checks=False)
    bias_retrain = np.array(retrained_test_y_val).mean() - test_y_val if load_checkpoint else 0.0
    log("Difference in prediction after retraining     : %s" % bias_retrain)
    log("Difference in train loss after retraining     : %s" % (np.mean(retrained_train_loss_val) - train_loss_val))

    for counter, pos in enumerate(indices_to_remove):
        feed = model.fill_feed_dict_with_all_but_one_ex(train, rows[counter])
        ys = []
        for _ in range(retrain_times):
            if reset_adam:
                model.reset_optimizer()
            model.retrain(num_steps=num_steps, feed_dict=feed)
            ys.append(model.predict_test(test_idx))
            if load_checkpoint:
                model.load_checkpoint(iter_to_load, do_checks=False)
        ys = np.asarray(ys)
        ys = ys[~np.isnan(ys)]
        actual_y_diffs[counter] = ys.mean() - test_y_val - bias_retrain
        if np.abs(predicted_y_diffs[counter]) > 1:
            predicted_y_diffs[counter] = 0
        log("=== #%d === removed train row %d: actual %.6g predicted %.6g" % (
            counter, rows[counter], actual_y_diffs[counter], predicted_y_diffs[counter]))
    return actual_y_diffs, predicted_y_diffs, indices_to_remove
