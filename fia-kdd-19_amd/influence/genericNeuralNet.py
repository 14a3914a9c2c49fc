"""Model base of the FIA path: the reference's constructor contract and the
FIA query methods, backed by the HIP library (libfia.so) instead of a
TensorFlow session.

Reference: src/influence/genericNeuralNet.py (GenericNeuralNet.__init__
:82-181) and the per-model FIA methods of matrix_factorization.py:38-67,
152-351 / NCF.py:43-66, 181-380.  Training (gnn:367-449), the classic
full-parameter influence variants (gnn:511-808) and TF checkpoints are not
part of this build.
"""
import os
import time

import numpy as np

from influence import _lib
from influence.dataset import DataSet


class GenericNeuralNet(object):
    MODEL_ID = None          # _lib.FIA_MODEL_MF / _lib.FIA_MODEL_NCF
    PARAM_NAMES = ()         # reference variable names, include/fia.h table order

    def __init__(self, **kwargs):
        np.random.seed(0)    # gnn:83 -- RQ1's query choice (RQ1.py:132) depends on it
        self.batch_size = kwargs.pop("batch_size")
        self.data_sets = kwargs.pop("data_sets")
        self.train_dir = kwargs.pop("train_dir", "output")
        self.log_dir = kwargs.pop("log_dir", "log")
        self.model_name = kwargs.pop("model_name")
        self.num_classes = kwargs.pop("num_classes")
        self.initial_learning_rate = kwargs.pop("initial_learning_rate")
        self.decay_epochs = kwargs.pop("decay_epochs")
        self.avextol = kwargs.pop("avextol")
        self.keep_probs = kwargs.pop("keep_probs", None)
        self.mini_batch = kwargs.pop("mini_batch", True)
        self.damping = kwargs.pop("damping", 0.0)
        self.device = kwargs.pop("device", 0)
        self.verbose = kwargs.pop("verbose", True)
        self.save_inverse_hvp = kwargs.pop("save_inverse_hvp", True)
        params = kwargs.pop("params", None)
        if not os.path.exists(self.train_dir):
            os.makedirs(self.train_dir)
        train = self.data_sets["train"]
        self.num_train_examples = train.labels.shape[0]
        self.num_test_examples = self.data_sets["test"].labels.shape[0]
        self.ctx = _lib.Context(self.device)
        self.params = self.init_params(seed=0) if params is None else self._checked(params)
        self._upload_params()
        self._build_index(train)
        self.ctx.prepare()

    # ------------------------------------------------------------------ params
    def param_shapes(self):
        raise NotImplementedError

    def init_params(self, seed=0):
        raise NotImplementedError

    def _checked(self, params):
        shapes = self.param_shapes()
        out = {}
        for name in self.PARAM_NAMES:
            if name not in params:
                raise ValueError("missing parameter %s" % name)
            a = np.ascontiguousarray(np.asarray(params[name], np.float32).reshape(-1))
            if a.shape != shapes[name]:
                raise ValueError("parameter %s has shape %s, expected %s" % (name, a.shape, shapes[name]))
            out[name] = a
        return out

    def _upload_params(self):
        import torch
        self._dev_params = [torch.from_numpy(self.params[n]).to(self.ctx.torch_device) for n in self.PARAM_NAMES]
        self.ctx.set_params(self.MODEL_ID, self.embedding_size, self.num_users, self.num_items, self._dev_params,
                            self.weight_decay, self.damping)

    def load_params(self, params):
        """Replace the parameter values (e.g. trained elsewhere) and rebuild the Hessian caches."""
        self.params = self._checked(params)
        self._upload_params()
        self.ctx.prepare()

    def prepare_for(self, test_indices):
        """Rebuild the Hessian caches for only the users/items of these test ratings
        (fia_prepare_for: one GPU's share of a sharded query set at large k).  Queries
        outside the set then raise FIAError until the next prepare."""
        qu, qi = self._query_tensors(test_indices)
        self.ctx.prepare_for(qu, qi)

    def get_all_params(self):
        """Parameter values in the reference's get_all_params order (mf:30-36)."""
        return [self.params[n] for n in self.PARAM_NAMES]

    def save_checkpoint(self, step):
        path = os.path.join(self.train_dir, "%s-checkpoint-%s.npz" % (self.model_name, step))
        np.savez(path, **{n.replace("/", "__"): v for n, v in self.params.items()})
        return path

    def load_checkpoint(self, iter_to_load, do_checks=True):
        """npz parameter checkpoints written by save_checkpoint (TF checkpoints are not read)."""
        path = os.path.join(self.train_dir, "%s-checkpoint-%s.npz" % (self.model_name, iter_to_load))
        with np.load(path, allow_pickle=False) as z:
            self.load_params({n.replace("__", "/"): z[n] for n in z.files})
        if self.verbose:
            print("Loading successful...")

    # ------------------------------------------------------------------- index
    def _build_index(self, train):
        import torch
        x = np.asarray(train.x)
        users = getattr(train, "users", None)
        items = getattr(train, "items", None)
        if users is None:
            users = x[:, 0].astype(np.int32)
            items = x[:, 1].astype(np.int32)
        dev = self.ctx.torch_device
        self._train_users = torch.from_numpy(np.ascontiguousarray(users, np.int32)).to(dev)
        self._train_items = torch.from_numpy(np.ascontiguousarray(items, np.int32)).to(dev)
        self._train_ratings = torch.from_numpy(np.ascontiguousarray(train.labels, np.float32)).to(dev)
        self.ctx.build_index(self._train_users, self._train_items, self._train_ratings, self.num_users,
                             self.num_items)

    # --------------------------------------------------------------- queries
    def _test_pair(self, test_index):
        test_u, test_i = self.data_sets["test"].x[test_index]
        return int(test_u), int(test_i)

    def _query_tensors(self, test_indices):
        import torch
        pairs = np.array([self._test_pair(t) for t in test_indices], np.int32).reshape(-1, 2)
        dev = self.ctx.torch_device
        qu = torch.from_numpy(np.ascontiguousarray(pairs[:, 0])).to(dev)
        qi = torch.from_numpy(np.ascontiguousarray(pairs[:, 1])).to(dev)
        return qu, qi

    def get_train_indices_of_test_case(self, test_indices):
        """rel = where(train.x[:,0]==u) ++ where(train.x[:,1]==i) (mf:315-322), from the GPU index."""
        import torch
        assert len(test_indices) == 1
        self.test_u, self.test_i = self._test_pair(test_indices[0])
        qu, qi = self._query_tensors(test_indices)
        offsets, total = self.ctx.count_related(qu, qi)
        rel = torch.empty(max(total, 1), dtype=torch.int64, device=self.ctx.torch_device)
        self.ctx.related(qu, qi, offsets, rel)
        return rel[:total].cpu().numpy()

    def get_test_params(self, test_index):
        """theta_t values in the reference block order (mf:38-67 / ncf:43-66)."""
        u, i = self._test_pair(test_index[0])
        return self._theta_blocks(u, i)

    def get_influence_batch(self, test_indices, K=1, full=True, return_x=True):
        """Batched FIA over many test ratings (one fia_query_batch call).

        Returns dict(offsets, rel_idx, influence, x, topk_pos, topk_idx, topk_val) as numpy
        arrays; influence[offsets[q]:offsets[q+1]] is get_influence_on_test_loss([t_q], ...)."""
        import torch
        qu, qi = self._query_tensors(test_indices)
        Q = qu.numel()
        dev = self.ctx.torch_device
        offsets, total = self.ctx.count_related(qu, qi)
        D = self.ctx.num_params()
        rel = torch.empty(max(total, 1), dtype=torch.int64, device=dev) if full else None
        infl = torch.empty(max(total, 1), dtype=torch.float64, device=dev) if full else None
        x = torch.empty(max(Q * D, 1), dtype=torch.float64, device=dev) if return_x else None
        tp = torch.empty(max(Q * K, 1), dtype=torch.int64, device=dev) if K else None
        ti = torch.empty(max(Q * K, 1), dtype=torch.int64, device=dev) if K else None
        tv = torch.empty(max(Q * K, 1), dtype=torch.float64, device=dev) if K else None
        self.ctx.query_batch(qu, qi, offsets, total, rel, infl, x, K, tp, ti, tv)
        out = dict(offsets=offsets.cpu().numpy())
        if full:
            out["rel_idx"] = rel[:total].cpu().numpy()
            out["influence"] = infl[:total].cpu().numpy()
        if return_x:
            out["x"] = x[:Q * D].cpu().numpy().reshape(Q, D)
        if K:
            out["topk_pos"] = tp[:Q * K].cpu().numpy().reshape(Q, K)
            out["topk_idx"] = ti[:Q * K].cpu().numpy().reshape(Q, K)
            out["topk_val"] = tv[:Q * K].cpu().numpy().reshape(Q, K)
        return out

    def get_influence_on_test_loss(self, test_indices, train_idx, approx_type="cg", approx_params=None,
                                   force_refresh=True, test_description=None, loss_type="normal_loss",
                                   X=None, Y=None):
        """Predicted change of r-hat(test pair) when each related training rating is
        removed (mf:164-251, ncf:193-280).  Returns float64[n] aligned with
        self.train_indices_of_test_case.

        Differences from the reference, by design: the inverse HVP is the exact fp64
        solve (the reference's fmin_ncg approximates it, mf:424-431); errors raise
        ValueError (the reference raises tuples, mf:173-177); the phantom-point branch
        (train_idx None, mf:228-235) is shape-inconsistent in the reference and raises
        NotImplementedError here."""
        if train_idx is None:
            if X is None or Y is None:
                raise ValueError("X and Y must be specified if using phantom points.")
            if X.shape[0] != len(Y):
                raise ValueError("X and Y must have the same length.")
            raise NotImplementedError("phantom points (train_idx=None) are not supported")
        if X is not None or Y is not None:
            raise ValueError("X and Y cannot be specified if train_idx is specified.")
        if approx_type not in ("cg", "lissa"):
            raise ValueError("approx_type must be 'cg' or 'lissa'")
        if loss_type != "normal_loss":
            raise ValueError("Loss must be normal")
        assert len(test_indices) == 1
        t0 = time.time()
        self.test_index = test_indices[0]
        self.test_u, self.test_i = self._test_pair(self.test_index)
        res = self.get_influence_batch(test_indices, K=0, full=True, return_x=True)
        self.train_indices_of_test_case = res["rel_idx"]
        x = res["x"][0]
        self.num_params = x.size
        self.inverse_hvp = self._split_theta(x)
        if test_description is None:
            test_description = test_indices
        if self.save_inverse_hvp:
            fname = os.path.join(self.train_dir, "%s-%s-%s-test-%s.npz" % (
                self.model_name, approx_type, loss_type, test_description))
            np.savez(fname, inverse_hvp=x)
        dt = time.time() - t0
        if self.verbose:
            print("FIA test %s (u=%d, i=%d): %d related ratings, total time %.6f sec" % (
                self.test_index, self.test_u, self.test_i, res["influence"].size, dt))
        return res["influence"]

    def _split_theta(self, x):
        raise NotImplementedError

    def _theta_blocks(self, u, i):
        raise NotImplementedError
