"""MF model with the reference's FIA interface (src/influence/matrix_factorization.py).

    r-hat(a, b) = p_a . q_b + b_a + b_b + g                   (mf:89-116)
    loss = mean squared error + wd/2 (|P|^2 + |Q|^2)           (mf:122-132, gnn:40-65)
    theta_t = [p_u (k), q_i (k), b_u, b_i]                     (mf:38-67, 152-162)
"""
import numpy as np

from influence import _lib
from influence.genericNeuralNet import GenericNeuralNet
from influence.synth import _truncated_normal, MF_PARAM_NAMES


class MF(GenericNeuralNet):
    MODEL_ID = _lib.FIA_MODEL_MF
    PARAM_NAMES = tuple(MF_PARAM_NAMES)

    def __init__(self, num_users, num_items, embedding_size, weight_decay, **kwargs):
        self.num_users = num_users
        self.num_items = num_items
        self.embedding_size = embedding_size
        self.weight_decay = weight_decay
        super(MF, self).__init__(**kwargs)

    def param_shapes(self):
        U, I, k = self.num_users, self.num_items, self.embedding_size
        return dict(zip(self.PARAM_NAMES, [(U * k,), (I * k,), (U,), (I,), (1,)]))

    def init_params(self, seed=0):
        """Reference initialisers: truncated normal stddev 1/sqrt(k) for the tables
        (mf:92-97), zeros for the biases (mf:103-109)."""
        rng = np.random.default_rng(seed)
        U, I, k = self.num_users, self.num_items, self.embedding_size
        s = 1.0 / np.sqrt(k)
        return {
            self.PARAM_NAMES[0]: _truncated_normal(rng, (U * k,), s),
            self.PARAM_NAMES[1]: _truncated_normal(rng, (I * k,), s),
            self.PARAM_NAMES[2]: np.zeros(U, np.float32),
            self.PARAM_NAMES[3]: np.zeros(I, np.float32),
            self.PARAM_NAMES[4]: np.zeros(1, np.float32),
        }

    def retrain(self, num_steps, feed_dict):
        """MF.retrain (mf:69-76): reset_optimizer_op, then num_steps Adam steps on mini-batches
        of self.batch_size drawn by DataSet.next_batch from the feed's rows (a fresh DataSet,
        so the batches start at row 0 and shuffle at the epoch wrap, dataset.py:49-70)."""
        self.reset_optimizer()
        self._retrain_minibatch(num_steps, feed_dict)

    def _split_theta(self, x):
        k = self.embedding_size
        return [x[:k], x[k:2 * k], x[2 * k:2 * k + 1], x[2 * k + 1:2 * k + 2]]

    def _theta_blocks(self, u, i):
        k = self.embedding_size
        P = self.params[self.PARAM_NAMES[0]]
        Q = self.params[self.PARAM_NAMES[1]]
        return [P[u * k:(u + 1) * k].copy(), Q[i * k:(i + 1) * k].copy(),
                self.params[self.PARAM_NAMES[2]][u:u + 1].copy(), self.params[self.PARAM_NAMES[3]][i:i + 1].copy()]

    def predict(self, users, items):
        k = self.embedding_size
        P = self.params[self.PARAM_NAMES[0]].reshape(-1, k).astype(np.float64)
        Q = self.params[self.PARAM_NAMES[1]].reshape(-1, k).astype(np.float64)
        users = np.asarray(users, np.int64)
        items = np.asarray(items, np.int64)
        return (np.einsum("nk,nk->n", P[users], Q[items]) + self.params[self.PARAM_NAMES[2]][users]
                + self.params[self.PARAM_NAMES[3]][items] + self.params[self.PARAM_NAMES[4]][0])
