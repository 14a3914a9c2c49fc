"""NCF model with the reference's FIA interface (src/influence/NCF.py).

    h1 = relu(W1^T [Pm_a; Qm_b] + b1)   W1: 2k x k              (NCF.py:138-139)
    h2 = relu(W2^T h1 + b2)             W2: k x k/2             (NCF.py:140-141)
    r-hat = W3^T [h2 ; Pg_a * Qg_b] + b3   W3: 3k/2 x 1          (NCF.py:142-144)
    all four tables and W1..W3 decayed                          (NCF.py:88-94, 105-129)
    theta_t = [Pm_u, Qm_i, Pg_u, Qg_i]                          (NCF.py:43-66, 181-191)
"""
import numpy as np

from influence import _lib
from influence.genericNeuralNet import GenericNeuralNet
from influence.synth import _truncated_normal, NCF_PARAM_NAMES


class NCF(GenericNeuralNet):
    MODEL_ID = _lib.FIA_MODEL_NCF
    PARAM_NAMES = tuple(NCF_PARAM_NAMES)

    def __init__(self, num_users, num_items, embedding_size, weight_decay, **kwargs):
        if embedding_size % 2:
            raise ValueError("NCF needs an even embedding size (h2 has embedding_size/2 units)")
        self.num_users = num_users
        self.num_items = num_items
        self.embedding_size = embedding_size
        self.weight_decay = weight_decay
        super(NCF, self).__init__(**kwargs)

    def param_shapes(self):
        U, I, k = self.num_users, self.num_items, self.embedding_size
        h = k // 2
        return dict(zip(self.PARAM_NAMES, [(U * k,), (I * k,), (U * k,), (I * k,), (2 * k * k,), (k,),
                                           (k * h,), (h,), (3 * h,), (1,)]))

    def init_params(self, seed=0):
        """Reference initialisers: truncated normal stddev 1/sqrt(fan_in) (NCF.py:88-94,
        fnn_layer :85-100), zero biases."""
        rng = np.random.default_rng(seed)
        U, I, k = self.num_users, self.num_items, self.embedding_size
        h = k // 2
        s = 1.0 / np.sqrt(k)
        n = self.PARAM_NAMES
        return {
            n[0]: _truncated_normal(rng, (U * k,), s), n[1]: _truncated_normal(rng, (I * k,), s),
            n[2]: _truncated_normal(rng, (U * k,), s), n[3]: _truncated_normal(rng, (I * k,), s),
            n[4]: _truncated_normal(rng, (2 * k * k,), 1.0 / np.sqrt(2 * k)), n[5]: np.zeros(k, np.float32),
            n[6]: _truncated_normal(rng, (k * h,), 1.0 / np.sqrt(k)), n[7]: np.zeros(h, np.float32),
            n[8]: _truncated_normal(rng, (3 * h,), 1.0 / np.sqrt(3 * h)), n[9]: np.zeros(1, np.float32),
        }

    def retrain(self, num_steps, feed_dict):
        """NCF.retrain (NCF.py:68-72): num_steps Adam steps on mini-batches of self.batch_size
        drawn by DataSet.next_batch from the feed's rows; unlike MF, the Adam state is NOT
        reset."""
        self._retrain_minibatch(num_steps, feed_dict)

    def _split_theta(self, x):
        k = self.embedding_size
        return [x[:k], x[k:2 * k], x[2 * k:3 * k], x[3 * k:4 * k]]

    def _theta_blocks(self, u, i):
        k = self.embedding_size
        n = self.PARAM_NAMES
        return [self.params[n[0]][u * k:(u + 1) * k].copy(), self.params[n[1]][i * k:(i + 1) * k].copy(),
                self.params[n[2]][u * k:(u + 1) * k].copy(), self.params[n[3]][i * k:(i + 1) * k].copy()]
