"""Trainer for the MF / NCF models on PyTorch-ROCm.

The reference trains with TensorFlow 1.x (genericNeuralNet.py:367-449): Adam at
lr 1e-3 on mini-batches from DataSet.next_batch (dataset.py:49-70), loss =
mean squared error + the 'losses' collection of wd * l2_loss(var) over the
variable_with_weight_decay tables (genericNeuralNet.py:40-65,
matrix_factorization.py:89-132, NCF.py:85-161).  Leave-one-out retraining
(experiments.py:55-150) runs full-batch steps on all training rows but one
(genericNeuralNet.py:218-227, 344-347).

This module restates that training, not the TF graph:
  * parameters are fp32 device tensors under the reference variable names;
  * ``TFAdam`` is tf.train.AdamOptimizer's dense update (beta1 .9, beta2 .999,
    eps 1e-8, lr_t = lr * sqrt(1 - beta2^t) / (1 - beta1^t), epsilon outside
    the bias correction); the beta powers live on the device so a whole step
    can be captured;
  * a full-batch retrain step (static shapes) is captured once in a HIP graph
    (torch.cuda.CUDAGraph on ROCm) and replayed, so the 27,000-step retrains of
    RQ1 cost one graph launch per step.
Training is not the FIA hot path: it runs wherever torch runs (CPU in the CPU
tests, cuda:N on the box); the influence itself always goes through libfia.
"""
import numpy as np


# variables in the reference 'losses' collection (variable_with_weight_decay)
DECAYED = {
    "MF": ("embedding_layer/embedding_users", "embedding_layer/embedding_items"),
    "NCF": ("embedding_layer/mlp/embedding_users", "embedding_layer/mlp/embedding_items",
            "embedding_layer/gmf/embedding_users", "embedding_layer/gmf/embedding_items",
            "h1/weights", "h2/weights", "h3/weights"),
}


def predict(model, k, P, users, items):
    """r-hat for index tensors users/items (mf:110-116, ncf:130-145)."""
    import torch
    if model == "MF":
        pu = P["embedding_layer/embedding_users"].view(-1, k)[users]
        qi = P["embedding_layer/embedding_items"].view(-1, k)[items]
        return ((pu * qi).sum(1) + P["embedding_layer/bias_users"][users] + P["embedding_layer/bias_items"][items]
                + P["embedding_layer/global_bias"][0])
    h = k // 2
    pm = P["embedding_layer/mlp/embedding_users"].view(-1, k)[users]
    qm = P["embedding_layer/mlp/embedding_items"].view(-1, k)[items]
    pg = P["embedding_layer/gmf/embedding_users"].view(-1, k)[users]
    qg = P["embedding_layer/gmf/embedding_items"].view(-1, k)[items]
    h1 = torch.relu(torch.cat([pm, qm], 1) @ P["h1/weights"].view(2 * k, k) + P["h1/biases"])
    h2 = torch.relu(h1 @ P["h2/weights"].view(k, h) + P["h2/biases"])
    return (torch.cat([h2, pg * qg], 1) @ P["h3/weights"].view(3 * h, 1)).squeeze(1) + P["h3/biases"][0]


def total_loss(model, k, wd, P, users, items, labels):
    """mean (r-hat - y)^2 + wd * sum 0.5 ||var||^2 over the decayed variables (mf:122-132)."""
    err = predict(model, k, P, users, items) - labels
    reg = sum((P[n] * P[n]).sum() for n in DECAYED[model]) * (0.5 * wd)
    return (err * err).mean() + reg


class TFAdam(object):
    """tf.train.AdamOptimizer, dense update (gnn:432-440); state on the device."""

    def __init__(self, params, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8):
        import torch
        self.params = params
        self.lr, self.b1, self.b2, self.eps = lr, beta1, beta2, eps
        dev = params[0].device
        self.m = [torch.zeros_like(p) for p in params]
        self.v = [torch.zeros_like(p) for p in params]
        # beta1_power / beta2_power variables (start at beta, multiplied after each update)
        self.b1p = torch.full((), beta1, dtype=torch.float32, device=dev)
        self.b2p = torch.full((), beta2, dtype=torch.float32, device=dev)

    def step(self, grads):
        import torch
        lr_t = self.lr * torch.sqrt(1.0 - self.b2p) / (1.0 - self.b1p)
        torch._foreach_mul_(self.m, self.b1)
        torch._foreach_add_(self.m, grads, alpha=1.0 - self.b1)
        torch._foreach_mul_(self.v, self.b2)
        torch._foreach_addcmul_(self.v, grads, grads, value=1.0 - self.b2)
        den = torch._foreach_sqrt(self.v)
        torch._foreach_add_(den, self.eps)
        upd = torch._foreach_div(self.m, den)
        torch._foreach_mul_(upd, lr_t)
        torch._foreach_sub_(self.params, upd)
        self.b1p.mul_(self.b1)
        self.b2p.mul_(self.b2)

    def state(self):
        return {"m": [t.detach().cpu().numpy() for t in self.m], "v": [t.detach().cpu().numpy() for t in self.v],
                "b1p": float(self.b1p), "b2p": float(self.b2p)}

    def load_state(self, st):
        import torch
        with torch.no_grad():
            for t, a in zip(self.m, st["m"]):
                t.copy_(torch.from_numpy(np.asarray(a, np.float32)))
            for t, a in zip(self.v, st["v"]):
                t.copy_(torch.from_numpy(np.asarray(a, np.float32)))
            self.b1p.fill_(float(st["b1p"]))
            self.b2p.fill_(float(st["b2p"]))

    def reset(self):
        """reset_optimizer_op (gnn:437-438): zero the Adam slots and powers."""
        import torch
        with torch.no_grad():
            for t in self.m + self.v:
                t.zero_()
            self.b1p.fill_(self.b1)
            self.b2p.fill_(self.b2)


class Trainer(object):
    """Parameters + TF-Adam state of one MF / NCF model on one device."""

    def __init__(self, model, k, wd, lr, params, names, device):
        import torch
        self.model, self.k, self.wd, self.lr = model, k, float(wd), float(lr)
        self.names = list(names)
        self.device = torch.device(device)
        self.P = {n: torch.tensor(np.asarray(params[n], np.float32), device=self.device).requires_grad_(True)
                  for n in self.names}
        self.plist = [self.P[n] for n in self.names]
        self.opt = TFAdam(self.plist, lr=self.lr)
        self._graph = None
        self._graph_key = None

    # ---- state ----
    def params_numpy(self):
        return {n: self.P[n].detach().cpu().numpy().copy() for n in self.names}

    def set_params(self, params):
        import torch
        with torch.no_grad():
            for n in self.names:
                self.P[n].copy_(torch.from_numpy(np.asarray(params[n], np.float32).reshape(-1)))

    # ---- steps ----
    def _tensors(self, users, items, labels):
        import torch
        return (torch.as_tensor(np.ascontiguousarray(users, np.int64), device=self.device),
                torch.as_tensor(np.ascontiguousarray(items, np.int64), device=self.device),
                torch.as_tensor(np.ascontiguousarray(labels, np.float32), device=self.device))

    def _step(self, u, i, y):
        import torch
        loss = total_loss(self.model, self.k, self.wd, self.P, u, i, y)
        grads = torch.autograd.grad(loss, self.plist)
        with torch.no_grad():
            self.opt.step(list(grads))
        return loss

    def step(self, users, items, labels):
        """One Adam step on a mini-batch (train_op, gnn:388-390); returns the loss as a
        device scalar (no host sync)."""
        u, i, y = self._tensors(users, items, labels)
        return self._step(u, i, y).detach()

    def loss(self, users, items, labels):
        import torch
        u, i, y = self._tensors(users, items, labels)
        with torch.no_grad():
            return float(total_loss(self.model, self.k, self.wd, self.P, u, i, y))

    def predict(self, users, items):
        import torch
        u, i, _ = self._tensors(users, items, np.zeros(len(users)))
        with torch.no_grad():
            return predict(self.model, self.k, self.P, u, i).double().cpu().numpy()

    def full_batch(self, users, items, labels, num_steps):
        """num_steps full-batch Adam steps on fixed rows (retrain, gnn:344-347).  On a GPU
        the step is captured once in a HIP graph and replayed."""
        import torch
        u, i, y = self._tensors(users, items, labels)
        if num_steps <= 0:
            return
        if self.device.type != "cuda":
            for _ in range(num_steps):
                self._step(u, i, y)
            return
        key = (u.numel(),)
        if self._graph is None or self._graph_key != key:
            self._gu, self._gi, self._gy = u.clone(), i.clone(), y.clone()
            side = torch.cuda.Stream(device=self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))
            saved = self.params_numpy(), self.opt.state()
            with torch.cuda.stream(side):
                for _ in range(2):        # warm-up on a side stream (allocator, autograd)
                    self._step(self._gu, self._gi, self._gy)
            torch.cuda.current_stream(self.device).wait_stream(side)
            self.set_params(saved[0])
            self.opt.load_state(saved[1])
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._step(self._gu, self._gi, self._gy)
            self._graph, self._graph_key = g, key
            # capture ran no step (graph capture records only); state is the saved one
        else:
            self._gu.copy_(u)
            self._gi.copy_(i)
            self._gy.copy_(y)
        for _ in range(num_steps):
            self._graph.replay()
        torch.cuda.synchronize(self.device)
