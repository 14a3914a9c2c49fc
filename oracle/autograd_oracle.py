"""Torch-CPU double-backward restatement of the reference TF graph (fp64).

TEST INFRASTRUCTURE ONLY (see oracle/fia_oracle.py header; parity unpinned
against reference outputs).  This file checks the closed form in
fia_oracle.py by following the reference graph literally instead of using
any closed form:

  * every table is ONE flat variable reshaped at lookup time
    (matrix_factorization.py:92-101, NCF.py:105-136);
  * total_loss = mean squared error over the fed batch + wd * l2_loss of each
    decayed variable (genericNeuralNet.py:40-65, mf:122-132);
  * first backprop over ALL params, slice to theta_t by flat ranges
    (get_test_grad, mf:152-162 / NCF.py:181-191), elementwise product with a
    stopped v, second backprop over all params, slice again
    (hessian_vector_product_test, mf:324-351), + damping * v (mf:306);
  * v = sliced gradient of the squeezed prediction of the test row (gnn:155);
  * per-rating train gradient = sliced gradient of total_loss on a batch of one
    (mf:240-246).

H is materialised column by column from HVPs with unit vectors; x = H^-1 v is
the exact fp64 solve.  Small problems only.
"""
import numpy as np
import torch


def _mf_graph(params, k, U, I):
    P = torch.tensor(np.asarray(params["embedding_layer/embedding_users"], np.float64), requires_grad=True)
    Q = torch.tensor(np.asarray(params["embedding_layer/embedding_items"], np.float64), requires_grad=True)
    bu = torch.tensor(np.asarray(params["embedding_layer/bias_users"], np.float64), requires_grad=True)
    bi = torch.tensor(np.asarray(params["embedding_layer/bias_items"], np.float64), requires_grad=True)
    g = torch.tensor(np.asarray(params["embedding_layer/global_bias"], np.float64), requires_grad=True)
    plist = [P, Q, bu, bi, g]

    def logits(users, items):
        ue = P.reshape(U, k)[users]
        ie = Q.reshape(I, k)[items]
        return (ue * ie).sum(1) + bu.reshape(U, 1)[users][:, 0] + bi.reshape(I, 1)[items][:, 0] + g

    decayed = [P, Q]
    return plist, logits, decayed


def _ncf_graph(params, k, U, I):
    h = k // 2
    t = lambda n: torch.tensor(np.asarray(params[n], np.float64), requires_grad=True)
    Pm, Qm = t("embedding_layer/mlp/embedding_users"), t("embedding_layer/mlp/embedding_items")
    Pg, Qg = t("embedding_layer/gmf/embedding_users"), t("embedding_layer/gmf/embedding_items")
    W1, b1, W2, b2, W3, b3 = t("h1/weights"), t("h1/biases"), t("h2/weights"), t("h2/biases"), \
        t("h3/weights"), t("h3/biases")
    plist = [Pm, Qm, Pg, Qg, W1, b1, W2, b2, W3, b3]

    def logits(users, items):
        x0 = torch.cat([Pm.reshape(U, k)[users], Qm.reshape(I, k)[items]], 1)
        h1 = torch.relu(x0 @ W1.reshape(2 * k, k) + b1)
        h2 = torch.relu(h1 @ W2.reshape(k, h) + b2)
        gmf = Pg.reshape(U, k)[users] * Qg.reshape(I, k)[items]
        return (torch.cat([h2, gmf], 1) @ W3.reshape(3 * h, 1) + b3)[:, 0]

    decayed = [Pm, Qm, Pg, Qg, W1, W2, W3]
    return plist, logits, decayed


def _slices(model, k, u, i):
    """(param index, flat start, length) per theta_t block, in reference order."""
    if model == "MF":
        return [(0, u * k, k), (1, i * k, k), (2, u, 1), (3, i, 1)]
    return [(0, u * k, k), (1, i * k, k), (2, u * k, k), (3, i * k, k)]


def query(model, params, k, U, I, train_users, train_items, train_ratings, u, i, wd, damping):
    build = _mf_graph if model == "MF" else _ncf_graph
    plist, logits, decayed = build(params, k, U, I)
    sl = _slices(model, k, u, i)
    D = sum(s[2] for s in sl)

    tx = np.stack([np.asarray(train_users), np.asarray(train_items)], 1).astype(np.float32)
    rel = np.concatenate((np.where(tx[:, 0] == u)[0], np.where(tx[:, 1] == i)[0]))
    n = rel.size
    users = torch.tensor(np.asarray(train_users)[rel], dtype=torch.long)
    items = torch.tensor(np.asarray(train_items)[rel], dtype=torch.long)
    y = torch.tensor(np.asarray(train_ratings, np.float64)[rel])

    def total_loss(us, its, ys):
        mse = ((logits(us, its) - ys) ** 2).mean()
        l2 = sum(0.5 * (p ** 2).sum() for p in decayed) * wd
        return mse + l2

    def sliced(grads):
        return torch.cat([grads[pi].reshape(-1)[s:s + L] for pi, s, L in sl])

    r_test = logits(torch.tensor([u]), torch.tensor([i])).squeeze()
    v = sliced(torch.autograd.grad(r_test, plist, allow_unused=False)).detach().numpy()
    if n == 0:
        return dict(rel=rel, v=v, H=None, x=None, influence=np.zeros(0))

    loss = total_loss(users, items, y)
    g1 = torch.autograd.grad(loss, plist, create_graph=True)
    g1s = sliced(g1)
    H = np.zeros((D, D))
    for c in range(D):
        e = torch.zeros(D, dtype=torch.float64)
        e[c] = 1.0
        hv = torch.autograd.grad((g1s * e).sum(), plist, retain_graph=True, allow_unused=True)
        hv = [torch.zeros_like(p) if h is None else h for p, h in zip(plist, hv)]
        H[:, c] = sliced(hv).detach().numpy()
    H += damping * np.eye(D)
    x = np.linalg.solve(H, v)

    infl = np.zeros(n)
    for j in range(n):
        lj = total_loss(users[j:j + 1], items[j:j + 1], y[j:j + 1])
        gj = sliced(torch.autograd.grad(lj, plist, allow_unused=True)).detach().numpy()
        infl[j] = x @ gj / n
    return dict(rel=rel, v=v, H=H, x=x, influence=infl)
