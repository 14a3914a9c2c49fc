"""CPU fp64 closed-form oracle of the FIA per-test-rating influence path.

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker; the product path (the HIP library
behind fia-kdd-19_amd/influence) never imports or calls anything here.

Parity status: UNPINNED against reference outputs.  The reference path is
TensorFlow graph code (src/influence/matrix_factorization.py, NCF.py) and
TensorFlow is not installed here, and the reference ships no tests, golden
vectors or trained checkpoints.  This restatement is
cross-checked instead by (a) oracle/autograd_oracle.py, a torch double-backward
restatement of the TF graph semantics (dense flat tables, total_loss with the
L2 collection, slice-then-double-backward), and (b) oracle/ncg_port.py, the
reference's own solver (scipy fmin_ncg with the reference arguments).  What IS
pinned against the reference: the RQ1 query selection (known answer listed in
SURVEY.md 8d) and the related-set / DataSet float32 semantics.

Math (verified against (a) in tests):
  MF  r(a,b) = p_a.q_b + b_a + b_b + g                   matrix_factorization.py:89-116
      loss over a fed batch B = mean_B (r - y)^2 + wd/2 (|P|^2 + |Q|^2)   :122-132, gnn:40-65
      theta_t = [p_u, q_i, b_u, b_i]                     :38-67, :152-162
  NCF r = W3.[relu(W2^T relu(W1^T[Pm_a;Qm_b]+b1)+b2) ; Pg_a*Qg_b] + b3     NCF.py:102-145
      all four tables and W1..W3 decayed                  NCF.py:88-94,105-129
      theta_t = [Pm_u, Qm_i, Pg_u, Qg_i]                  NCF.py:43-66, 181-191
  rel  = where(x[:,0]==u) ++ where(x[:,1]==i)            matrix_factorization.py:315-322
  v    = d r(u,i) / d theta_t                            gnn:155, mf:194, 201
  H    = (2/n) sum_rel (g g^T + e d2r) + wd*M + damping*I   mf:288-308, 324-351
  x    = H^-1 v (exact fp64 solve; the reference approximates it with fmin_ncg, mf:419-433)
  infl_j = x . (2 e_j g_j + wd*M*theta_t) / n            mf:237-246
"""
import numpy as np


# ----------------------------------------------------------------------------
# related set (matrix_factorization.py:315-322, NCF.py:344-351)
# ----------------------------------------------------------------------------
def related_indices(train_x, u, i):
    """np.where over the float32 id columns, user rows then item rows."""
    x = np.asarray(train_x, dtype=np.float32)
    u_idx = np.where(x[:, 0] == np.float32(u))[0]
    i_idx = np.where(x[:, 1] == np.float32(i))[0]
    return np.concatenate((u_idx, i_idx)).astype(np.int64)


def topk(values, K):
    """Caller's top-K (experiments.py:46-48: argsort(|pred|)[-K:][::-1]) with
    the build's deterministic tie rule: |value| descending, rel position ascending."""
    v = np.asarray(values, np.float64)
    if v.size == 0 or K <= 0:
        return np.zeros(0, np.int64)
    order = np.lexsort((np.arange(v.size), -np.abs(v)))
    return order[:K].astype(np.int64)


# ----------------------------------------------------------------------------
# MF
# ----------------------------------------------------------------------------
def _mf_tables(params, k):
    P = np.asarray(params["embedding_layer/embedding_users"], np.float64).reshape(-1, k)
    Q = np.asarray(params["embedding_layer/embedding_items"], np.float64).reshape(-1, k)
    bu = np.asarray(params["embedding_layer/bias_users"], np.float64).reshape(-1)
    bi = np.asarray(params["embedding_layer/bias_items"], np.float64).reshape(-1)
    g = float(np.asarray(params["embedding_layer/global_bias"], np.float64).reshape(-1)[0])
    return P, Q, bu, bi, g


def mf_predict(params, k, users, items):
    P, Q, bu, bi, g = _mf_tables(params, k)
    users = np.asarray(users, np.int64)
    items = np.asarray(items, np.int64)
    return np.einsum("nk,nk->n", P[users], Q[items]) + bu[users] + bi[items] + g


def mf_query(params, k, train_users, train_items, train_ratings, u, i, wd, damping):
    """One MF FIA query. Returns dict(rel, n, v, H, x, influence) (fp64)."""
    tu = np.asarray(train_users)
    ti = np.asarray(train_items)
    rel = related_indices(np.stack([tu, ti], 1).astype(np.float32), u, i)
    return _mf_core(_mf_tables(params, k), k, tu, ti, train_ratings, u, i, wd, damping, rel)


def _mf_core(tables, k, tu, ti, train_ratings, u, i, wd, damping, rel):
    """mf_query's math for a given related list rel (mf:152-162, 237-246, 288-351)."""
    P, Q, bu, bi, g = tables
    n = rel.size
    D = 2 * k + 2
    theta = np.concatenate([P[u], Q[i], [bu[u]], [bi[i]]])
    v = np.concatenate([Q[i], P[u], [1.0], [1.0]])
    if n == 0:
        # TF's mean over an empty batch is NaN; the scored set is empty.
        return dict(rel=rel, n=0, v=v, H=np.full((D, D), np.nan), x=np.full(D, np.nan),
                    influence=np.zeros(0))
    uj = tu[rel].astype(np.int64)
    ij = ti[rel].astype(np.int64)
    yj = np.asarray(train_ratings, np.float64)[rel]
    e = np.einsum("nk,nk->n", P[uj], Q[ij]) + bu[uj] + bi[ij] + g - yj
    G = np.zeros((n, D))
    is_u = uj == u
    is_i = ij == i
    G[is_u, 0:k] = Q[ij[is_u]]
    G[is_u, 2 * k] = 1.0
    G[is_i, k:2 * k] = P[uj[is_i]]
    G[is_i, 2 * k + 1] = 1.0
    H = (2.0 / n) * (G.T @ G)
    both = is_u & is_i                      # the test pair itself is a train row
    if np.any(both):
        s = (2.0 / n) * e[both].sum()
        idx = np.arange(k)
        H[idx, k + idx] += s                # d2 r / dp_u dq_i = I
        H[k + idx, idx] += s
    M = np.concatenate([np.ones(2 * k), np.zeros(2)])
    H += np.diag(wd * M + damping)
    x = np.linalg.solve(H, v)
    grads = 2.0 * e[:, None] * G + (wd * M * theta)[None, :]
    infl = grads @ x / n
    return dict(rel=rel, n=n, v=v, H=H, x=x, influence=infl, theta=theta, G=G, e=e)


# ----------------------------------------------------------------------------
# NCF
# ----------------------------------------------------------------------------
def _ncf_tables(params, k):
    h = k // 2
    f = lambda name: np.asarray(params[name], np.float64)
    return dict(
        Pm=f("embedding_layer/mlp/embedding_users").reshape(-1, k),
        Qm=f("embedding_layer/mlp/embedding_items").reshape(-1, k),
        Pg=f("embedding_layer/gmf/embedding_users").reshape(-1, k),
        Qg=f("embedding_layer/gmf/embedding_items").reshape(-1, k),
        W1=f("h1/weights").reshape(2 * k, k), b1=f("h1/biases").reshape(k),
        W2=f("h2/weights").reshape(k, h), b2=f("h2/biases").reshape(h),
        W3=f("h3/weights").reshape(3 * h), b3=float(f("h3/biases").reshape(-1)[0]))


def ncf_forward_backward(T, k, users, items):
    """r-hat and d r-hat / d(Pm_a, Qm_b, Pg_a, Qg_b) for rows (a, b) (NCF.py:85-145).
    ReLU derivative is 1[z > 0] (TF ReluGrad)."""
    h = k // 2
    users = np.asarray(users, np.int64)
    items = np.asarray(items, np.int64)
    x0 = np.concatenate([T["Pm"][users], T["Qm"][items]], 1)
    z1 = x0 @ T["W1"] + T["b1"]
    h1 = np.maximum(z1, 0.0)
    z2 = h1 @ T["W2"] + T["b2"]
    h2 = np.maximum(z2, 0.0)
    gmf = T["Pg"][users] * T["Qg"][items]
    W3m, W3g = T["W3"][:h], T["W3"][h:]
    r = h2 @ W3m + gmf @ W3g + T["b3"]
    d2 = W3m[None, :] * (z2 > 0)
    d1 = (d2 @ T["W2"].T) * (z1 > 0)
    dx0 = d1 @ T["W1"].T
    return r, dx0[:, :k], dx0[:, k:], W3g[None, :] * T["Qg"][items], W3g[None, :] * T["Pg"][users]


def ncf_predict(params, k, users, items):
    return ncf_forward_backward(_ncf_tables(params, k), k, users, items)[0]


def ncf_query(params, k, train_users, train_items, train_ratings, u, i, wd, damping):
    """One NCF FIA query. Returns dict(rel, n, v, H, x, influence) (fp64)."""
    tu = np.asarray(train_users)
    ti = np.asarray(train_items)
    rel = related_indices(np.stack([tu, ti], 1).astype(np.float32), u, i)
    return _ncf_core(_ncf_tables(params, k), k, tu, ti, train_ratings, u, i, wd, damping, rel)


def _ncf_core(T, k, tu, ti, train_ratings, u, i, wd, damping, rel):
    """ncf_query's math for a given related list rel (ncf:181-191, 266-274, 317-380)."""
    h = k // 2
    n = rel.size
    D = 4 * k
    theta = np.concatenate([T["Pm"][u], T["Qm"][i], T["Pg"][u], T["Qg"][i]])
    _, vPm, vQm, vPg, vQg = ncf_forward_backward(T, k, [u], [i])
    v = np.concatenate([vPm[0], vQm[0], vPg[0], vQg[0]])
    if n == 0:
        return dict(rel=rel, n=0, v=v, H=np.full((D, D), np.nan), x=np.full(D, np.nan),
                    influence=np.zeros(0))
    uj = tu[rel].astype(np.int64)
    ij = ti[rel].astype(np.int64)
    yj = np.asarray(train_ratings, np.float64)[rel]
    r, dPm, dQm, dPg, dQg = ncf_forward_backward(T, k, uj, ij)
    e = r - yj
    is_u = (uj == u)[:, None]
    is_i = (ij == i)[:, None]
    G = np.concatenate([dPm * is_u, dQm * is_i, dPg * is_u, dQg * is_i], 1)
    H = (2.0 / n) * (G.T @ G)
    both = is_u[:, 0] & is_i[:, 0]
    if np.any(both):
        s = (2.0 / n) * e[both].sum()
        W3g = T["W3"][h:]
        idx = np.arange(k)
        H[2 * k + idx, 3 * k + idx] += s * W3g   # d2 r / dPg_u dQg_i = diag(W3g)
        H[3 * k + idx, 2 * k + idx] += s * W3g
    H += np.eye(D) * (wd + damping)
    x = np.linalg.solve(H, v)
    grads = 2.0 * e[:, None] * G + wd * theta[None, :]
    infl = grads @ x / n
    return dict(rel=rel, n=n, v=v, H=H, x=x, influence=infl, theta=theta, G=G, e=e)


def query(model, params, k, train_users, train_items, train_ratings, u, i, wd, damping):
    f = mf_query if model == "MF" else ncf_query
    return f(params, k, train_users, train_items, train_ratings, u, i, wd, damping)


def num_params(model, k):
    return 2 * k + 2 if model == "MF" else 4 * k


class CsrExact(object):
    """The closed form above with the related lists read from a CSR (by user) / CSC (by
    item) index of stably sorted train rows -- rel(u, i) is the same array as the O(N)
    np.where scans give (mf:315-322) -- and the parameter tables converted once.  This is
    the vectorized exact-solve CPU figure bench.py's cpu_baseline reports beside the
    reference algorithm; it is a checker-side restatement, never
    the product path."""

    def __init__(self, model, params, k, train_users, train_items, train_ratings, wd, damping):
        self.model, self.k, self.wd, self.damping = model, k, wd, damping
        self.tu = np.asarray(train_users)
        self.ti = np.asarray(train_items)
        self.tr = np.asarray(train_ratings)
        self.tables = _mf_tables(params, k) if model == "MF" else _ncf_tables(params, k)
        self.lists = []
        for ids in (self.tu, self.ti):
            order = np.argsort(ids, kind="stable").astype(np.int64)
            ptr = np.searchsorted(ids[order], np.arange(int(ids.max(initial=-1)) + 2), side="left")
            self.lists.append((order, ptr))

    def related(self, u, i):
        (uo, up), (io, ip) = self.lists
        ru = uo[up[u]:up[u + 1]] if u + 1 < up.size else uo[:0]
        ri = io[ip[i]:ip[i + 1]] if i + 1 < ip.size else io[:0]
        return np.concatenate([ru, ri])

    def query(self, u, i):
        core = _mf_core if self.model == "MF" else _ncf_core
        return core(self.tables, self.k, self.tu, self.ti, self.tr, u, i, self.wd, self.damping, self.related(u, i))
