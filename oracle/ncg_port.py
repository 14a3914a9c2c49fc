"""CPU port of the reference FIA *algorithm* (Newton-CG solve + per-rating loop).

TEST INFRASTRUCTURE ONLY (see oracle/fia_oracle.py header).  Used for two
things: (1) quantify how far the reference's approximate solve lands from the
exact fp64 solve (the documented CG-vs-exact gap), and (2)
bench.py's cpu_baseline leg ("kind": "port"): the reference algorithm timed on
the GPU box's host cores.

It follows MF.get_influence_on_test_loss (matrix_factorization.py:164-251)
step by step, with TensorFlow's sess.run replaced by numpy on the same rows:
  * related set: two O(N) np.where scans over float32 x (mf:315-322);
  * v = d r(u,i)/d theta_t (mf:201, gnn:155);
  * every HVP re-gathers the related rows (the feed of mf:295) and evaluates
    the restricted Hessian-vector product in the HVP dtype (fp32 like TF by
    default), then adds damping * v (mf:306);
  * scipy.optimize.fmin_ncg(f, x0=v, fprime, fhess_p, callback,
    avextol=avextol, maxiter=100) (mf:424-431) with the reference closures
    (mf:372-392) and the verbose callback of gnn:503-508 -> mf:401-415
    (one train-row-5 gradient + two extra HVPs per iteration);
  * scoring: one single-row gradient evaluation per related rating, then
    dot(inverse_hvp, grad) / n (mf:240-246).
The reference's dense (U+I)*k gradient materialisation per sess.run and the
per-query graph growth are NOT reproduced (they are TF artefacts), so this
port is faster than the reference it stands for.
"""
import time
import numpy as np
from scipy.optimize import fmin_ncg

from oracle import fia_oracle as fo


class RefAlgorithm(object):
    def __init__(self, model, params, k, train_users, train_items, train_ratings, wd, damping,
                 avextol=1e-3, hvp_dtype=np.float32, verbose_callback=True):
        self.model = model
        self.k = k
        self.wd = wd
        self.damping = damping
        self.avextol = avextol
        self.dt = hvp_dtype
        self.verbose_callback = verbose_callback
        self.x = np.stack([train_users, train_items], 1).astype(np.float32)   # DataSet x (dataset.py:14)
        self.users = np.asarray(train_users)
        self.items = np.asarray(train_items)
        self.labels = np.asarray(train_ratings, np.float64)
        if model == "MF":
            self.P, self.Q, self.bu, self.bi, self.g = [np.asarray(a, hvp_dtype) if np.ndim(a) else a
                                                        for a in fo._mf_tables(params, k)]
        else:
            T = fo._ncf_tables(params, k)
            self.T = {kk: (np.asarray(vv, hvp_dtype) if np.ndim(vv) else vv) for kk, vv in T.items()}

    # -- rows -> (residual e, restricted gradient rows G, second-derivative weight) --
    def _rows(self, idx, u, i):
        k = self.k
        uj = self.users[idx].astype(np.int64)
        ij = self.items[idx].astype(np.int64)
        y = self.labels[idx].astype(self.dt)
        is_u = (uj == u)
        is_i = (ij == i)
        if self.model == "MF":
            e = (np.einsum("nk,nk->n", self.P[uj], self.Q[ij]) + self.bu[uj] + self.bi[ij] + self.g - y)
            G = np.zeros((idx.size, 2 * k + 2), self.dt)
            G[is_u, :k] = self.Q[ij[is_u]]
            G[is_u, 2 * k] = 1
            G[is_i, k:2 * k] = self.P[uj[is_i]]
            G[is_i, 2 * k + 1] = 1
        else:
            r, dPm, dQm, dPg, dQg = fo.ncf_forward_backward(self.T, k, uj, ij)
            e = (r - y).astype(self.dt)
            G = np.concatenate([dPm * is_u[:, None], dQm * is_i[:, None], dPg * is_u[:, None],
                                dQg * is_i[:, None]], 1).astype(self.dt)
        return e, G, is_u & is_i

    def _theta_mask(self, u, i):
        k = self.k
        if self.model == "MF":
            th = np.concatenate([self.P[u], self.Q[i], [self.bu[u]], [self.bi[i]]]).astype(self.dt)
            M = np.concatenate([np.ones(2 * k), np.zeros(2)]).astype(self.dt)
        else:
            T = self.T
            th = np.concatenate([T["Pm"][u], T["Qm"][i], T["Pg"][u], T["Qg"][i]]).astype(self.dt)
            M = np.ones(4 * k, self.dt)
        return th, M

    def _second(self, vec):
        """d2 r / d theta^2 . vec for the (u, i) row itself (zero elsewhere)."""
        k = self.k
        out = np.zeros_like(vec)
        if self.model == "MF":
            out[:k] = vec[k:2 * k]
            out[k:2 * k] = vec[:k]
        else:
            W3g = self.T["W3"][k // 2:]
            out[2 * k:3 * k] = W3g * vec[3 * k:4 * k]
            out[3 * k:4 * k] = W3g * vec[2 * k:3 * k]
        return out

    # -- reference steps --
    def get_train_indices_of_test_case(self, u, i):
        u_idx = np.where(self.x[:, 0] == u)[0]
        i_idx = np.where(self.x[:, 1] == i)[0]
        return np.concatenate((u_idx, i_idx))

    def hvp(self, rel, u, i, vec):
        """minibatch_hessian_vector_val (mf:288-308): rows re-fed every call."""
        vec32 = np.asarray(vec, self.dt)
        e, G, both = self._rows(rel, u, i)
        n = rel.size
        _, M = self._theta_mask(u, i)
        hv = (2.0 / n) * (G.T @ (G @ vec32))
        if np.any(both):
            hv = hv + (2.0 / n) * e[both].sum() * self._second(vec32)
        hv = hv + self.wd * M * vec32
        return hv.astype(np.float64) + self.damping * np.asarray(vec, np.float64)

    def train_grad(self, idx, u, i):
        e, G, _ = self._rows(np.array([idx]), u, i)
        th, M = self._theta_mask(u, i)
        return (2.0 * e[0] * G[0] + self.wd * M * th).astype(np.float64)

    def test_grad(self, u, i):
        _, G, _ = self._rows_test(u, i)
        return G

    def _rows_test(self, u, i):
        k = self.k
        if self.model == "MF":
            v = np.concatenate([self.Q[i], self.P[u], [1], [1]]).astype(np.float64)
        else:
            _, a, b, c, d = fo.ncf_forward_backward(self.T, k, [u], [i])
            v = np.concatenate([a[0], b[0], c[0], d[0]]).astype(np.float64)
        return None, v, None

    def get_influence_on_test_loss(self, u, i):
        t0 = time.time()
        rel = self.get_train_indices_of_test_case(u, i)
        n = rel.size
        v = self._rows_test(u, i)[1]
        if n == 0:
            return rel, np.zeros(0), np.full(v.size, np.nan), dict(hvp_calls=0)
        calls = [0]

        def H(vec):
            calls[0] += 1
            return self.hvp(rel, u, i, vec)

        f = lambda x: 0.5 * np.dot(H(x), x) - np.dot(v, x)               # mf:374-377
        fprime = lambda x: H(x) - v                                       # mf:382-385
        fhess_p = lambda x, p: H(p)                                       # mf:389-392

        def callback(x):                                                  # mf:401-415
            g5 = self.train_grad(min(5, self.x.shape[0] - 1), u, i)
            _ = np.dot(x, g5) / n
            if self.verbose_callback:
                _ = f(x)
                _ = (0.5 * np.dot(H(x), x), -np.dot(v, x))

        # ill-conditioned systems (an entity with no train ratings leaves only the damping
        # on its bias) can overflow the fp32 HVPs, as they would in TF
        with np.errstate(over="ignore", invalid="ignore"):
            x = fmin_ncg(f=f, x0=v.copy(), fprime=fprime, fhess_p=fhess_p, callback=callback,
                         avextol=self.avextol, maxiter=100, disp=False)
        t1 = time.time()
        infl = np.zeros(n)
        for c, j in enumerate(rel):                                       # mf:240-246
            infl[c] = np.dot(x, self.train_grad(j, u, i)) / n
        t2 = time.time()
        return rel, infl, x, dict(hvp_calls=calls[0], t_solve=t1 - t0, t_score=t2 - t1)
