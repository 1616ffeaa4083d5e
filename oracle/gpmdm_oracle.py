"""CPU oracle: a numpy fp64 restatement of the reference GPMDM particle-filter step.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the checker
(or as the timed CPU baseline).  The product path (``gpmdm_amd``) never imports it:
every product computation runs in the HIP library and fails loudly without it.

It restates, formula for formula, what the reference computes on the hot path:

* ``/root/reference/gpmdm/gpmdm_pf.py``   -- the particle filter (``GPMDM_PF``)
* ``/root/reference/gpmdm/gpmdm.py``      -- the GP predictive maps it calls

including the reference's quirks: the double-counted log-variance,
the float32-rounded ``ln 2*pi`` constant, the non-recursive weights, post-resample
classes paired with pre-resample weights in the read-outs, and ``ll + log_w`` in the
posterior.  torch's CPU sampling primitives are restated from their algorithms
(``multinomial(p, 1) = argmax(p / Exp(1))``; ``multinomial(w, P, True)`` = inverse CDF
by binary search over ``cumsum(w)/sum``), so the random draws enter as explicit
arrays.  Parity is pinned against golden vectors produced by the unmodified reference
(``tests/golden/make_golden.py``), see ``tests/test_oracle_golden.py``.

The dynamics inverse is restricted to each class block.  The reference inverts the
full masked ``Nx x Nx`` matrix (`gpmdm.py:1299-1305`); that matrix is block diagonal
(other-class blocks are ``1e-6 I``) and the masked kernel rows are exactly zero
(`gpmdm.py:1061`), so the restriction is exact up to rounding.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

# gpmdm_pf.py:5 -- torch.log(torch.tensor(2*pi)) is a float32 tensor whose value is
# 1.8378770351409912 (torch's float32 log; numpy's float32 log rounds to 1.8378771543...).
LOG_2PI_F32 = np.float32(1.8378770351409912)


def loglik_const(D: int) -> float:
    """``0.5 * D * _LOG_2PI`` evaluated in float32 as in gpmdm_pf.py:191."""
    return float(np.float32(np.float32(0.5 * D) * LOG_2PI_F32))


# ----------------------------------------------------------------------------
# kernels (gpmdm.py:381-548)
# ----------------------------------------------------------------------------

def weighted_distances(X1, X2, log_ls):
    """gpmdm.py:483-517 -- expansion form |a|^2 + |b|^2 - 2 a.b with a = x / l."""
    ls = np.exp(log_ls)
    a = X1 / ls
    b = X2 / ls
    a2 = np.sum(a * a, axis=1, keepdims=True)
    b2 = np.sum(b * b, axis=1, keepdims=True)
    return a2 + b2.T - 2.0 * (a @ b.T)


def rbf_kernel(X1, X2, log_ls, log_sigma_n=None, sigma_n_num=0.0, noise=False):
    """gpmdm.py:436-481 -- exp(-dist) (no 1/2), optional noise on the diagonal."""
    K = np.exp(-weighted_distances(X1, X2, log_ls))
    if noise:
        n = X1.shape[0]
        K = K + np.exp(log_sigma_n) ** 2 * np.eye(n) + sigma_n_num ** 2 * np.eye(n)
    return K


def lin_kernel(X1, X2, log_lin_coeff):
    """gpmdm.py:520-548 -- [x,1] diag(c^2) [x',1]^T."""
    S = np.diag(np.exp(log_lin_coeff) ** 2)
    X1 = np.concatenate([X1, np.ones((X1.shape[0], 1))], 1)
    X2 = np.concatenate([X2, np.ones((X2.shape[0], 1))], 1)
    return X1 @ (S @ X2.T)


def x_diag_kernel(Xs, log_lin_coeff):
    """gpmdm.py:1070-1101 with flg_noise=False: 1 + sum([x,1] diag(c^2) * [x,1])."""
    S = np.diag(np.exp(log_lin_coeff) ** 2)
    Xt = np.concatenate([Xs, np.ones((Xs.shape[0], 1))], 1)
    return np.ones(Xs.shape[0]) + np.sum((Xt @ S) * Xt, axis=1)


def chol_inverse(K):
    """gpmdm.py:1286-1289: U = chol(K, upper); U^-1 U^-T."""
    L = np.linalg.cholesky(K)
    U = L.T
    Uinv = np.linalg.inv(U)
    return Uinv @ Uinv.T


# ----------------------------------------------------------------------------
# model
# ----------------------------------------------------------------------------

@dataclass
class OracleModel:
    X: np.ndarray                 # (N, d) latent training points, class-major
    Y: np.ndarray                 # (N, D) observations (meanY = 0, gpmdm.py:791)
    seq_lengths: list             # seq_lengths[c] = list of sequence lengths of class c
    y_log_lengthscales: np.ndarray
    y_log_lambdas: np.ndarray
    y_log_sigma_n: float
    x_log_lengthscales: np.ndarray
    x_log_lambdas: np.ndarray
    x_log_sigma_n: float
    x_log_lin_coeff: np.ndarray
    sigma_n_num_X: float = 0.0
    sigma_n_num_Y: float = 0.0
    # derived
    Ky_inv: np.ndarray = field(default=None, repr=False)
    Xin_c: list = field(default=None, repr=False)
    Xout_c: list = field(default=None, repr=False)
    Kx_inv_c: list = field(default=None, repr=False)
    Kx_R_c: list = field(default=None, repr=False)

    @property
    def n_classes(self):
        return len(self.seq_lengths)

    @property
    def D(self):
        return self.Y.shape[1]

    @property
    def d(self):
        return self.X.shape[1]

    def X_for_class(self, c):
        """gpmdm.py:906-921."""
        per = [sum(s) for s in self.seq_lengths]
        start = sum(per[:c])
        return self.X[start:start + per[c]]

    def xin_xout(self):
        """gpmdm.py:630-718, target 'full', back_step 1: per sequence X[:-1] / X[1:],
        concatenated in observations_list order (class-major)."""
        Xin, Xout, cls = [], [], []
        off = 0
        for c, lens in enumerate(self.seq_lengths):
            for L in lens:
                seq = self.X[off:off + L]
                Xin.append(seq[:-1])
                Xout.append(seq[1:])
                cls.append(np.full(L - 1, c))
                off += L
        return np.concatenate(Xin), np.concatenate(Xout), np.concatenate(cls)

    def precompute(self, obs_factor: str = "inverse", dyn_form: str = "inverse"):
        """gpmdm.py:1284-1305 (class blocks only for the dynamics inverse).

        ``obs_factor="cholesky"`` keeps the lower Cholesky factor L of K_y instead of the
        explicit inverse and evaluates the observation map with triangular solves
        (``k^T K_y^-1 k = |L^-1 k|^2``, mean weights ``K_y^-1 Y`` by two solves): the same
        mathematics with a third of the O(N^3) setup, for the N = 10^4 / 2 x 10^4
        configurations where the explicit recipe would dominate a test's run time.

        ``dyn_form="triangular"`` evaluates the dynamics GP's quadratic form as |R_c^T k|^2
        with R_c = U_c^-1 (the same Cholesky recipe, gpmdm.py:1299-1305: A_c = R_c R_c^T) and
        the linear kernel folded into H = (X~in C^2)^T R_c (k^T R_c = k_rbf^T R_c + x~^T H):
        the same mathematics in another fp64 association.  The dynamics variance
        vc = k_diag - k^T A_c k cancels (k_diag carries the linear kernel's diagonal, ~1e2 at
        config 3), so the two associations differ by ~1e-7..1e-6 relative in vc and ~1e-6 in
        the next weights (tools/oracle_recipe_spread.py): the large-config tests check the
        device, which uses the triangular association, against both forms."""
        Ky = rbf_kernel(self.X, self.X, self.y_log_lengthscales, self.y_log_sigma_n,
                        self.sigma_n_num_Y, noise=True)
        self.Ly = None
        if obs_factor == "cholesky":
            from scipy.linalg import cho_factor, cho_solve
            L, _ = cho_factor(Ky, lower=True, overwrite_a=True, check_finite=False)
            self.Ly = np.tril(L)
            self.beta_y = cho_solve((self.Ly, True), self.Y, check_finite=False)
        else:
            self.Ky_inv = chol_inverse(Ky)
        del Ky
        Xin, Xout, cls = self.xin_xout()
        self.Xin_c, self.Xout_c, self.Kx_inv_c, self.Kx_R_c = [], [], [], []
        for c in range(self.n_classes):
            m = cls == c
            xi, xo = Xin[m], Xout[m]
            K = rbf_kernel(xi, xi, self.x_log_lengthscales, self.x_log_sigma_n,
                           self.sigma_n_num_X, noise=True)
            K = K + lin_kernel(xi, xi, self.x_log_lin_coeff)
            K = K + 1e-6 * np.eye(K.shape[0])
            self.Xin_c.append(xi)
            self.Xout_c.append(xo)
            if dyn_form == "triangular":
                Rc = np.linalg.inv(np.linalg.cholesky(K).T)            # U^-1, upper
                self.Kx_R_c.append(Rc)
                self.Kx_inv_c.append(Rc @ Rc.T)
            else:
                self.Kx_inv_c.append(chol_inverse(K))
        return self

    def with_triangular_dynamics(self):
        """A copy sharing this model's observation factor whose dynamics GPs use the
        triangular association (precompute's ``dyn_form="triangular"``)."""
        import copy
        o = copy.copy(self)
        o.Kx_R_c, o.Kx_inv_c = [], []
        for c in range(self.n_classes):
            xi = self.Xin_c[c]
            K = rbf_kernel(xi, xi, self.x_log_lengthscales, self.x_log_sigma_n, self.sigma_n_num_X, noise=True)
            K = K + lin_kernel(xi, xi, self.x_log_lin_coeff) + 1e-6 * np.eye(K.shape[0])
            Rc = np.linalg.inv(np.linalg.cholesky(K).T)
            o.Kx_R_c.append(Rc)
            o.Kx_inv_c.append(Rc @ Rc.T)
        return o

    # -- predictive maps ------------------------------------------------------

    def map_x_to_y(self, Xs):
        """gpmdm.py:923-963 (flg_noise=False)."""
        Ks = rbf_kernel(self.X, Xs, self.y_log_lengthscales)            # N x P
        if getattr(self, "Ly", None) is not None:
            from scipy.linalg import solve_triangular
            mean = Ks.T @ self.beta_y
            V = solve_triangular(self.Ly, Ks, lower=True, check_finite=False)
            vc = np.ones(Xs.shape[0]) - np.sum(V * V, axis=0)
        else:
            mean = ((self.Y.T @ self.Ky_inv) @ Ks).T
            vc = np.ones(Xs.shape[0]) - np.sum((Ks.T @ self.Ky_inv) * Ks.T, axis=1)
        lam = np.exp(self.y_log_lambdas) ** -2
        return mean, vc[:, None] * lam[None, :]

    def map_x_dynamics_for_class(self, Xs, c):
        """gpmdm.py:1032-1068 (flg_noise=False), restricted to the class-c block."""
        xi, xo, A = self.Xin_c[c], self.Xout_c[c], self.Kx_inv_c[c]
        Ks = rbf_kernel(xi, Xs, self.x_log_lengthscales) + lin_kernel(xi, Xs, self.x_log_lin_coeff)
        kd = x_diag_kernel(Xs, self.x_log_lin_coeff)
        mean = ((xo.T @ A) @ Ks).T
        if getattr(self, "Kx_R_c", None):                # precompute(dyn_form="triangular")
            R = self.Kx_R_c[c]
            c2 = np.exp(self.x_log_lin_coeff) ** 2
            xt_in = np.concatenate([xi, np.ones((xi.shape[0], 1))], 1)
            xt = np.concatenate([Xs, np.ones((Xs.shape[0], 1))], 1)
            V = rbf_kernel(xi, Xs, self.x_log_lengthscales).T @ R + xt @ ((xt_in * c2).T @ R)
            vc = kd - np.sum(V * V, axis=1)
        else:
            vc = kd - np.sum((Ks.T @ A) * Ks.T, axis=1)
        lam = np.exp(self.x_log_lambdas) ** -2
        return mean, vc[:, None] * lam[None, :]


# ----------------------------------------------------------------------------
# training loss (gpmdm.py:550-628, 721-760): next-row oracle for GPMDM.gpdm_loss
# ----------------------------------------------------------------------------

def y_neg_log_likelihood(model: OracleModel):
    """gpmdm.py:550-590: D/2 log|K_y| + 1/2 tr(K_y^-1 Y W^2 Y^T) - N * 2 sum(y_log_lambdas)
    (the reference's ``log_det_W`` is 2 sum(log lambda), i.e. log|W^2|)."""
    N, D = model.Y.shape
    Ky = rbf_kernel(model.X, model.X, model.y_log_lengthscales, model.y_log_sigma_n,
                    model.sigma_n_num_Y, noise=True)
    L = np.linalg.cholesky(Ky)
    logdet = 2.0 * np.sum(np.log(np.diag(L)))
    W2 = np.exp(model.y_log_lambdas) ** 2
    tr = np.trace(chol_inverse(Ky) @ ((model.Y * W2) @ model.Y.T))
    return D / 2 * logdet + 0.5 * tr - N * 2.0 * np.sum(model.y_log_lambdas)


def x_neg_log_likelihood(model: OracleModel):
    """gpmdm.py:592-628 with the class mask (gpmdm.py:311-341): K_x = (RBF + noise + lin)
    (Xin, Xin) * M is block diagonal, so log|K_x| and the trace split over class blocks."""
    Xin, Xout, cls = model.xin_xout()
    d = Xout.shape[1]
    W2 = np.exp(model.x_log_lambdas) ** 2
    logdet, tr = 0.0, 0.0
    for c in range(model.n_classes):
        m = cls == c
        xi, xo = Xin[m], Xout[m]
        K = rbf_kernel(xi, xi, model.x_log_lengthscales, model.x_log_sigma_n,
                       model.sigma_n_num_X, noise=True) + lin_kernel(xi, xi, model.x_log_lin_coeff)
        L = np.linalg.cholesky(K)
        logdet += 2.0 * np.sum(np.log(np.diag(L)))
        tr += np.trace(chol_inverse(K) @ ((xo * W2) @ xo.T))
    return d / 2 * logdet + 0.5 * tr - Xin.shape[0] * 2.0 * np.sum(model.x_log_lambdas)


def gpdm_loss(model: OracleModel, balance: float = 1.0):
    """gpmdm.py:721-760: L_y + balance * L_x."""
    return y_neg_log_likelihood(model) + balance * x_neg_log_likelihood(model)


# ----------------------------------------------------------------------------
# particle filter (gpmdm_pf.py)
# ----------------------------------------------------------------------------

def divide_into_n_parts(x, n):
    """gpmdm_pf.py:287-292."""
    g, r = divmod(x, n)
    return [g + (1 if i < r else 0) for i in range(n)]


def init_particles(model: OracleModel, P: int, init_idx: list):
    """gpmdm_pf.py:87-115; init_idx[c] = the randint draws of class c."""
    counts = divide_into_n_parts(P, model.n_classes)
    states, classes = [], []
    for c in range(model.n_classes):
        Xc = model.X_for_class(c)
        idx = np.asarray(init_idx[c], dtype=np.int64)
        assert idx.shape[0] == counts[c]
        states.append(Xc[idx])
        classes += [c] * counts[c]
    return np.concatenate(states, 0).copy(), np.asarray(classes, dtype=np.int64)


def switch_classes(classes, T, E):
    """gpmdm_pf.py:137-151 with torch.multinomial(p, 1) = argmax(p / Exp(1)) (first max)."""
    probs = T[classes]
    return np.argmax(probs / E, axis=1).astype(np.int64)


def class_grouped_order(classes, C):
    """Particle indices grouped by class, ascending inside a class (gpmdm_pf.py:158-161)."""
    return [np.nonzero(classes == c)[0] for c in range(C)]


def propagate_dynamics(model: OracleModel, states, classes, normals):
    """gpmdm_pf.py:153-168; ``normals`` is the concatenation over classes (in class order)
    of the randn(P_c, d) draws of torch.normal(mean, std) = mean + std * eps."""
    out = states.copy()
    pos = 0
    for c, idx in enumerate(class_grouped_order(classes, model.n_classes)):
        n = idx.shape[0]
        if n == 0:
            continue
        mu, var = model.map_x_dynamics_for_class(states[idx], c)
        eps = normals[pos:pos + n]
        out[idx] = eps * np.sqrt(var) + mu
        pos += n
    return out


def log_likelihoods(model: OracleModel, states, z):
    """gpmdm_pf.py:183-192 (the per-particle loop, vectorised; same formula)."""
    mean, var = model.map_x_to_y(states)
    z = np.asarray(z, dtype=np.float64)
    mu_term = -0.5 * np.sum((z[None, :] - mean) ** 2 / var + np.log(var), axis=1)
    sig_term = np.sum(-np.log(np.sqrt(var)), axis=1)
    return mu_term + sig_term - loglik_const(model.D)


def normalise(ll):
    """gpmdm_pf.py:200-204."""
    log_w = ll - np.max(ll)
    w = np.exp(log_w)
    return log_w, w / np.sum(w)


def multinomial_resample_indices(w, u):
    """torch CPU multinomial(w, n, replacement=True): sequential cumsum, divide by the
    sum, last bucket forced to 1, first index with cum >= u (binary search)."""
    cum = np.cumsum(w)
    s = cum[-1]
    if s > 0 or (0.99999 < s < 1.00001):
        cum = cum / s
    cum[-1] = 1.0
    return np.searchsorted(cum, u, side="left").astype(np.int64)


def systematic_resample_indices(w, u0):
    """Systematic resampling (BASELINE.json north_star; not in the reference, which only
    has multinomial, gpmdm_pf.py:211): slot s takes the first index whose normalised CDF
    (the same CDF as the multinomial search) reaches (s + u0) / P."""
    P = w.shape[0]
    cum = np.cumsum(w)
    cum = cum / cum[-1]
    cum[-1] = 1.0
    u = (np.arange(P, dtype=np.float64) + u0) / float(P)
    return np.searchsorted(cum, u, side="left").astype(np.int64)


def class_probabilities(ll, log_w, classes, C):
    """gpmdm_pf.py:224-248 (post-resample classes with pre-resample ll/log_w)."""
    lw = ll + log_w
    lw = lw - np.max(lw)
    e = np.exp(lw)
    cl = np.array([np.sum(e[classes == c]) for c in range(C)])
    return cl / np.sum(cl)


def current_state_mean(states, w):
    """gpmdm_pf.py:256-262."""
    return np.sum(states * w[:, None], axis=0)


def log_likelihood_readout(ll, log_w):
    """gpmdm_pf.py:215-222, 302-312 (not a log, as in the reference)."""
    lw = log_w + ll
    return float(np.sum(np.exp(lw - np.max(lw))))


@dataclass
class StepResult:
    classes_switched: np.ndarray
    states_propagated: np.ndarray
    ll: np.ndarray
    log_w: np.ndarray
    w: np.ndarray
    resample_idx: np.ndarray
    states: np.ndarray          # post-resample
    classes: np.ndarray         # post-resample
    posterior: np.ndarray
    mean: np.ndarray
    lik: float


def step(model: OracleModel, T, states, classes, z, E, normals, u, resample="multinomial",
         normals_by_particle=False) -> StepResult:
    """One ``GPMDM_PF.update(z)`` (gpmdm_pf.py:117-135) plus the read-outs.

    ``u``: P uniforms (multinomial, the reference) or the systematic offset u0.
    ``normals_by_particle``: the draws are indexed by particle (Philox filters,
    ``oracle.philox.dynamics_normals``) instead of the reference's class-grouped order."""
    C = model.n_classes
    cls1 = switch_classes(classes, T, E)
    if normals_by_particle:
        normals = np.concatenate([normals[cls1 == c] for c in range(C)], 0)
    st1 = propagate_dynamics(model, states, cls1, normals)
    ll = log_likelihoods(model, st1, z)
    log_w, w = normalise(ll)
    if resample == "multinomial":
        idx = multinomial_resample_indices(w, u)
    else:
        idx = systematic_resample_indices(w, float(np.asarray(u).reshape(-1)[0]))
    st2, cls2 = st1[idx], cls1[idx]
    post = class_probabilities(ll, log_w, cls2, C)
    mean = current_state_mean(st2, w)
    lik = log_likelihood_readout(ll, log_w)
    return StepResult(cls1, st1, ll, log_w, w, idx, st2, cls2, post, mean, lik)
