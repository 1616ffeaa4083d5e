"""GPDM training on the GPU: the reference's loss and Adam loop.

Mirrors ``/root/reference/gpmdm/gpmdm.py``:

* ``get_y_neg_log_likelihood`` (gpmdm.py:550-590)
      L_y = D/2 log|K_y| + 1/2 tr(K_y^-1 Y W_y^2 Y^T) - N log|W_y^2|
* ``get_x_neg_log_likelihood`` (gpmdm.py:592-628)
      L_x = d/2 log|K_x| + 1/2 tr(K_x^-1 Xout W_x^2 Xout^T) - Nx log|W_x^2|
  with K_x = (RBF + noise + linear)(Xin, Xin) masked to the class blocks (gpmdm.py:311-341);
* ``gpdm_loss`` (gpmdm.py:721-760) = L_y + balance L_x;
* ``train_adam`` (gpmdm.py:817-885): Adam over every parameter (``set_training_mode('all')``).

Design (MI355X): everything runs in fp64 on the model's device through torch (rocSOLVER
Cholesky and inverse, rocBLAS GEMMs, autograd).  Each log-determinant comes from the
Cholesky diagonal and each (log|K|, trace) pair has a closed-form backward
(``_LogdetTrace``); the dynamics term is evaluated block by block (the masked matrix is
block diagonal, so the blocks are the whole of it): O(sum N_c^2) memory instead of the
dense mask's O(Nx^2).

Reference behaviour kept: ``cholesky_ex`` info is not checked (a non-positive-definite
kernel gives NaN, and ``train_adam`` stops with a message as the reference does); the
``balance`` argument of ``train_adam`` reaches ``gpdm_loss`` in the position of its unused
``M`` argument (gpmdm.py:865 vs 721), so the dynamics term always has weight 1.
"""
from __future__ import annotations

import time

import torch

PARAM_NAMES = ("y_log_lengthscales", "y_log_lambdas", "y_log_sigma_n", "x_log_lengthscales",
               "x_log_lambdas", "x_log_sigma_n", "x_log_lin_coeff", "X")


def sq_dist(X1, X2, log_ls):
    """gpmdm.py:483-517 (expansion form |a|^2 + |b|^2 - 2 a.b, a = x / l)."""
    ls = torch.exp(log_ls)
    a = X1 / ls
    b = X2 / ls
    return (a * a).sum(1, keepdim=True) + (b * b).sum(1, keepdim=True).T - 2.0 * (a @ b.T)


def lin_kernel(X1, X2, log_c):
    """gpmdm.py:520-548: [x, 1] diag(c^2) [x', 1]^T."""
    c2 = torch.exp(log_c) ** 2
    o1 = torch.ones(X1.shape[0], 1, dtype=X1.dtype, device=X1.device)
    o2 = torch.ones(X2.shape[0], 1, dtype=X2.dtype, device=X2.device)
    return (torch.cat([X1, o1], 1) * c2) @ torch.cat([X2, o2], 1).T


# Above this size K^-1 and log|K| come from the library (gpmdm_spd_inverse: rocSOLVER potrf +
# potri on the tensor's own buffer, with a library-owned rocBLAS handle): this ROCm build's
# torch hipSOLVER / hipBLAS paths fail to allocate workspace for N x N right-hand sides at
# N >= 10^4 (tools/inv_probe.sh).  Below it, torch's cholesky_ex + cholesky_inverse.
_LIB_MIN_N = 8193


def _inverse_and_logdet(K):
    """(K^-1, log|K|) of a symmetric positive-definite device matrix.  A matrix that is not
    positive definite gives NaN (the reference ignores cholesky_ex's info)."""
    n = K.shape[0]
    if n < _LIB_MIN_N:
        L, _ = torch.linalg.cholesky_ex(K)
        return torch.cholesky_inverse(L), 2.0 * torch.sum(torch.log(torch.diagonal(L)))
    import ctypes
    from . import _lib
    if n > 46340:                       # the library's own bound (rocBLAS int32 indexing of n*n)
        raise ValueError(f"gpmdm_spd_inverse: n={n} exceeds 46340")
    A = K.detach().contiguous().clone()
    ld = ctypes.c_double()
    rc = _lib.load().gpmdm_spd_inverse(A.device.index or 0, ctypes.c_void_p(A.data_ptr()), n, ctypes.byref(ld),
                                       ctypes.c_void_p(torch.cuda.current_stream(A.device).cuda_stream))
    if rc == _lib.GPMDM_E_INVALID:      # not positive definite: NaN, as the reference's cholesky_ex
        A.fill_(float("nan"))
    else:                               # HIP / rocSOLVER failure, out of memory, n too large: raise
        _lib.check(rc, "gpmdm_spd_inverse")
    return A, torch.tensor(ld.value, dtype=K.dtype, device=K.device)


class _LogdetTrace(torch.autograd.Function):
    """(log|K|, tr(K^-1 B B^T)) with a closed-form backward.

    forward:  K^-1 and log|K| from the Cholesky factor (potrf + potri; info unchecked, as
              the reference: NaN), A = K^-1 B, tr = sum(A * B)
    backward: d log|K| / dK = K^-1,  d tr / dK = -A A^T,  d tr / dB = 2 A
    Autograd through the Cholesky factor would run a trsm with an N x N right-hand side,
    which this ROCm build's hipBLAS fails to allocate for at N = 10^4; the closed form needs
    only GEMMs and the inverse the forward already has (the reference's own explicit
    inverse, gpmdm.py:582-584).
    """

    @staticmethod
    def forward(ctx, K, B):
        Kinv, logdet = _inverse_and_logdet(K)
        A = Kinv @ B
        ctx.save_for_backward(Kinv, A)
        return logdet, torch.sum(A * B)

    @staticmethod
    def backward(ctx, g_logdet, g_tr):
        Kinv, A = ctx.saved_tensors
        gK = g_logdet * Kinv - g_tr * (A @ A.T)
        gB = (2.0 * g_tr) * A
        return gK, gB


def _logdet_and_trace(K, B):
    """(log|K|, tr(K^-1 B B^T))."""
    return _LogdetTrace.apply(K, B)


def y_neg_log_likelihood(p, Y, sigma_n_num_Y):
    """L_y (gpmdm.py:550-590) for parameters ``p`` (dict of device tensors) and Y (N x D)."""
    N, D = Y.shape
    X = p["X"]
    eye = torch.eye(N, dtype=X.dtype, device=X.device)
    K = torch.exp(-sq_dist(X, X, p["y_log_lengthscales"])) \
        + (torch.exp(p["y_log_sigma_n"]) ** 2 + sigma_n_num_Y ** 2) * eye
    logdet, tr = _logdet_and_trace(K, Y * torch.exp(p["y_log_lambdas"]))
    return D / 2 * logdet + 0.5 * tr - N * (2.0 * torch.sum(p["y_log_lambdas"]))


def x_neg_log_likelihood(p, Xin, Xout, class_rows, sigma_n_num_X):
    """L_x (gpmdm.py:592-628): the masked K_x is block diagonal over the class blocks of
    Xin (``class_rows`` rows each, class-major)."""
    d = Xout.shape[1]
    W = torch.exp(p["x_log_lambdas"])
    s2 = torch.exp(p["x_log_sigma_n"]) ** 2 + sigma_n_num_X ** 2
    logdet = torch.zeros((), dtype=Xin.dtype, device=Xin.device)
    tr = torch.zeros((), dtype=Xin.dtype, device=Xin.device)
    off = 0
    for n_c in class_rows:
        xi, xo = Xin[off:off + n_c], Xout[off:off + n_c]
        off += n_c
        eye = torch.eye(n_c, dtype=xi.dtype, device=xi.device)
        K = torch.exp(-sq_dist(xi, xi, p["x_log_lengthscales"])) + s2 * eye \
            + lin_kernel(xi, xi, p["x_log_lin_coeff"])
        ld, t = _logdet_and_trace(K, xo * W)
        logdet = logdet + ld
        tr = tr + t
    return d / 2 * logdet + 0.5 * tr - Xin.shape[0] * (2.0 * torch.sum(p["x_log_lambdas"]))


class Trainer:
    """Device-resident copies of a GPMDM's trainable parameters and its observation matrix.

    ``model`` is a ``gpmdm_amd.GPMDM`` with data and latents (``init_X`` or a loaded model).
    """

    def __init__(self, model, device=None):
        if model.dyn_back_step != 1:
            # the reference's mask (gpmdm.py:320) counts len(seq) - 1 rows per sequence,
            # which only matches Xin for back_step 1
            raise NotImplementedError("training supports dyn_back_step=1, as the reference's mask does")
        self.model = model
        self.device = torch.device(device) if device is not None else model.device
        f64 = dict(dtype=torch.float64, device=self.device)
        self.Y = torch.as_tensor(model.get_Y(), **f64)
        self.p = {n: getattr(model, n).detach().to(**f64).clone().requires_grad_(True) for n in PARAM_NAMES}
        self.class_rows = model._class_dynamics_rows()

    def terms(self):
        m = self.model
        Xin, Xout, _ = m.get_Xin_Xout_matrices(X=self.p["X"])
        ly = y_neg_log_likelihood(self.p, self.Y, m.sigma_n_num_Y)
        lx = x_neg_log_likelihood(self.p, Xin, Xout, self.class_rows, m.sigma_n_num_X)
        return ly, lx

    def loss(self, balance=1.0):
        ly, lx = self.terms()
        return ly + balance * lx

    def write_back(self):
        """Copy the trained values into the model's (CPU) parameters."""
        m = self.model
        with torch.no_grad():
            for n in PARAM_NAMES:
                m._set_param(n, self.p[n].detach().to("cpu"))


def train_adam(model, num_opt_steps, num_print_steps=0, lr=0.01, balance=1.0):
    """gpmdm.py:817-885 on the model's GPU; returns the per-step losses and leaves the trained
    parameters in ``model`` with its device factors rebuilt (gpmdm.py:883)."""
    tr = Trainer(model)
    params = [tr.p[n] for n in PARAM_NAMES if model._trainable.get(n, True)]
    opt = torch.optim.Adam(params, lr=lr)
    if num_print_steps != 0:
        print("\n### Model Training (Adam) ###")
    losses = []
    t_start = time.time()
    # balance lands in gpdm_loss's unused M slot in the reference (gpmdm.py:865): weight 1
    del balance
    for epoch in range(num_opt_steps):
        opt.zero_grad()
        loss = tr.loss(1.0)
        loss.backward()
        if torch.isnan(loss):
            print("Loss is nan")
            break
        opt.step()
        losses.append(loss.item())
        if num_print_steps != 0 and epoch % num_print_steps == 0:
            print("\nGPDM Opt. EPOCH:", epoch)
            print("Running loss:", "{:.4e}".format(loss.item()))
            t_stop = time.time()
            print("Update time:", t_stop - t_start)
            t_start = t_stop
    tr.write_back()
    model._precompute_kernel_inverses()
    return losses
