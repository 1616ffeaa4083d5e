"""GPU: the device-side GP factor (gpmdm_gp_factor).

R = U^-1 of the upper Cholesky factor and M = R R^T B from rocSOLVER/rocBLAS on the
device, checked against the CPU recipe the reference uses (torch cholesky_ex(upper) ->
inverse, gpmdm.py:1284-1305) and against the oracle's predictive maps when a whole model
is precomputed on the device.  Tolerances: R, M normwise rel <= 1e-9 (cond(K) ~ 1e3 here);
predictive means <= 1e-8, variances <= 1e-6 (as the golden tests).
"""
import ctypes

import numpy as np
import pytest
import torch

from conftest import nrel, oracle_model, product_model

pytestmark = pytest.mark.gpu


def _device_factor(X, ls, lin_c2, a, b, c, B):
    from gpmdm_amd import _lib
    lib = _lib.load()
    n, d = X.shape
    R, M = np.empty((n, n)), np.empty((n, B.shape[1]))
    c2 = None if lin_c2 is None else np.ascontiguousarray(lin_c2)
    _lib.check(lib.gpmdm_gp_factor(0, _lib.dptr(np.ascontiguousarray(X)), n, d, _lib.dptr(np.ascontiguousarray(ls)),
                                   _lib.dptr(c2), a, b, c, _lib.dptr(np.ascontiguousarray(B)), B.shape[1],
                                   _lib.dptr(R), _lib.dptr(M)), "gp_factor")
    return R, M


def _cpu_factor(X, ls, lin_c2, a, b, c, B):
    Xs = X / ls
    sq = (Xs * Xs).sum(1)
    K = np.exp(-(sq[:, None] + sq[None, :] - 2 * Xs @ Xs.T)) + (a + b) * np.eye(len(X))
    if lin_c2 is not None:
        Xt = np.concatenate([X, np.ones((len(X), 1))], 1)
        K = K + Xt @ np.diag(lin_c2) @ Xt.T
    K = K + c * np.eye(len(X))
    U, info = torch.linalg.cholesky_ex(torch.tensor(K), upper=True)
    assert int(info) == 0
    R = torch.triu(torch.inverse(U)).numpy()
    return R, (R @ R.T) @ B


@pytest.mark.parametrize("n,d,k,lin", [(1, 1, 1, False), (257, 3, 62, False), (1500, 8, 5, True), (999, 16, 16, True)])
def test_gp_factor_matches_cpu_recipe(n, d, k, lin):
    rng = np.random.RandomState(n)
    X = rng.randn(n, d)
    ls = rng.uniform(1.0, 2.0, d)
    c2 = rng.uniform(0.1, 0.6, d + 1) if lin else None
    B = rng.randn(n, k)
    a, b, c = 0.1 ** 2, 1e-4, (1e-6 if lin else 0.0)
    R, M = _device_factor(X, ls, c2, a, b, c, B)
    Rc, Mc = _cpu_factor(X, ls, c2, a, b, c, B)
    assert np.all(np.tril(R, -1) == 0.0)
    assert nrel(R, Rc) < 1e-9
    assert nrel(M, Mc) < 1e-9


def test_gp_factor_rejects_non_pd():
    from gpmdm_amd import _lib
    X = np.zeros((4, 2))                      # identical points: K = all ones, a = b = c = 0
    with pytest.raises(ValueError, match="positive definite"):
        _device_factor(X, np.ones(2), None, 0.0, 0.0, 0.0, np.ones((4, 1)))


def test_device_precomputed_model_vs_oracle(fx_config1):
    """A whole GPMDM precomputed on the device gives the oracle's predictive maps."""
    from gpmdm_amd import GPMDM
    m = product_model(fx_config1)
    m._precompute_device = "device"
    m._precompute_kernel_inverses()
    om = oracle_model(fx_config1)
    rng = np.random.RandomState(5)
    X = fx_config1["X"]
    xs = X[rng.randint(0, X.shape[0], 300)] + 0.1 * rng.randn(300, X.shape[1])
    mu, var = m.map_x_to_y(torch.tensor(xs))
    omu, ovar = om.map_x_to_y(xs)
    assert nrel(mu.numpy(), omu) < 1e-8 and nrel(var.numpy(), ovar) < 1e-6
    for c in range(m.n_classes):
        mu, var = m.map_x_dynamics_for_class(torch.tensor(xs), c)
        omu, ovar = om.map_x_dynamics_for_class(xs, c)
        assert nrel(mu.numpy(), omu) < 1e-8 and nrel(var.numpy(), ovar) < 1e-5
