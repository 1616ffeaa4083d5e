"""GPDM training on the GPU (gpmdm_amd/training.py) against the reference's own values
(tests/golden/training_n500.npz, made by tests/golden/make_golden_training.py from the
unmodified reference): loss terms and parameter gradients at the PCA initialisation of the
config-1 model, and five steps of train_adam(lr=0.01).

Tolerances: losses rel 1e-9; gradients normwise rel 1e-7 (the reference forms explicit
inverses, this a Cholesky + triangular solve; cond(K_y) ~ 1e4); Adam losses rel 1e-9 and
trained parameters normwise rel 1e-7.
"""
import numpy as np
import pytest
import torch

from conftest import load_fixture, nrel, oracle_model, product_model

pytestmark = pytest.mark.gpu

PARAMS = ("y_log_lengthscales", "y_log_lambdas", "y_log_sigma_n", "x_log_lengthscales",
          "x_log_lambdas", "x_log_sigma_n", "x_log_lin_coeff", "X")


@pytest.fixture(scope="module")
def ft():
    return load_fixture("training_n500")


def test_loss_terms_and_gradients_match_reference(ft):
    from gpmdm_amd import training
    m = product_model(ft)
    Y = m.get_Y()
    N = Y.shape[0]
    Xin, Xout, _ = m.get_Xin_Xout_matrices()
    ly = float(m.get_y_neg_log_likelihood(Y, m.X, N))
    lx = float(m.get_x_neg_log_likelihood(Xout, Xin))
    assert abs(ly - ft["loss_y0"]) <= 1e-9 * abs(ft["loss_y0"])
    assert abs(lx - ft["loss_x0"]) <= 1e-9 * abs(ft["loss_x0"])
    assert abs(float(m.gpdm_loss(Y, N)) - ft["loss0"]) <= 1e-9 * abs(ft["loss0"])
    tr = training.Trainer(m)
    loss = tr.loss()
    assert loss.device.type == "cuda"
    loss.backward()
    for p in PARAMS:
        g = tr.p[p].grad.detach().cpu().numpy().reshape(-1)
        assert nrel(g, ft[f"grad0_{p}"]) < 1e-7, p


def test_train_adam_matches_reference(ft):
    from oracle import gpmdm_oracle as O
    m = product_model(ft)
    losses = m.train_adam(5, lr=0.01, balance=1)
    ref = ft["adam_losses"]
    assert len(losses) == 5
    assert np.max(np.abs(np.asarray(losses) - ref) / np.abs(ref)) < 1e-9
    for p in PARAMS:
        v = getattr(m, p).detach().cpu().numpy().reshape(-1)
        assert nrel(v, ft[f"adam5_{p}"]) < 1e-7, p
    # the device model was rebuilt from the trained parameters
    arr = dict(ft)
    for p in PARAMS:
        arr[p] = ft[f"adam5_{p}"].reshape(np.shape(ft[p]))
    om = oracle_model(arr)
    xs = arr["X"][::7][:50] + 0.03
    mu, var = m.map_x_to_y(torch.tensor(xs))
    omu, ovar = om.map_x_to_y(xs)
    assert nrel(mu.numpy(), omu) < 1e-8 and nrel(var.numpy(), ovar) < 1e-6


def test_train_adam_balance_is_ignored_like_the_reference(ft):
    """gpmdm.py:865 passes ``balance`` into gpdm_loss's unused ``M`` slot, so the dynamics
    term keeps weight 1 whatever ``balance`` is."""
    m = product_model(ft)
    losses = m.train_adam(1, lr=0.01, balance=0.25)
    assert abs(losses[0] - ft["adam_losses"][0]) <= 1e-9 * abs(ft["adam_losses"][0])


def test_library_inverse_path_matches_reference(ft, monkeypatch):
    """The large-N path (K^-1 and log|K| from gpmdm_spd_inverse: rocSOLVER potrf + potri in
    the HIP library), forced at N = 500: loss terms and gradients against the reference."""
    from gpmdm_amd import training
    monkeypatch.setattr(training, "_LIB_MIN_N", 1)
    m = product_model(ft)
    tr = training.Trainer(m)
    ly, lx = tr.terms()
    assert abs(float(ly) - ft["loss_y0"]) <= 1e-9 * abs(ft["loss_y0"])
    assert abs(float(lx) - ft["loss_x0"]) <= 1e-9 * abs(ft["loss_x0"])
    (ly + lx).backward()
    for p in PARAMS:
        assert nrel(tr.p[p].grad.detach().cpu().numpy().reshape(-1), ft[f"grad0_{p}"]) < 1e-7, p


def test_spd_inverse_rejects_indefinite():
    import ctypes
    from gpmdm_amd import _lib
    A = torch.tensor([[1.0, 2.0], [2.0, 1.0]], dtype=torch.float64, device="cuda")
    ld = ctypes.c_double()
    rc = _lib.load().gpmdm_spd_inverse(0, ctypes.c_void_p(A.data_ptr()), 2, ctypes.byref(ld), None)
    assert rc == -1 and np.isnan(ld.value)
    assert b"positive definite" in _lib.load().gpmdm_last_error()
