"""GPU: a checkpoint written by the reference's GPMDM.save (tests/golden/make_checkpoint.py,
after 20 steps of the reference's own train_adam) loads through GPMDM.load and its
predictive maps match the reference's outputs for that trained model (gpmdm.py:923-963,
1032-1068; tolerances of tests/test_gpu_parity.py), and a filter on it steps like the
oracle built from the same parameters."""
import numpy as np
import pytest
import torch

from conftest import GOLDEN, assert_step_matches, nrel, oracle_model

pytestmark = pytest.mark.gpu


def test_reference_checkpoint_predictive_maps_and_step():
    from gpmdm_amd import GPMDM, GPMDM_PF, synthetic
    from oracle import gpmdm_oracle as O
    f = dict(np.load(GOLDEN / "ref_checkpoint_config1.npz", allow_pickle=False))
    m = GPMDM.load(GOLDEN / "ref_checkpoint_config1.pth")
    for c in range(m.n_classes):
        mu, var = m.map_x_dynamics_for_class(torch.tensor(f[f"dyn{c}_xs"]), c)
        assert nrel(mu.numpy(), f[f"dyn{c}_mu"]) < 1e-8, c
        assert nrel(var.numpy(), f[f"dyn{c}_var"]) < 1e-5, c
    mu, var = m.map_x_to_y(torch.tensor(f["obs_xs"]))
    assert nrel(mu.numpy(), f["obs_mu"]) < 1e-8
    assert nrel(var.numpy(), f["obs_var"]) < 1e-6
    om = oracle_model(f)
    T = synthetic.markov_matrix(2)
    P = 3000
    pf = GPMDM_PF(m, torch.tensor(T), P, rng="torch")
    st0 = pf.export_state()
    rng = np.random.RandomState(3)
    E, nrm, u = rng.exponential(size=(P, 2)), rng.randn(P, 3), rng.rand(P)
    z = f["Y"][42] + 0.02
    pf.update_with_draws(z, E, nrm, u)
    r = O.step(om, T, st0["states"], st0["classes"], z, E, nrm, u)
    assert_step_matches(pf.export_state(), r, pf.class_probabilities().numpy(), pf.current_state_mean().numpy(), u)


def test_map_performance_readouts_match_reference():
    """train_gpmdm.ipynb's evaluation calls (gpmdm.py:1147-1273) on the reference-written
    checkpoint against the reference's own outputs for it (tests/golden/
    make_map_performance.py).  NMSE is a mean of floors, (target - mu)^2 // var, so a
    value within rounding of an integer may floor the other way: at most 0.2% of the
    entries may differ by one."""
    from gpmdm_amd import GPMDM
    g = dict(np.load(GOLDEN / "ref_map_performance_config1.npz", allow_pickle=False))
    m = GPMDM.load(GOLDEN / "ref_checkpoint_config1.pth")

    def nmse_close(got, want, n):
        assert abs(got - want) * n <= max(1.0, 0.002 * n), (got, want)

    for c in range(m.n_classes):
        mu, var, Xout, Xin, nmse = m.get_dynamics_map_performance_for_class(c)
        assert np.array_equal(Xin, g["dyn_Xin"]) and np.array_equal(Xout, g["dyn_Xout"])
        assert nrel(mu, g[f"dyn{c}_mu"]) < 1e-8, c
        assert nrel(var, g[f"dyn{c}_var"]) < 1e-5, c
        nmse_close(nmse, float(g[f"dyn{c}_nmse"]), mu.size)
        lo, hi = g[f"obs{c}_rows"]
        mu, var, Y, nmse = m.get_latent_map_performance_for_class(c)
        assert nrel(mu, g["obs_mu"][lo:hi]) < 1e-8, c
        assert nrel(var, g["obs_var"][lo:hi]) < 1e-6, c
        nmse_close(nmse, float(g[f"obs{c}_nmse"]), mu.size)
    mu, var, Y, nmse = m.get_latent_map_performance()
    assert nrel(mu, g["obs_mu"]) < 1e-8
    assert nrel(var, g["obs_var"]) < 1e-6
    nmse_close(nmse, float(g["obs_nmse"]), mu.size)
    # get_next_x: the mean for 'full' targets, a N(mean, var) draw with flg_sample
    x = m.get_next_x(torch.ones(1, 3), torch.full((1, 3), 1e-12), torch.zeros(1, 3), flg_sample=True)
    assert torch.allclose(x, torch.ones(1, 3), atol=1e-4)


def test_all_class_dynamics_map_matches_reference():
    """map_x_dynamics (gpmdm.py:993-1030: the M-masked, un-jittered Kx_inv against the
    unmasked kernel) on the reference-trained checkpoint."""
    from gpmdm_amd import GPMDM
    g = dict(np.load(GOLDEN / "ref_map_performance_config1.npz", allow_pickle=False))
    m = GPMDM.load(GOLDEN / "ref_checkpoint_config1.pth")
    mu, var = m.map_x_dynamics(torch.tensor(g["alldyn_xs"]))
    assert nrel(mu.numpy(), g["alldyn_mu"]) < 1e-8
    assert nrel(var.numpy(), g["alldyn_var"]) < 1e-6


def test_load_state_dict_rebuilds_the_device_model():
    """load_state_dict installs parameters by the reference's names and rebuilds the device
    model; a filter built before rebinds (the reference filter reads its model live)."""
    from gpmdm_amd import GPMDM, GPMDM_PF, synthetic
    m = GPMDM.load(GOLDEN / "ref_checkpoint_config1.pth")
    xs = torch.tensor(np.random.RandomState(4).randn(64, 3))
    mu0, var0 = m.map_x_to_y(xs)
    pf = GPMDM_PF(m, torch.tensor(synthetic.markov_matrix(2)), 1000, rng="philox", seed=3)
    sd = m.state_dict()
    sd["y_log_lambdas"] = sd["y_log_lambdas"] + 0.1
    m.load_state_dict(sd)
    mu1, var1 = m.map_x_to_y(xs)
    assert nrel(mu1.numpy(), mu0.numpy()) < 1e-12            # the mean does not use the lambdas
    assert nrel(var1.numpy(), var0.numpy() * np.exp(-0.2)) < 1e-12
    pf.update(np.zeros(m.D))                                 # rebinds to the rebuilt model
    assert np.isfinite(pf.class_probabilities().numpy()).all()
