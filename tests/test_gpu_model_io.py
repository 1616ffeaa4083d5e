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


def test_notebook_train_save_load_filter_chain(tmp_path):
    """train_gpmdm.ipynb cells 3-5 (construct, add_data, init_X, train_adam, save to .pth)
    -> test_gpmdm_pf.ipynb / view_gpmdm_pf.ipynb (GPMDM.load of that .pth, GPMDM_PF with
    100 particles, the per-frame update / get_most_likely_class / class_probabilities /
    current_state_mean loop writing into a torch tensor), unchanged but for the import
    line.  The loaded model is the trained one bit for bit: its maps and a filter run under
    the same torch seed equal the trained model's."""
    from gpmdm_amd import GPMDM, GPMDM_PF, synthetic
    data = synthetic.make_sequences(C=2, S=3, L=40, D=12, d=4, seed=5)
    d, DOFs = 4, 12
    gpdm = GPMDM(D=DOFs, d=d, n_classes=2, dyn_target='full', dyn_back_step=1,
                 y_lambdas_init=np.ones(DOFs), y_lengthscales_init=np.ones(d), y_sigma_n_init=1e-2,
                 x_lambdas_init=np.ones(d), x_lengthscales_init=np.ones(d), x_sigma_n_init=1e-2,
                 x_lin_coeff_init=np.ones(d + 1))
    for c, seqs in enumerate(data.sequences):
        for arr in seqs:
            gpdm.add_data(np.asarray(arr, dtype=np.float32), c)
    gpdm.init_X()
    gpdm.train_adam(num_opt_steps=5, num_print_steps=0, lr=0.01)
    path = tmp_path / "gpmdm_4d_30fps.pth"
    gpdm.save(f"{path}")
    assert path.exists()

    loaded = GPMDM.load(path)
    assert torch.equal(loaded.X, gpdm.X)
    xs = torch.tensor(np.random.RandomState(2).randn(50, d))
    for c in range(2):
        a, b = gpdm.map_x_dynamics_for_class(xs, c), loaded.map_x_dynamics_for_class(xs, c)
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    assert torch.equal(gpdm.map_x_to_y(xs)[1], loaded.map_x_to_y(xs)[1])

    T = torch.tensor([[0.9, 0.1], [0.1, 0.9]])
    frames = data.observation_stream(30, seed=1).astype(np.float32)

    def run(model):
        torch.manual_seed(0)
        gpdm_pf = GPMDM_PF(model, markov_switching_model=T, num_particles=100)
        gpdm_pf.reset()
        states = torch.zeros((len(frames), gpdm_pf.latent_dim))
        labels, probs = [], []
        for total, z in enumerate(frames):
            gpdm_pf.update(z)
            labels.append(gpdm_pf.get_most_likely_class())
            probs.append(gpdm_pf.class_probabilities().numpy().copy())
            states[total] = gpdm_pf.current_state_mean()
        return labels, np.array(probs), states

    l1, p1, s1 = run(gpdm)
    l2, p2, s2 = run(loaded)
    assert l1 == l2 and np.array_equal(p1, p2) and torch.equal(s1, s2)
    assert np.all(np.isfinite(p1)) and np.allclose(p1.sum(1), 1.0)


def test_external_optimizer_step_rebuilds_device_model():
    """An optimiser over GPMDM.parameters() on the reference's loss (gpdm_loss, gpmdm.py:
    721-760, differentiable through the model's parameters): after opt.step() the next use
    rebuilds the device model from the new parameters -- the maps equal those of a model
    freshly loaded from the updated state_dict, and a filter built before the step rebinds."""
    from gpmdm_amd import GPMDM, GPMDM_PF, synthetic
    m = GPMDM.load(GOLDEN / "ref_checkpoint_config1.pth")
    pf = GPMDM_PF(m, torch.tensor(synthetic.markov_matrix(2)), 500, rng="philox", seed=2)
    m.set_training_mode("all")
    gen0 = m.generation
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    loss = m.gpdm_loss(m.get_Y(), m.X.shape[0])
    loss.backward()
    assert m.X.grad is not None and torch.isfinite(m.X.grad).all()
    opt.step()
    xs = torch.tensor(np.random.RandomState(1).randn(40, 3))
    mu, var = m.map_x_to_y(xs)                   # triggers the rebuild
    assert m.generation == gen0 + 1
    fresh = GPMDM.load(GOLDEN / "ref_checkpoint_config1.pth")
    fresh.load_state_dict(m.state_dict())
    mu2, var2 = fresh.map_x_to_y(xs)
    assert torch.equal(mu, mu2) and torch.equal(var, var2)
    pf.update(np.zeros(m.D))                     # rebinds to the rebuilt model
    assert pf._model_gen == m.generation
