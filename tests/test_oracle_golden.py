"""Pin the CPU oracle against golden vectors produced by the unmodified reference
(tests/golden/make_golden.py).  CPU only.

Tolerances: the oracle restates the reference formula for formula but inverts the
dynamics kernel per class block and uses numpy's LAPACK path, so it differs from the
reference by rounding amplified by conditioning (cond(K_x) ~ 1e6 because of the linear
kernel): dynamics variances ~4e-7 normwise, everything downstream far below the 1e-5
BASELINE tolerance.
"""
import numpy as np
import pytest

from conftest import load_fixture, nrel, oracle_model
from oracle import gpmdm_oracle as O


@pytest.mark.parametrize("name", ["config1_n500_p100_f200", "config2_n2000_p1000", "stress_n500_sigma001"])
def test_predictive_maps(name):
    from conftest import load_fixture
    f = load_fixture(name)
    m = oracle_model(f)
    var_tol = 5e-6 if "stress" not in name else 5e-4
    for c in range(m.n_classes):
        mu, var = m.map_x_dynamics_for_class(f[f"dyn{c}_xs"], c)
        assert nrel(mu, f[f"dyn{c}_mu"]) < 1e-8
        assert nrel(var, f[f"dyn{c}_var"]) < var_tol
    mu, var = m.map_x_to_y(f["obs_xs"])
    assert nrel(mu, f["obs_mu"]) < 1e-8
    assert nrel(var, f["obs_var"]) < 1e-6


def _per_step(f, pre):
    m = oracle_model(f)
    nF = f[pre + "E"].shape[0]
    z0 = f["z"].shape[0] - nF
    worst = {}
    for k in range(nF):
        r = O.step(m, f["T"], f[pre + "pre_states"][k], f[pre + "pre_classes"][k], f["z"][z0 + k],
                   f[pre + "E"][k], f[pre + "normals"][k], f[pre + "u"][k])
        assert np.array_equal(r.classes_switched, f[pre + "classes_switched"][k].reshape(-1))
        assert np.array_equal(r.classes, f[pre + "classes"][k].reshape(-1))
        for key, got, ref in [("st1", r.states_propagated, f[pre + "states_propagated"][k]),
                              ("w", r.w, f[pre + "w"][k]), ("states", r.states, f[pre + "states"][k]),
                              ("mean", r.mean, f[pre + "mean"][k])]:
            worst[key] = max(worst.get(key, 0.0), nrel(got, ref))
        worst["post"] = max(worst.get("post", 0.0), float(np.max(np.abs(r.posterior - f[pre + "posterior"][k]))))
        worst["lik"] = max(worst.get("lik", 0.0), abs(r.lik - f[pre + "lik"][k]) / abs(f[pre + "lik"][k]))
    return worst


def test_per_step_config1():
    from conftest import load_fixture
    w = _per_step(load_fixture("config1_n500_p100_f200"), "traj_")
    # weights / likelihood sum inherit the ~1e-8 state noise through a steep likelihood
    assert w["st1"] < 1e-7 and w["states"] < 1e-7 and w["w"] < 1e-5, w
    assert w["post"] < 1e-7 and w["mean"] < 1e-7 and w["lik"] < 1e-5, w


def test_per_step_config2():
    from conftest import load_fixture
    w = _per_step(load_fixture("config2_n2000_p1000"), "step_")
    assert w["st1"] < 1e-7 and w["states"] < 1e-7 and w["w"] < 1e-5, w
    assert w["post"] < 1e-7 and w["mean"] < 1e-7, w


def test_per_step_stress_sigma001():
    from conftest import load_fixture
    w = _per_step(load_fixture("stress_n500_sigma001"), "step_")
    assert w["states"] < 1e-6 and w["post"] < 1e-6, w


def test_trajectory_config1(fx_config1):
    """200 frames from the initial state with the captured draws: the trajectory stays
    on the reference's (sigma_n = 0.1)."""
    f = fx_config1
    m = oracle_model(f)
    parts = np.split(f["traj_init_idx"], np.cumsum(f["traj_init_counts"])[:-1])
    s, c = O.init_particles(m, 100, parts)
    assert np.array_equal(s, f["traj_pre_states"][0])
    wp = wm = 0.0
    for k in range(200):
        r = O.step(m, f["T"], s, c, f["z"][k], f["traj_E"][k], f["traj_normals"][k], f["traj_u"][k])
        s, c = r.states, r.classes
        assert np.array_equal(c, f["traj_classes"][k])
        wp = max(wp, float(np.max(np.abs(r.posterior - f["traj_posterior"][k]))))
        wm = max(wm, nrel(r.mean, f["traj_mean"][k]))
    assert wp < 1e-6 and wm < 1e-6, (wp, wm)


def test_loglik_constant_is_float32():
    # gpmdm_pf.py:5 -- float32 tensor; 0.5 * D * it stays float32 (gpmdm_pf.py:191)
    assert float(O.LOG_2PI_F32) == 1.8378770351409912
    assert O.loglik_const(62) == float(np.float32(31.0) * np.float32(1.8378770351409912))


def test_resample_edge_cases():
    w = np.array([0.0, 0.5, 0.0, 0.5])
    u = np.array([0.0, 0.25, 0.5, 0.5000001, 0.9999999])
    # u = 0 lands on the leading zero-weight bucket, exactly as torch's binary search does
    assert list(O.multinomial_resample_indices(w, u)) == [0, 1, 1, 3, 3]
    # a single particle
    assert list(O.multinomial_resample_indices(np.array([1.0]), np.array([0.3]))) == [0]


def test_switch_first_max_tie():
    T = np.array([[0.5, 0.5], [0.0, 1.0]])
    E = np.array([[1.0, 1.0], [1.0, 1.0]])
    assert list(O.switch_classes(np.array([0, 1]), T, E)) == [0, 1]


def test_oracle_training_loss_matches_reference():
    """The oracle's GPDM loss terms (gpmdm.py:550-628, 721-760) against the reference's
    values at the PCA initialisation of the config-1 model (tests/golden/training_n500.npz)."""
    from oracle import gpmdm_oracle as O
    f = load_fixture("training_n500")
    om = oracle_model(f)
    ly, lx = O.y_neg_log_likelihood(om), O.x_neg_log_likelihood(om)
    assert abs(ly - f["loss_y0"]) <= 1e-9 * abs(f["loss_y0"])
    assert abs(lx - f["loss_x0"]) <= 1e-9 * abs(f["loss_x0"])
    assert abs(O.gpdm_loss(om) - f["loss0"]) <= 1e-9 * abs(f["loss0"])


@pytest.mark.parametrize("name", ["config1_n500_p100_f200", "config2_n2000_p1000"])
def test_cholesky_observation_oracle_matches_reference(name):
    """precompute("cholesky") (triangular solves instead of the explicit K_y^-1 recipe; the
    large-configuration checker) against the reference's observation-map goldens."""
    f = load_fixture(name)
    m = oracle_model(f)
    mc = O.OracleModel(X=m.X, Y=m.Y, seq_lengths=m.seq_lengths, y_log_lengthscales=m.y_log_lengthscales,
                       y_log_lambdas=m.y_log_lambdas, y_log_sigma_n=m.y_log_sigma_n,
                       x_log_lengthscales=m.x_log_lengthscales, x_log_lambdas=m.x_log_lambdas,
                       x_log_sigma_n=m.x_log_sigma_n, x_log_lin_coeff=m.x_log_lin_coeff,
                       sigma_n_num_X=m.sigma_n_num_X, sigma_n_num_Y=m.sigma_n_num_Y).precompute("cholesky")
    mu, var = mc.map_x_to_y(f["obs_xs"])
    assert nrel(mu, f["obs_mu"]) < 1e-8
    assert nrel(var, f["obs_var"]) < 1e-6
    xs = f["obs_xs"] + 0.05
    assert nrel(mc.map_x_to_y(xs)[1], m.map_x_to_y(xs)[1]) < 1e-8


def test_philox_known_answers():
    """oracle/philox.py against the Philox4x32-10 known-answer vectors of Salmon et al.
    (Random123's kat_vectors: counter, key -> output)."""
    from oracle import philox as X
    kat = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
           ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
           ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
            (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]
    for ctr, key, out in kat:
        got = X.philox4x32_10(*[np.uint32(c) for c in ctr], *key)
        assert tuple(int(v) for v in got) == out


def test_philox_draw_transforms():
    """Shapes, ranges and moments of the restated device draws; streams and frames are
    independent; a bank's filter f equals a single filter keyed seed + f."""
    from oracle import philox as X
    P = 200_000
    E = X.switch_draws(7, 3, P, 3)
    assert E.shape == (P, 3) and np.all(E > 0) and abs(E.mean() - 1.0) < 0.01
    nrm = X.dynamics_normals(7, 3, P, 5)
    assert nrm.shape == (P, 5) and abs(nrm.mean()) < 0.01 and abs(nrm.std() - 1.0) < 0.01
    u = X.resample_uniforms(7, 3, P)
    assert np.all((u >= 0) & (u < 1)) and abs(u.mean() - 0.5) < 0.01
    assert not np.array_equal(u, X.resample_uniforms(7, 4, P))
    assert np.array_equal(X.resample_uniforms(7, 3, 50, f=2), X.resample_uniforms(9, 3, 50))
    assert 0.0 <= X.systematic_u0(7, 3) < 1.0
    # 64-bit key carry: seed + f crosses the 32-bit boundary
    k = X.filter_key(2 ** 32 - 1, 1)
    assert k == (0, 1)


def test_systematic_resample_oracle():
    """Systematic resampling: offspring counts within floor/ceil(P w_i); identical to an
    inverse-CDF search of the stratified uniforms (s + u0) / P."""
    rng = np.random.RandomState(3)
    for P in (1, 7, 1000):
        w = rng.exponential(size=P) ** 3
        w = w / w.sum()
        u0 = rng.rand()
        idx = O.systematic_resample_indices(w, u0)
        n = np.bincount(idx, minlength=P)
        assert np.all(n >= np.floor(P * w - 1e-9)) and np.all(n <= np.ceil(P * w + 1e-9))
        u = (np.arange(P) + u0) / P
        assert np.array_equal(idx, O.multinomial_resample_indices(w, u))


def test_oracle_map_performance_matches_reference():
    """The oracle's maps on the reference-trained checkpoint reproduce the reference's
    train_gpmdm.ipynb read-outs (gpmdm.py:1147-1273; tests/golden/make_map_performance.py),
    NMSE with the reference's floor division (up to 0.2% of entries flooring the other way)."""
    from conftest import GOLDEN
    f = dict(np.load(GOLDEN / "ref_checkpoint_config1.npz", allow_pickle=False))
    g = dict(np.load(GOLDEN / "ref_map_performance_config1.npz", allow_pickle=False))
    om = oracle_model(f)
    Xin, Xout, _ = om.xin_xout()
    assert np.array_equal(Xin, g["dyn_Xin"]) and np.array_equal(Xout, g["dyn_Xout"])
    for c in range(om.n_classes):
        mu, var = om.map_x_dynamics_for_class(Xin, c)
        assert nrel(mu, g[f"dyn{c}_mu"]) < 1e-8 and nrel(var, g[f"dyn{c}_var"]) < 1e-5
        nmse = float(np.mean((Xout - mu) ** 2 // var))
        assert abs(nmse - g[f"dyn{c}_nmse"]) * mu.size <= max(1.0, 0.002 * mu.size)
    mu, var = om.map_x_to_y(om.X)
    assert nrel(mu, g["obs_mu"]) < 1e-8 and nrel(var, g["obs_var"]) < 1e-6
    nmse = float(np.mean((om.Y - mu) ** 2 // var))
    assert abs(nmse - g["obs_nmse"]) * mu.size <= max(1.0, 0.002 * mu.size)
