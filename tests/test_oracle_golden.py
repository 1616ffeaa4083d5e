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
