"""GPU: model lifetime and failure detection.

* A filter outlives a rebuild of its model (``GPMDM.set_latents`` destroys the old device
  model): models are reference counted, and the filter rebinds to the rebuilt model on
  its next call, as the reference filter reads its GPMDM's current state
  (gpmdm_pf.py:164, 183).  The rebound filter must equal a filter built on the new model.
* Failure counters (``GPMDM_PF.health``): the reference's NaN propagation
  is kept, and every non-positive variance / non-finite log-likelihood or state is
  counted.  A deliberately inconsistent model (K_y^-1 scaled by 9: kT K^-1 k > 1) makes
  the observation variance negative and ll NaN, as the reference would; the sigma_n = 0.01
  stress model stays healthy in fp64 (fp32 would not).
"""
import numpy as np
import pytest
import torch

from conftest import product_model

pytestmark = pytest.mark.gpu


def test_filter_survives_model_rebuild(fx_config1):
    from gpmdm_amd import GPMDM_PF
    f = fx_config1
    m = product_model(f)
    T = torch.tensor(f["T"])
    pf = GPMDM_PF(m, T, 500, rng="torch")
    torch.manual_seed(1)
    pf.update(f["z"][0])
    old_gen = m.generation
    m.set_latents(m.X.detach().numpy() * 1.01)          # destroys the old handle, uploads a new model
    assert m.generation == old_gen + 1
    st0 = pf.export_state()
    rng = np.random.RandomState(2)
    E, nrm, u = rng.exponential(size=(500, 2)), rng.randn(500, m.d), rng.rand(500)
    pf.update_with_draws(f["z"][1], E, nrm, u)  # rebinds, then steps on the new model
    fresh = GPMDM_PF(m, T, 500, rng="torch")
    fresh.load_state(st0["states"], st0["classes"])
    fresh.update_with_draws(f["z"][1], E, nrm, u)
    a, b = pf.export_state(), fresh.export_state()
    for key in ("states", "classes", "ll", "resample_idx"):
        assert np.array_equal(a[key], b[key]), key
    assert np.array_equal(pf.predict().numpy(), fresh.predict().numpy())
    del m                                       # the filter still holds its model
    pf.update(f["z"][2])
    assert np.all(np.isfinite(pf.export_state()["states"]))


def test_health_counts_indefinite_model(fx_config1, monkeypatch):
    from gpmdm_amd import GPMDM_PF, model as model_mod
    f = fx_config1
    good = product_model(f)
    orig = model_mod._chol_inv_factor

    def scaled(K, what):
        R = orig(K, what)
        return 3.0 * R if what == "K_y" else R  # K_y^-1 -> 9 K_y^-1

    monkeypatch.setattr(model_mod, "_chol_inv_factor", scaled)
    bad = product_model(f)
    monkeypatch.setattr(model_mod, "_chol_inv_factor", orig)
    T = torch.tensor(f["T"])
    P = 1000
    for m, expect_bad in ((good, False), (bad, True)):
        pf = GPMDM_PF(m, T, P, rng="philox", seed=3)
        pf.update(f["z"][0])
        h = pf.health()
        ll = pf.export_state()["ll"]
        if expect_bad:
            n_neg = int(np.sum(~np.isfinite(ll)))
            assert h["obs_var_nonpositive"] > 0 and h["obs_ll_nonfinite"] == n_neg > 0, h
        else:
            assert h == {k: 0 for k in h}, h
        pf.health(reset=True)
        assert all(v == 0 for v in pf.health().values())


def test_stress_model_is_healthy_in_fp64(fx_stress):
    from gpmdm_amd import GPMDM_PF
    f = fx_stress
    m = product_model(f)
    pf = GPMDM_PF(m, torch.tensor(f["T"]), 5000, rng="philox", seed=12)
    for k in range(10):
        pf.update(f["z"][k % f["z"].shape[0]])
    assert all(v == 0 for v in pf.health().values()), pf.health()


def test_predictive_maps_on_concurrent_streams(fx_config2):
    """map_x_to_y / map_x_dynamics_for_class issued on two streams at once: each call owns
    its scratch (stream-ordered allocation) and passes its segment table by value, so the
    results equal the one-stream results bitwise."""
    m = product_model(fx_config2)
    rng = np.random.RandomState(5)
    X = m.X.detach().numpy()
    xa = torch.tensor(X[rng.randint(0, X.shape[0], 20_000)] + 0.1 * rng.randn(20_000, m.d)).cuda()
    xb = torch.tensor(X[rng.randint(0, X.shape[0], 7_000)] + 0.1 * rng.randn(7_000, m.d)).cuda()
    ref = [m.map_x_to_y(xa), m.map_x_to_y(xb), m.map_x_dynamics_for_class(xa, 0), m.map_x_dynamics_for_class(xb, 1)]
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        with torch.cuda.stream(s1):
            ga = m.map_x_to_y(xa)
            da = m.map_x_dynamics_for_class(xa, 0)
        with torch.cuda.stream(s2):
            gb = m.map_x_to_y(xb)
            db = m.map_x_dynamics_for_class(xb, 1)
        torch.cuda.synchronize()
        for got, want in zip((ga, gb, da, db), ref):
            assert torch.equal(got[0], want[0]) and torch.equal(got[1], want[1])


def test_step_call_order_is_enforced(fx_config1):
    """switch -> propagate_dynamics -> weigh -> resample (or switch -> propagate -> resample):
    a call out of order returns GPMDM_E_STATE and leaves the filter usable, and a step done
    in halves is bitwise the one-call step."""
    from gpmdm_amd import GPMDM_PF, _lib
    m = product_model(fx_config1)
    T = torch.tensor(fx_config1["T"])
    z = np.ascontiguousarray(fx_config1["z"][0], dtype=np.float64)
    lib = _lib.load()
    pfs = []
    for _ in range(2):
        torch.manual_seed(0)                 # same initial particles
        pfs.append(GPMDM_PF(m, T, 3000, rng="philox", seed=3))
    h, s = pfs[0]._h, pfs[0]._stream()
    assert lib.gpmdm_pf_weigh(h, _lib.dptr(z), s) == _lib.GPMDM_E_STATE
    assert lib.gpmdm_pf_propagate_dynamics(h, None, s) == _lib.GPMDM_E_STATE
    _lib.check(lib.gpmdm_pf_switch(h, None, None, s), "switch")
    _lib.check(lib.gpmdm_pf_propagate_dynamics(h, None, s), "propagate_dynamics")
    assert lib.gpmdm_pf_resample(h, None, s) == _lib.GPMDM_E_STATE
    assert lib.gpmdm_pf_set_dedup(h, 0) == _lib.GPMDM_E_STATE
    _lib.check(lib.gpmdm_pf_weigh(h, _lib.dptr(z), s), "weigh")
    _lib.check(lib.gpmdm_pf_resample(h, None, s), "resample")
    pfs[1].update(z)
    a, b = pfs[0].export_state(), pfs[1].export_state()
    for key in ("states", "classes", "ll", "resample_idx"):
        assert np.array_equal(a[key], b[key]), key
    # after a resample the next switch is already launched (pre-switch), but the order still
    # holds: propagate before gpmdm_pf_switch is refused, and the step completes after it
    assert lib.gpmdm_pf_propagate_dynamics(h, None, s) == _lib.GPMDM_E_STATE
    assert lib.gpmdm_pf_propagate(h, _lib.dptr(z), None, s) == _lib.GPMDM_E_STATE
    _lib.check(lib.gpmdm_pf_switch(h, None, None, s), "switch")
    _lib.check(lib.gpmdm_pf_propagate(h, _lib.dptr(z), None, s), "propagate")
    _lib.check(lib.gpmdm_pf_resample(h, None, s), "resample")
    pfs[1].update(z)
    a, b = pfs[0].export_state(), pfs[1].export_state()
    for key in ("states", "classes", "ll", "resample_idx"):
        assert np.array_equal(a[key], b[key]), key
