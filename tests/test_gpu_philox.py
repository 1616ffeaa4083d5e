"""GPU parity of the device-RNG mode (``rng='philox'``) -- the mode ``bench.py`` measures --
against the CPU oracle driven by the restated Philox draws (``oracle/philox.py``).

Each step is *resynced*: the oracle starts from the GPU's own pre-step particles (export),
draws the frame's numbers with the restated Philox4x32-10 keyed exactly as the kernels
key them (seed + filter, frame, particle index, stream), runs the reference step
(``oracle.gpmdm_oracle.step``, gpmdm_pf.py:117-262) and the GPU's post-step state must
match (``conftest.assert_step_matches``: weights 1e-5 normwise; resample indices equal to
the oracle's search of the GPU's weights with the restated uniforms, up to 2 last-ulp CDF
ties; classes exact; states 1e-6 normwise; posterior 1e-6 abs; state mean 1e-6).  The device's log /
sincos and numpy's may differ in the last ulp, which moves an Exp(1) or normal draw by
~1e-16 relative: far below every tolerance, and an argmax(T/E) flip would need a tie at
that level.
"""
import numpy as np
import pytest
import torch

from conftest import assert_step_matches, nrel, oracle_model, product_model

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def m2(fx_config2):
    return product_model(fx_config2)


@pytest.fixture(scope="module")
def om2(fx_config2):
    return oracle_model(fx_config2)


def _oracle_step(om, T, pre, z, seed, frame, resample, f=0):
    """(oracle StepResult, uniforms) of one step with the restated Philox draws."""
    from oracle import gpmdm_oracle as O
    from oracle import philox as X
    P, C, d = pre["states"].shape[0], T.shape[0], pre["states"].shape[1]
    E = X.switch_draws(seed, frame, P, C, f)
    nrm = X.dynamics_normals(seed, frame, P, d, f)
    u = X.resample_uniforms(seed, frame, P, f) if resample == "multinomial" else X.systematic_u0(seed, frame, f)
    r = O.step(om, T, pre["states"], pre["classes"], z, E, nrm, u, resample=resample, normals_by_particle=True)
    return r, u


@pytest.mark.parametrize("resample,P", [("multinomial", 100_000), ("systematic", 20_011)])
def test_philox_steps_vs_oracle(m2, om2, fx_config2, resample, P):
    """Config-2 model (N=2000, D=62, d=3, C=2): the benchmarked configuration's P = 100k
    with multinomial resampling, and systematic resampling (north_star) at an odd P;
    three resynced steps after one warm-up step (so particles share ancestors and the
    de-duplicated dynamics path is the one checked)."""
    from gpmdm_amd import GPMDM_PF
    T = np.asarray(fx_config2["T"], dtype=np.float64)
    seed = 11
    pf = GPMDM_PF(m2, torch.tensor(T), P, rng="philox", seed=seed, resample=resample)
    Y = m2.get_Y()
    pf.update(Y[10])
    for k in range(3):
        pre = pf.export_state()
        frame = pf.frame
        z = Y[11 + k] + 0.01
        pf.update(z)
        post = pf.export_state()
        r, u = _oracle_step(om2, T, pre, z, seed, frame, resample)
        assert_step_matches(post, r, pf.class_probabilities().numpy(), pf.current_state_mean().numpy(), u,
                            resample, (resample, k))
        assert abs(pf.log_likelihood() - r.lik) <= 1e-5 * abs(r.lik)
        assert pf.health() == {k2: 0 for k2 in pf.health()}


def test_bank_filters_vs_oracle(m2, om2, fx_config2):
    """every filter of a bank against the oracle with the Philox draws
    of its own key (seed + f): two resynced steps per filter."""
    from gpmdm_amd import GPMDM_PF_Bank
    T = np.asarray(fx_config2["T"], dtype=np.float64)
    F, P, seed = 4, 1500, 900
    bank = GPMDM_PF_Bank(m2, torch.tensor(T), F, P, seed=seed)
    Y = m2.get_Y()
    bank.update(np.stack([Y[100 * i] for i in range(F)]))
    for k in range(2):
        pre = bank.export_state()
        frame = bank.frame
        Z = np.stack([Y[100 * i + 1 + k] for i in range(F)])
        bank.update(Z)
        post = bank.export_state()
        gp, gm = bank.class_probabilities().numpy(), bank.current_state_mean().numpy()
        for f in range(F):
            pre_f = {key: pre[key][f] for key in ("states", "classes")}
            r, u = _oracle_step(om2, T, pre_f, Z[f], seed, frame, "multinomial", f=f)
            post_f = {key: post[key][f] for key in ("states", "classes", "w", "resample_idx")}
            assert_step_matches(post_f, r, gp[f], gm[f], u, "multinomial", (k, f))


def test_predict_device_vs_oracle(m2, om2, fx_config2):
    """GPMDM_PF.predict() (north_star): the mean over particles of each particle's class
    dynamics-GP mean, on the device, against the oracle's map_x_dynamics_for_class
    (gpmdm.py:1032-1068); the filter state is unchanged."""
    from gpmdm_amd import GPMDM_PF, GPMDM_PF_Bank
    T = np.asarray(fx_config2["T"], dtype=np.float64)
    Y = m2.get_Y()
    for P in (1, 777, 50_000):
        pf = GPMDM_PF(m2, torch.tensor(T), P, rng="philox", seed=5)
        for k in range(2):
            pf.update(Y[300 + k])
        st = pf.export_state()
        got = pf.predict().numpy()
        acc = np.zeros(m2.d)
        for c in range(2):
            sel = st["classes"] == c
            if sel.any():
                acc += om2.map_x_dynamics_for_class(st["states"][sel], c)[0].sum(0)
        assert nrel(got, acc / P) < 1e-9, P   # fp64 GP means; the oracle's BLAS threading varies by box
        st2 = pf.export_state()
        for key in ("states", "classes", "ll", "w", "resample_idx"):
            assert np.array_equal(st[key], st2[key]), key
        pf.update(Y[310])                         # the next step still runs normally
    bank = GPMDM_PF_Bank(m2, torch.tensor(T), 3, 400, seed=8)
    bank.update(np.stack([Y[1], Y[2], Y[3]]))
    st = bank.export_state()
    got = bank.predict().numpy()
    for f in range(3):
        acc = np.zeros(m2.d)
        for c in range(2):
            sel = st["classes"][f] == c
            if sel.any():
                acc += om2.map_x_dynamics_for_class(st["states"][f][sel], c)[0].sum(0)
        assert nrel(got[f], acc / 400) < 1e-9, f
