"""GPU: particle-filter checkpoint / resume (gpmdm_pf_import).

The reference filter's state is _particle_states, _particle_classes, _log_likelihoods,
_log_weights, _weights (gpmdm_pf.py:78-82, 100-104).  A filter run 5 frames, exported,
imported into a fresh filter of the same configuration and run 5 more frames must be
bitwise the filter run 10 frames uninterrupted, and its read-outs right after the import
must be the exporter's -- Philox and replay draws, multinomial and systematic
resampling, a small (one-launch) and a large (multi-kernel) particle count, and a bank."""
import numpy as np
import pytest
import torch

from conftest import load_fixture, product_model

pytestmark = pytest.mark.gpu

KEYS = ("states", "classes", "ll", "log_w", "w", "resample_idx")


@pytest.fixture(scope="module")
def model():
    f = load_fixture("config2_n2000_p1000")
    m = product_model(f)
    return m, torch.tensor(np.asarray(f["T"], dtype=np.float64)), m.get_Y()


def _z(Y, k):
    return np.ascontiguousarray(np.asarray(Y[40 + 13 * k], dtype=np.float64) + 0.01)


def _readouts(pf):
    return pf.class_probabilities().numpy(), pf.current_state_mean().numpy(), pf.log_likelihood()


@pytest.mark.parametrize("P", [777, 3001])
@pytest.mark.parametrize("rng", ["philox", "torch"])
@pytest.mark.parametrize("resample", ["multinomial", "systematic"])
def test_export_import_resumes_bitwise(model, P, rng, resample):
    from gpmdm_amd import GPMDM_PF
    m, T, Y = model
    seed = 21 if rng == "philox" else None
    torch.manual_seed(7)
    a = GPMDM_PF(m, T, P, rng=rng, seed=seed, resample=resample)
    for k in range(5):
        a.update(_z(Y, k))
    st = a.export_state()
    ro = _readouts(a)
    rng_state = torch.get_rng_state()        # a replay filter's generator is the caller's state
    for k in range(5, 10):
        a.update(_z(Y, k))
    ref, ref_ro = a.export_state(), _readouts(a)

    torch.manual_seed(12345)                 # a fresh filter whose own init draws differ
    b = GPMDM_PF(m, T, P, rng=rng, seed=seed, resample=resample)
    b.import_state(st)
    got = _readouts(b)
    assert np.array_equal(got[0], ro[0]) and np.array_equal(got[1], ro[1]) and got[2] == ro[2]
    st_b = b.export_state()
    for key in KEYS:
        assert np.array_equal(st_b[key], st[key]), key
    assert b.frame == st["frame"] == 5
    torch.set_rng_state(rng_state)
    for k in range(5, 10):
        b.update(_z(Y, k))
    out, out_ro = b.export_state(), _readouts(b)
    for key in KEYS:
        assert np.array_equal(out[key], ref[key]), key
    assert np.array_equal(out_ro[0], ref_ro[0]) and np.array_equal(out_ro[1], ref_ro[1]) and out_ro[2] == ref_ro[2]


def test_bank_export_import_resumes_bitwise(model):
    from gpmdm_amd import GPMDM_PF_Bank
    m, T, Y = model
    a = GPMDM_PF_Bank(m, T, 4, 500, seed=3)
    Z = lambda k: np.stack([_z(Y, k + 3 * i) for i in range(4)])  # noqa: E731
    for k in range(4):
        a.update(Z(k))
    st = a.export_state()
    ro = (a.class_probabilities().numpy(), a.current_state_mean().numpy())
    for k in range(4, 8):
        a.update(Z(k))
    ref = a.export_state()
    b = GPMDM_PF_Bank(m, T, 4, 500, seed=3)
    b.update(Z(9))                           # a filter mid-run: the import replaces its state
    b.import_state(st)
    assert np.array_equal(b.class_probabilities().numpy(), ro[0])
    assert np.array_equal(b.current_state_mean().numpy(), ro[1])
    for k in range(4, 8):
        b.update(Z(k))
    out = b.export_state()
    for key in KEYS:
        assert np.array_equal(out[key], ref[key]), key


def test_import_rejects_inconsistent_state(model):
    from gpmdm_amd import GPMDM_PF
    m, T, Y = model
    torch.manual_seed(1)
    a = GPMDM_PF(m, T, 300, rng="philox", seed=2)
    a.update(_z(Y, 0))
    st = a.export_state()
    bad = dict(st, log_w=st["log_w"] + 1e-9)
    with pytest.raises(ValueError, match="log_w"):
        a.import_state(bad)
    with pytest.raises(ValueError, match="seed"):
        GPMDM_PF(m, T, 300, rng="philox", seed=3).import_state(st)
    with pytest.raises(ValueError):
        a.import_state(dict(st, resample_idx=np.full(300, 300, dtype=np.int64)))
    with pytest.raises(ValueError):
        a.load_state(st["states"], st["classes"], ll=st["ll"])
    # after a rejected import the filter still steps
    a.update(_z(Y, 1))
    assert np.isfinite(a.class_probabilities().numpy()).all()
