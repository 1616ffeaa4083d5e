"""Ancestor de-duplication of the dynamics GP (gpmdm_pf_set_dedup).

Offspring of one resampling ancestor hold bit-identical states, so the dynamics GP
(gpmdm.py:1032-1068) is evaluated once per distinct (ancestor, new class) key.  The bar is
bitwise identity with the undeduplicated path (every particle evaluated, as the
reference's _propogate_dynamics does, gpmdm_pf.py:153-168) for states, classes,
log-likelihoods and resample indices, frame after frame (for d <= 12 the default's wide
tiles without de-duplication are bitwise the narrow ones -- test_wide_dynamics_tiles_vs_narrow;
for d > 12 the 64 x 512 wide image differs from the narrow one in summation order, so the
identity tests pin both filters to one shape).
"""
import numpy as np
import pytest
import torch

from conftest import product_model

pytestmark = pytest.mark.gpu

KEYS = ("states", "classes", "ll", "resample_idx")


@pytest.fixture(scope="module")
def m2(fx_config2):
    return product_model(fx_config2)


def _pair(m, T, P, frames, zs, **kw):
    from gpmdm_amd import GPMDM_PF
    pfs = []
    for dd in (True, False):
        torch.manual_seed(5)
        pfs.append(GPMDM_PF(m, T, P, dedup=dd, dyn_tiles="narrow", **kw))
    rows = []
    for k in range(frames):
        st = torch.get_rng_state()          # replay mode: both filters see the same draws
        for pf in pfs:
            torch.set_rng_state(st)
            pf.update(zs[k])
        a, b = pfs[0].export_state(), pfs[1].export_state()
        for key in KEYS:
            assert np.array_equal(a[key], b[key]), (k, key)
        assert np.array_equal(pfs[0].class_probabilities().numpy(), pfs[1].class_probabilities().numpy())
        assert np.array_equal(pfs[0].current_state_mean().numpy(), pfs[1].current_state_mean().numpy())
        rows.append((pfs[0].dynamics_rows(), pfs[1].dynamics_rows()))
    return rows


@pytest.mark.parametrize("resample", ["multinomial", "systematic"])
def test_dedup_bitwise_philox_config2(m2, resample):
    T = torch.tensor([[0.9, 0.1], [0.1, 0.9]])
    Y = m2.get_Y()
    P = 20_000
    rows = _pair(m2, T, P, 5, [Y[30 + k] for k in range(5)], rng="philox", seed=99, resample=resample)
    assert rows[0] == (P, P)                       # first frame after init: no shared ancestors
    assert all(r[1] == P for r in rows)
    assert all(r[0] < P for r in rows[1:]), rows   # later frames share ancestors


def test_dedup_bitwise_replay_config1(fx_config1):
    m = product_model(fx_config1)
    f = fx_config1
    _pair(m, torch.tensor(f["T"]), 3000, 6, list(f["z"][:6]), rng="torch")


def test_dedup_bitwise_sharded_and_many_classes():
    """Two shards on one GPU (uneven split) with C = 5: the leader of a key is the slice's
    own smallest particle index, so each shard de-duplicates independently."""
    from conftest import synthetic_model
    from gpmdm_amd import GPMDM_PF
    m, T, Y = synthetic_model(C=5, d=4, D=12, L=30)
    P = 7001
    outs = []
    for dd in (True, False):
        pfs = []
        for shard in ((2, 0), (2, 1)):
            torch.manual_seed(3)
            pfs.append(GPMDM_PF(m, T, P, rng="philox", seed=5, shard=shard, dedup=dd, dyn_tiles="narrow"))
        hist = []
        for k in range(4):
            sends = [pf._stage_propagate(Y[k]) for pf in pfs]
            full = torch.cat(sends, 0)
            for pf in pfs:
                pf._recv.copy_(full)
                pf._stage_resample()
            hist.append(pfs[0].export_state())
            assert np.array_equal(hist[-1]["states"], pfs[1].export_state()["states"])
        outs.append(hist)
    for a, b in zip(*outs):
        for key in KEYS:
            assert np.array_equal(a[key], b[key]), key


def test_dedup_bank(m2):
    from gpmdm_amd import GPMDM_PF_Bank
    T = torch.tensor([[0.9, 0.1], [0.1, 0.9]])
    Y = m2.get_Y()
    banks = [GPMDM_PF_Bank(m2, T, 3, 2000, seed=8, dedup=dd, dyn_tiles="narrow") for dd in (True, False)]
    for k in range(4):
        z = np.stack([Y[10 + k], Y[200 + k], Y[400 + k]])
        for b in banks:
            b.update(z)
        assert np.array_equal(banks[0].class_probabilities().numpy(), banks[1].class_probabilities().numpy())
        assert np.array_equal(banks[0].current_state_mean().numpy(), banks[1].current_state_mean().numpy())


def test_wide_dynamics_tiles_vs_narrow(m2, fx_config2):
    """dedup=False runs the dynamics GP on the wide (observation-GP-shaped) tile image by
    default: one resynced step from the same particles and draws as the narrow tiles and as
    the oracle -- bitwise the narrow path (the 32 x 512 kernel reduces each 256-column half
    of its blocks in the 16 x 256 order, gp_tile.h), everything against the oracle at the
    parity tolerances."""
    from conftest import assert_step_matches, oracle_model
    from gpmdm_amd import GPMDM_PF
    from oracle import gpmdm_oracle as O
    T = np.array([[0.9, 0.1], [0.1, 0.9]])
    P = 30_000
    rng = np.random.RandomState(17)
    om = oracle_model(fx_config2)
    Y = m2.get_Y()
    torch.manual_seed(2)
    warm = GPMDM_PF(m2, torch.tensor(T), P, rng="torch")
    warm.update(Y[30])
    st0 = warm.export_state()
    E, nrm, u = rng.exponential(size=(P, 2)), rng.randn(P, m2.d), rng.rand(P)
    out = {}
    for tiles in ("narrow", "wide"):
        pf = GPMDM_PF(m2, torch.tensor(T), P, rng="torch", dedup=False, dyn_tiles=tiles)
        pf.load_state(st0["states"], st0["classes"])
        pf.update_with_draws(Y[31], E, nrm, u)
        out[tiles] = (pf.export_state(), pf.class_probabilities().numpy(), pf.current_state_mean().numpy())
    a, b = out["narrow"][0], out["wide"][0]
    for key in ("states", "classes", "ll", "w", "resample_idx"):
        assert np.array_equal(a[key], b[key]), key
    assert np.array_equal(out["narrow"][1], out["wide"][1]) and np.array_equal(out["narrow"][2], out["wide"][2])
    r = O.step(om, T, st0["states"], st0["classes"], Y[31], E, nrm, u)
    assert_step_matches(b, r, out["wide"][1], out["wide"][2], u, what="wide")
