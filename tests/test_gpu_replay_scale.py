"""GPU: the drop-in default (rng='torch': the reference's draws from torch's global
generator, gpmdm_pf.py:137-213) at the headline's particle count.

From 16384 particles the filter draws torch's streams as parallel chunks of torch's own
samplers (replay.ParallelFrameDraws, placed by gpmdm_rng_walk), the next frame's switch
draws and first-class normals ahead on a background thread.  It must be bit for bit the
serial draws: the same filter with the serial FrameDraws takes the same classes, counts,
states and read-outs over several frames, and leaves torch's generator in the same state;
one step against the oracle with the draws it consumed checks the device side."""
import numpy as np
import pytest
import torch

from conftest import assert_step_matches, load_fixture, oracle_model, product_model

pytestmark = pytest.mark.gpu

P = 100_000


@pytest.fixture(scope="module")
def model():
    f = load_fixture("config2_n2000_p1000")
    return f, product_model(f), torch.tensor(np.asarray(f["T"], dtype=np.float64))


def _frames(pf, Y, n, between=None):
    outs = []
    for k in range(n):
        pf.update(np.asarray(Y[60 + 7 * k], dtype=np.float64) + 0.01)
        outs.append((pf.class_probabilities().numpy(), pf.current_state_mean().numpy(), pf._counts.copy(),
                     torch.get_rng_state().clone()))
        if between is not None and k == 1:
            between()
    return outs, pf.export_state()


@pytest.mark.parametrize("interleave", [False, True])
def test_parallel_replay_is_the_serial_replay(model, monkeypatch, interleave):
    from gpmdm_amd import GPMDM_PF, replay
    from gpmdm_amd import pf as pfmod
    f, m, T = model
    Y = m.get_Y()
    between = (lambda: torch.randn(5)) if interleave else None   # a user's own draw between frames
    torch.manual_seed(17)
    par = GPMDM_PF(m, T, P)
    a, sa = _frames(par, Y, 4, between)
    assert isinstance(par._draws, replay.ParallelFrameDraws)
    assert par._draws.prefetch_hits >= (1 if interleave else 3)
    monkeypatch.setattr(pfmod, "PARALLEL_REPLAY_P", 10 ** 12)
    torch.manual_seed(17)
    ser = GPMDM_PF(m, T, P)
    b, sb = _frames(ser, Y, 4, between)
    assert isinstance(ser._draws, replay.FrameDraws)
    for k, (x, y) in enumerate(zip(a, b)):
        assert np.array_equal(x[2], y[2]), (k, "class counts")
        assert np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]), (k, "read-outs")
        assert torch.equal(x[3], y[3]), (k, "torch generator state after the frame")
    for key in ("states", "classes", "ll", "w", "resample_idx"):
        assert np.array_equal(sa[key], sb[key]), key


def test_parallel_replay_step_vs_oracle(model):
    """One resynced step at P = 100k: the device consumes the parallel draws as the oracle
    consumes them (weights, resample indices, states, read-outs)."""
    from gpmdm_amd import GPMDM_PF
    from oracle import gpmdm_oracle as O
    f, m, T = model
    Y = m.get_Y()
    om = oracle_model(f)
    torch.manual_seed(23)
    pf = GPMDM_PF(m, T, P)
    pf.update(np.asarray(Y[30], dtype=np.float64) + 0.01)
    pf._draws.record = True                 # copies of the frame's draws (E and N are refilled ahead)
    pre = pf.export_state()
    z = np.asarray(Y[31], dtype=np.float64) + 0.01
    pf.update(z)
    dr = pf._draws
    post = pf.export_state()
    r = O.step(om, f["T"], pre["states"], pre["classes"], z, dr.last_E, dr.last_N, dr.last_U)
    assert np.array_equal(r.classes_switched, O.switch_classes(pre["classes"], f["T"], dr.last_E))
    counts = np.bincount(r.classes_switched, minlength=T.shape[0])
    assert np.array_equal(counts, pf._counts)             # the device's counts are the oracle's
    assert_step_matches(post, r, pf.class_probabilities().numpy(), pf.current_state_mean().numpy(), dr.last_U,
                        what="replay P=100k")


def test_replay_preswitch_consumed_replaced_or_dropped(model, monkeypatch):
    """gpmdm_pf_preswitch (replay filters with the draws made ahead): the next switch consumes
    it when handed the same E pointer; a second pre-switch replaces it; another E pointer
    drops it (the switch starts from scratch); predict / export between frames drop it; the
    normals staged ahead (gpmdm_pf_stage_normals) are used only for the pointer they were
    staged from -- every way bitwise the filter that never pre-switches or stages
    (GPMDM_NO_PRESWITCH=1)."""
    from gpmdm_amd import GPMDM_PF, _lib
    f, m, T = model
    Y = m.get_Y()
    lib = _lib.load()

    def run(mode):
        torch.manual_seed(29)
        pf = GPMDM_PF(m, T, 20000)
        outs = []
        for k in range(6):
            z = np.ascontiguousarray(np.asarray(Y[80 + 5 * k], dtype=np.float64) + 0.01)
            if mode == "poke" and k == 4:
                # this frame by hand, with a copy of the E the pre-switch was given
                h, s = pf._h, pf._stream()
                dr = pf._draws
                pE, pC, pN, pU = pf._draw_ptr
                dr.switch()
                E2 = dr.E.copy()
                _lib.check(lib.gpmdm_pf_switch(h, _lib.dptr(E2), pC, s), "switch")
                dr.dynamics(pf._counts)
                N2 = dr.N.copy()               # another normals pointer: the staged copy is not used
                pf._propagate(z, N2, s, _lib.dptr(N2))
                pf._n_staged = False
                dr.resample()
                _lib.check(lib.gpmdm_pf_resample(h, pU, s), "resample")
                pf._readout = None
                pf._pre_sw = False
            else:
                pf.update(z)
            outs.append((pf.class_probabilities().numpy(), pf.current_state_mean().numpy(), pf._counts.copy()))
            if mode == "poke":
                if k == 0:                 # replaced by a second pre-switch of the same draws
                    _lib.check(lib.gpmdm_pf_preswitch(pf._h, pf._draw_ptr[0], pf._stream()), "preswitch")
                elif k == 1:
                    outs.append((pf.predict().numpy(),))
                elif k == 2:
                    outs.append((pf.export_state()["states"],))
            elif mode == "nopre" and k in (1, 2):
                outs.append((pf.predict().numpy(),) if k == 1 else (pf.export_state()["states"],))
        assert pf._draws.prefetch_hits >= 4
        st = pf.export_state()
        return outs, st, torch.get_rng_state().clone()

    a = run("poke")
    monkeypatch.setenv("GPMDM_NO_PRESWITCH", "1")
    b = run("nopre")
    assert len(a[0]) == len(b[0])
    for k, (x, y) in enumerate(zip(a[0], b[0])):
        for u, v in zip(x, y):
            assert np.array_equal(u, v), k
    for key in ("states", "classes", "ll", "w", "resample_idx"):
        assert np.array_equal(a[1][key], b[1][key]), key
    assert torch.equal(a[2], b[2])


def test_preswitch_and_staging_contract(model):
    """gpmdm_pf_preswitch / gpmdm_pf_stage_normals: a Philox filter's explicit pre-switch is
    the one its resample launched (no-op, bitwise); inside a step both calls are refused;
    a bad normals range is a ValueError; a Philox filter has no normals to stage."""
    from gpmdm_amd import GPMDM_PF, _lib
    f, m, T = model
    Y = m.get_Y()
    lib = _lib.load()
    outs = []
    for poke in (False, True):
        torch.manual_seed(31)
        pf = GPMDM_PF(m, T, 5000, rng="philox", seed=3)
        for k in range(3):
            pf.update(np.asarray(Y[40 + k], dtype=np.float64) + 0.01)
            if poke:
                _lib.check(lib.gpmdm_pf_preswitch(pf._h, None, pf._stream()), "preswitch")
        outs.append((pf.class_probabilities().numpy(), pf.export_state()["states"]))
        with pytest.raises(RuntimeError):
            _lib.check(lib.gpmdm_pf_stage_normals(pf._h, None, 0, 1, pf._stream()), "stage")
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    torch.manual_seed(32)
    pf = GPMDM_PF(m, T, 20000)
    z = np.ascontiguousarray(np.asarray(Y[50], dtype=np.float64) + 0.01)
    pf.update(z)
    pN = pf._draw_ptr[2]
    with pytest.raises(ValueError):
        _lib.check(lib.gpmdm_pf_stage_normals(pf._h, pN, 0, 20000 * m.d + 1, pf._stream()), "stage")
    with pytest.raises(ValueError):
        _lib.check(lib.gpmdm_pf_stage_normals(pf._h, pN, 5, 4, pf._stream()), "stage")
    # inside a step: after the switch, before the propagate
    s = pf._stream()
    dr = pf._draws
    dr.switch()
    if pf._pre_sw and not dr.last_hit:
        _lib.check(lib.gpmdm_pf_preswitch(pf._h, pf._draw_ptr[0], s), "preswitch")
    _lib.check(lib.gpmdm_pf_switch(pf._h, pf._draw_ptr[0], pf._draw_ptr[1], s), "switch")
    with pytest.raises(RuntimeError):
        _lib.check(lib.gpmdm_pf_preswitch(pf._h, pf._draw_ptr[0], s), "preswitch")
    # the step completes as usual
    dr.dynamics(pf._counts)
    N2 = dr.N.copy()                       # (not the staged pointer: copied in full)
    pf._propagate(z, N2, s, _lib.dptr(N2))
    dr.resample()
    _lib.check(lib.gpmdm_pf_resample(pf._h, pf._draw_ptr[3], s), "resample")
    pf._readout = None
    pf._pre_sw = pf._n_staged = False
    assert np.isfinite(pf.class_probabilities().numpy()).all()


@pytest.mark.parametrize("resample,dedup", [("systematic", True), ("multinomial", False)])
def test_replay_preswitch_other_modes(model, monkeypatch, resample, dedup):
    """The replay pre-switch and staged normals with systematic resampling (one uniform per
    frame) and without ancestor de-duplication (every particle a dynamics row): bitwise the
    filter that switches in each update (GPMDM_NO_PRESWITCH=1)."""
    from gpmdm_amd import GPMDM_PF
    f, m, T = model
    Y = m.get_Y()

    def run():
        torch.manual_seed(37)
        pf = GPMDM_PF(m, T, 20000, resample=resample, dedup=dedup)
        outs = []
        for k in range(4):
            pf.update(np.asarray(Y[90 + 4 * k], dtype=np.float64) + 0.01)
            outs.append((pf.class_probabilities().numpy(), pf.current_state_mean().numpy()))
        return outs, pf.export_state(), torch.get_rng_state().clone()

    a = run()
    monkeypatch.setenv("GPMDM_NO_PRESWITCH", "1")
    b = run()
    for x, y in zip(a[0], b[0]):
        assert np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1])
    for key in ("states", "classes", "ll", "w", "resample_idx"):
        assert np.array_equal(a[1][key], b[1][key]), key
    assert torch.equal(a[2], b[2])
