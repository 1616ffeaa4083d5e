"""GPU: lifecycle calls wait for their own filter's work, not for the device.

A filter's create / init / import / rebind / destroy used to synchronise the whole device
(hipDeviceSynchronize; and hipFree / hipHostFree themselves wait for every stream of the
device: tools/microbench/sync_probe.hip).  They now wait for the handle's own pre-switch,
read-out number and side streams (capi_pf.hip quiesce), run their copies and read-out
launches on the library's lifecycle stream, and release memory in that stream's order from a
stream-ordered pool and a pinned-buffer cache (memory.hip).

The test keeps a filter bank stepping on a stream of its own (several frames queued, tens of
ms each) and, while that stream is busy, creates, initialises, imports, rebinds and destroys
another filter on the default stream: after every one of those calls the bank's stream must
still be busy (the call did not wait for it), and the bank's read-outs and final state must
be bitwise those of an undisturbed run (gpmdm_pf.py:78-115, 224-262)."""
import ctypes

import numpy as np
import pytest
import torch

from conftest import product_model

pytestmark = pytest.mark.gpu

F, PB, FRAMES = 64, 8000, 7


@pytest.fixture(scope="module")
def models(fx_config2):
    return product_model(fx_config2), product_model(fx_config2)


def _bank_run(m, T, zs, disturb=None):
    """Step the bank on its own stream; ``disturb(k)`` runs on the default stream after frame
    k was queued and returns the bank stream's business after each of its calls."""
    from gpmdm_amd import GPMDM_PF_Bank
    bank = GPMDM_PF_Bank(m, T, F, PB, seed=5)
    sb = torch.cuda.Stream()
    busy = []
    out = []
    for k in range(FRAMES):
        with torch.cuda.stream(sb):
            bank.update(zs[k])
        if disturb is not None:
            busy += disturb(k, sb)
        with torch.cuda.stream(sb):
            if k == FRAMES - 1 or disturb is None:
                out.append((bank.class_probabilities().numpy().copy(), bank.current_state_mean().numpy().copy()))
    with torch.cuda.stream(sb):
        st = bank.export_state()
    return out, st, busy


def test_lifecycle_calls_do_not_wait_for_another_filters_stream(models):
    from gpmdm_amd import GPMDM_PF, _lib
    m, m_other = models
    T = torch.tensor([[0.9, 0.1], [0.1, 0.9]], dtype=torch.float64)
    Y = m.get_Y()
    zs = [np.repeat(np.asarray(Y[40 + 3 * k], dtype=np.float64)[None, :] + 0.01, F, axis=0) for k in range(FRAMES)]
    lib = _lib.load()
    holder = {}

    def disturb(k, sb):
        """One lifecycle call per frame, made while the bank's stream is busy; returns
        (call, bank stream busy before, busy after)."""
        before = not sb.query()
        if k == 1:
            what = "create + init"
            holder["pf"] = GPMDM_PF(m, T, 5000, rng="philox", seed=3)
        elif k == 2:
            what = "init (reset)"
            holder["pf"].reset()
        elif k == 3:
            what = "import (load_state with weights)"
            P = 5000
            st = holder["st"]
            holder["pf"].load_state(st["states"], st["classes"], ll=st["ll"], log_w=st["log_w"], w=st["w"],
                                    resample_idx=st["resample_idx"], frame=st["frame"])
        elif k == 4:
            what = "rebind (gpmdm_pf_set_model)"
            _lib.check(lib.gpmdm_pf_set_model(holder["pf"]._h, m_other.handle), "set_model")
        elif k == 5:
            what = "destroy"
            pf = holder.pop("pf")
            h = pf._h
            pf._h = None                         # (the wrapper's __del__ must not destroy it again)
            _lib.check(lib.gpmdm_pf_destroy(h), "destroy")
        else:
            return []
        after = not sb.query()
        return [(what, before, after)]

    ref_out, ref_st, _ = _bank_run(m, T, zs)
    # a state to import, made before the bank runs (export synchronises its own stream only)
    pf0 = GPMDM_PF(m, T, 5000, rng="philox", seed=3)
    pf0.update(np.asarray(Y[10], dtype=np.float64))
    holder["st"] = pf0.export_state()
    torch.cuda.synchronize()
    out, st, busy = _bank_run(m, T, zs, disturb)
    assert len(busy) == 5, busy
    for what, before, after in busy:
        assert before, f"the bank's stream was idle before {what}: the check would be vacuous"
        assert after, f"{what} waited for the bank's stream (device-wide synchronisation)"
    p1, mu1 = ref_out[-1]
    p2, mu2 = out[-1]
    assert np.array_equal(p1, p2) and np.array_equal(mu1, mu2)
    for key in ("states", "classes", "ll", "w", "resample_idx"):
        assert np.array_equal(ref_st[key], st[key]), key


def test_lifecycle_filter_still_correct_after_scoped_waits(models):
    """The same calls on a filter of their own: init's read-outs are the reference's initial
    ones (w = 1/P), an import's read-outs equal the exporter's, a rebind to an identical model
    keeps the trajectory bitwise, and destroying a filter whose pre-switch is pending is clean."""
    from gpmdm_amd import GPMDM_PF, _lib
    m, m_other = models
    T = torch.tensor([[0.9, 0.1], [0.1, 0.9]], dtype=torch.float64)
    Y = m.get_Y()
    torch.manual_seed(9)                 # (the initial cloud comes from torch's generator)
    a = GPMDM_PF(m, T, 20_000, rng="philox", seed=9)
    torch.manual_seed(9)
    b = GPMDM_PF(m, T, 20_000, rng="philox", seed=9)
    for k in range(3):
        a.update(Y[20 + k])
        b.update(Y[20 + k])
    _lib.check(_lib.load().gpmdm_pf_set_model(b._h, m_other.handle), "set_model")   # identical model
    st = a.export_state()
    c = GPMDM_PF(m, T, 20_000, rng="philox", seed=9)
    c.load_state(st["states"], st["classes"], ll=st["ll"], log_w=st["log_w"], w=st["w"],
                 resample_idx=st["resample_idx"], frame=st["frame"])
    assert np.array_equal(a.class_probabilities().numpy(), c.class_probabilities().numpy())
    for k in range(3, 6):
        for pf in (a, b, c):
            pf.update(Y[20 + k])
        ra, rb, rc = (pf.export_state() for pf in (a, b, c))
        for key in ("states", "classes", "ll", "resample_idx"):
            assert np.array_equal(ra[key], rb[key]), (k, key, "rebind")
            assert np.array_equal(ra[key], rc[key]), (k, key, "import")
    # a pending Philox pre-switch (launched behind the last read-out) at destroy
    h = a._h
    a._h = None
    _lib.check(_lib.load().gpmdm_pf_destroy(h), "destroy")
    d = GPMDM_PF(m, T, 1000, rng="philox", seed=1)
    d.reset()
    post = d.class_probabilities().numpy()
    assert np.isclose(post.sum(), 1.0)
