"""GPU: the one-launch paths of small filters (pf_kernels.hip: k_small_switch -- switch, class
scan, grouping, leader compaction -- for P <= 1024 particles on one shard, k_small_resample
-- normalise, resample, read-out -- for P <= 1024 per filter) are bitwise the multi-kernel
path (GPMDM_NO_SMALL_PATH=1), the observation GP's 16-row tiles (capi_model.hip obs_pick)
are bitwise its 32-row tiles, and a small replay filter's class counts computed on the host
(no mid-frame sync) are the device's (GPMDM_NO_HOST_COUNTS=1), and a Philox filter whose
next switch the resample launches ahead (pre-switch) is bitwise one that switches in the next
update (GPMDM_NO_PRESWITCH=1), and de-duplicated dynamics passes on the wide image
(GPMDM_DYN_WIDE_ROWS=0), with predict / dynamics_rows / export between frames: replay and Philox draws, multinomial and systematic
resampling, with and without ancestor de-duplication, a bank of filters, several frames.
The environment switches are read once per process, so each configuration runs in its own
child process (one at a time)."""
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
CHILD = r'''
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[2]); sys.path.insert(0, sys.argv[2] + "/tests")
from conftest import load_fixture, product_model
from gpmdm_amd import GPMDM_PF, GPMDM_PF_Bank
f = load_fixture("config2_n2000_p1000")
m = product_model(f)
T = torch.tensor(np.asarray(f["T"], dtype=np.float64))
Y = m.get_Y()
out = {}
for name, P, rng, res, dd in (("replay100", 100, "torch", "multinomial", True),
                              ("philox1000", 1000, "philox", "multinomial", True),
                              ("nodedup1000", 1000, "philox", "multinomial", False),
                              ("sys777", 777, "philox", "systematic", True),
                              ("one", 1, "philox", "multinomial", True),
                              ("big1500", 1500, "philox", "multinomial", True),
                              ("philox20k", 20000, "philox", "multinomial", True),
                              ("replay1024sys", 1024, "torch", "systematic", True),
                              ("replay1025", 1025, "torch", "multinomial", True)):
    torch.manual_seed(3)
    pf = GPMDM_PF(m, T, P, rng=rng, seed=9 if rng == "philox" else None, resample=res, dedup=dd)
    for k in range(4):
        pf.update(Y[50 + 9 * k] + 0.01)
        if k == 1:                           # between frames: drops a pre-switch (capi_pf.hip drop_preswitch)
            out[f"{name}_{k}_pred"] = pf.predict().numpy()
        out[f"{name}_{k}_post"] = pf.class_probabilities().numpy()
        out[f"{name}_{k}_mean"] = pf.current_state_mean().numpy()
        out[f"{name}_{k}_lik"] = np.array([pf.log_likelihood()])
        out[f"{name}_{k}_rows"] = np.array([pf.dynamics_rows()])
    st = pf.export_state()
    for key in ("states", "classes", "ll", "w", "resample_idx"):
        out[f"{name}_{key}"] = st[key]
# replay updates with no read-out between them: the host class counts wait for the
# previous resample themselves (capi_internal.h gpmdm_pf::cls_ev)
torch.manual_seed(4)
pf = GPMDM_PF(m, T, 300, rng="torch")
for k in range(5):
    pf.update(Y[70 + 3 * k] + 0.01)
out["unread_post"] = pf.class_probabilities().numpy()
out["unread_states"] = pf.export_state()["states"]
bank = GPMDM_PF_Bank(m, T, 3, 300, seed=5)
for k in range(3):
    bank.update(np.stack([Y[10 * i + k] for i in range(3)]))
out["bank_post"] = bank.class_probabilities().numpy()
out["bank_states"] = bank.export_state()["states"]
np.savez(sys.argv[1], **out)
'''


def _run(tmp_path, tag, env_extra):
    env = dict(os.environ, **env_extra)
    path = tmp_path / f"{tag}.npz"
    r = subprocess.run([sys.executable, "-c", CHILD, str(path), str(ROOT)], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return dict(np.load(path))


@pytest.mark.timeout(600)
def test_small_path_is_bitwise_the_multi_kernel_path(tmp_path):
    """Default (fused small-filter kernels, 16-row observation tiles for small shards) vs
    neither, vs 16-row observation tiles for every filter size."""
    fused = _run(tmp_path, "fused", {})
    multi = _run(tmp_path, "multi", {"GPMDM_NO_SMALL_PATH": "1", "GPMDM_OBS_SMALL_TILES": "0"})
    tiles16 = _run(tmp_path, "tiles16", {"GPMDM_OBS_SMALL_TILES": "1"})
    # replay filters' class counts from the device with a mid-frame sync, not the host
    devcounts = _run(tmp_path, "devcounts", {"GPMDM_NO_HOST_COUNTS": "1"})
    # Philox filters' next switch launched by the resample (pre-switch) or by the next update
    nopre = _run(tmp_path, "nopre", {"GPMDM_NO_PRESWITCH": "1"})
    # de-duplicated dynamics passes on the wide 32 x 512 image every frame instead of the
    # narrow 16 x 256 one (capi_frame.hip dyn_frame_wide: the two are bitwise the same at d <= 12)
    widedyn = _run(tmp_path, "widedyn", {"GPMDM_DYN_WIDE_ROWS": "0"})
    assert fused.keys() == multi.keys() == tiles16.keys() == devcounts.keys() == nopre.keys() == widedyn.keys()
    for k in fused:
        assert np.array_equal(fused[k], multi[k]), k
        assert np.array_equal(fused[k], tiles16[k]), k
        assert np.array_equal(fused[k], devcounts[k]), k
        assert np.array_equal(fused[k], nopre[k]), k
        assert np.array_equal(fused[k], widedyn[k]), k


def test_deferred_likelihood_is_flushed_for_an_early_reader():
    """A single-shard small filter defers its likelihood finish into the resampling launch
    (capi_frame.hip weigh / capi_pf.hip flush_ll): an export between propagate and resample must still see
    the finished ll, and the frame must end bitwise as an uninterrupted update."""
    import torch
    from conftest import load_fixture, product_model
    from gpmdm_amd import GPMDM_PF, _lib
    f = load_fixture("config2_n2000_p1000")
    m = product_model(f)
    T = torch.tensor(np.asarray(f["T"], dtype=np.float64))
    Y = m.get_Y()
    torch.manual_seed(5)                      # the initial particles come from torch's generator
    a = GPMDM_PF(m, T, 300, rng="philox", seed=4)
    torch.manual_seed(5)
    b = GPMDM_PF(m, T, 300, rng="philox", seed=4)
    lib = _lib.load()
    for k in range(3):
        z = np.ascontiguousarray(np.asarray(Y[70 + 11 * k], dtype=np.float64) + 0.02)
        a.update(z)
        s = b._stream()
        _lib.check(lib.gpmdm_pf_switch(b._h, None, None, s), "switch")
        _lib.check(lib.gpmdm_pf_propagate(b._h, _lib.dptr(z), None, s), "propagate")
        mid = b.export_state()                # reads ll before the resampling launch
        _lib.check(lib.gpmdm_pf_resample(b._h, None, s), "resample")
        b._readout = None
        ea, eb = a.export_state(), b.export_state()
        assert np.array_equal(mid["ll"], ea["ll"])
        for key in ("states", "classes", "ll", "w", "resample_idx"):
            assert np.array_equal(ea[key], eb[key]), key
        assert np.array_equal(a.class_probabilities().numpy(), b.class_probabilities().numpy())
        assert np.array_equal(a.current_state_mean().numpy(), b.current_state_mean().numpy())


CHILD_IMAGE16 = r'''
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[2]); sys.path.insert(0, sys.argv[2] + "/tests")
from conftest import load_fixture, product_model
from gpmdm_amd import GPMDM_PF, GPMDM_PF_Bank
f = load_fixture("config1_n500_p100_f200")
m = product_model(f)
T = torch.tensor(np.asarray(f["T"], dtype=np.float64))
Y = m.get_Y()
out = {}
for name, P, rng in (("replay100", 100, "torch"), ("philox1000", 1000, "philox")):
    torch.manual_seed(3)
    pf = GPMDM_PF(m, T, P, rng=rng, seed=9 if rng == "philox" else None)
    for k in range(6):
        pf.update(Y[40 + 7 * k] + 0.01)
        out[f"{name}_{k}_post"] = pf.class_probabilities().numpy()
        out[f"{name}_{k}_mean"] = pf.current_state_mean().numpy()
    st = pf.export_state()
    for key in ("states", "classes", "ll", "resample_idx"):
        out[f"{name}_{key}"] = st[key]
bank = GPMDM_PF_Bank(m, T, 5, 100, seed=5)
for k in range(4):
    bank.update(np.stack([Y[10 * i + k] for i in range(5)]))
out["bank_post"] = bank.class_probabilities().numpy()
out["bank_states"] = bank.export_state()["states"]
np.savez(sys.argv[1], **out)
'''


@pytest.mark.timeout(600)
def test_small_observation_image_matches_the_default_image(tmp_path):
    """Small models and filters run the observation GP over a 16 x 256 image (capi_model.hip
    obs_pick): its column blocks partition the sums differently, so the filter agrees with
    the 32 x 512 image to rounding (not bit for bit) -- same classes and resampling
    indices, states and read-outs to 1e-9 -- on the config-1 model (N = 500)."""
    def run(tag, env_extra):
        env = dict(os.environ, **env_extra)
        path = tmp_path / f"{tag}.npz"
        r = subprocess.run([sys.executable, "-c", CHILD_IMAGE16, str(path), str(ROOT)], env=env,
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        return dict(np.load(path))
    small = run("image16", {})
    default = run("image32", {"GPMDM_OBS_IMAGE16": "0"})
    assert small.keys() == default.keys()
    for k in small:
        if k.endswith(("classes", "resample_idx")):
            assert np.array_equal(small[k], default[k]), k
        elif k.endswith("_ll"):
            np.testing.assert_allclose(small[k], default[k], rtol=1e-9, atol=1e-9, err_msg=k)
        else:
            np.testing.assert_allclose(small[k], default[k], rtol=1e-9, atol=1e-12, err_msg=k)
