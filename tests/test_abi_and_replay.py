"""CPU checks: the C-ABI library loads and exports exactly what include/gpmdm_hip.h
declares; the replay module reproduces the reference's random-number consumption;
host-side model helpers.  No GPU calls."""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest
import torch

from conftest import ROOT

HEADER = ROOT / "include" / "gpmdm_hip.h"


def _declared():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(gpmdm_\w+)\s*\(", text, re.M)))


def test_library_exports_every_declared_symbol():
    from gpmdm_amd import build, _lib
    build.build()                       # no-op when up to date
    lib = ctypes.CDLL(str(_lib.LIB_PATH))
    decl = _declared()
    assert len(decl) >= 18
    for name in decl:
        assert hasattr(lib, name), name
    assert sorted(_lib.EXPORTED_SYMBOLS) == decl


def test_library_version_and_error_without_gpu():
    from gpmdm_amd import _lib
    lib = _lib.load()
    assert b"gfx950" in lib.gpmdm_version()
    # a null descriptor is rejected before any HIP call
    h = ctypes.c_void_p()
    rc = lib.gpmdm_model_create(None, 0, ctypes.byref(h))
    assert rc == -1
    assert b"null" in lib.gpmdm_last_error()


def test_replay_matches_reference_consumption(fx_config1):
    """torch.manual_seed(11) then the replay draws in the reference order reproduce the
    streams the reference consumed (captured in the fixture)."""
    from gpmdm_amd import replay
    f = fx_config1
    P, C, d = 100, 2, 3
    torch.manual_seed(11)
    sizes = [250, 250]
    idx = replay.init_draws(sizes, list(f["traj_init_counts"]))
    assert np.array_equal(np.concatenate(idx), f["traj_init_idx"])
    for k in range(20):
        E = replay.switch_draws(P, C)
        assert np.array_equal(E, f["traj_E"][k])
        cls = f["traj_classes_switched"][k]
        counts = [int((cls == c).sum()) for c in range(C)]
        assert np.array_equal(replay.dynamics_draws(counts, d), f["traj_normals"][k])
        assert np.array_equal(replay.resample_draws(P), f["traj_u"][k])


def test_xin_xout_modes_host():
    """get_Xin_Xout_matrices (gpmdm.py:630-718) on the host model, all four modes."""
    from gpmdm_amd.model import GPMDM
    m = GPMDM.__new__(GPMDM)
    m.class_aware_observations_list = [[np.zeros((4, 2)), np.zeros((3, 2))], [np.zeros((5, 2))]]
    m.dyn_target, m.dyn_back_step = "full", 1
    m.X = torch.arange(24, dtype=torch.float64).reshape(12, 2)
    Xin, Xout, st = m.get_Xin_Xout_matrices()
    assert st == [0, 4, 7] and Xin.shape == (9, 2)
    assert torch.equal(Xout[0], m.X[1]) and torch.equal(Xin[3], m.X[4])
    Xin, Xout, _ = m.get_Xin_Xout_matrices(target="delta")
    assert torch.all(Xout == 2.0)
    Xin, Xout, _ = m.get_Xin_Xout_matrices(back_step=2)
    assert Xin.shape == (6, 4) and torch.equal(Xin[0], torch.cat([m.X[1], m.X[0]]))
    assert m._class_dynamics_rows() == [5, 4]


def test_pf_constructor_validation_without_gpu():
    """The class-count check of gpmdm_pf.py:74-75 fires before any device work."""
    import pytest
    from gpmdm_amd import GPMDM_PF

    class Fake:
        n_classes = 2
        dtype = torch.float64

        def set_evaluation_mode(self):
            pass

    with pytest.raises(ValueError, match="do not match"):
        GPMDM_PF(Fake(), torch.eye(3), 10)


def test_synthetic_shapes():
    from gpmdm_amd import synthetic
    data = synthetic.make_sequences(**{k: synthetic.CONFIGS[1][k] for k in ("C", "S", "L", "D", "d")})
    assert len(data.sequences) == 2 and data.sequences[0][0].shape == (50, 62)
    assert data.sequences[0][0].dtype == np.float32
    T = synthetic.markov_matrix(3)
    assert np.allclose(T.sum(1), 1.0) and T[0, 0] == 0.9


def test_c_host_builds_and_links():
    """examples/c_host/pf_main (the native C host of the C ABI) compiles with gcc against
    include/gpmdm_hip.h alone and resolves every symbol it uses from the in-tree library
    (run without arguments: usage, exit status 2, no GPU touched)."""
    import subprocess
    from gpmdm_amd import build
    exe = build.build_c_host()
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr


def test_frame_draws_are_the_replay_streams():
    """replay.FrameDraws (in-place, preallocated) draws the streams of switch_draws /
    dynamics_draws / resample_draws: class blocks below and above torch's 16-value
    vectorised threshold, empty classes, several frames."""
    from gpmdm_amd import replay
    P, C, d = 37, 3, 3
    frames = [[20, 0, 17], [1, 30, 6], [37, 0, 0], [5, 5, 27]]
    torch.manual_seed(11)
    want = []
    for counts in frames:
        want.append((replay.switch_draws(P, C).copy(), replay.dynamics_draws(counts, d).copy(),
                     replay.resample_draws(P).copy()))
    torch.manual_seed(11)
    fd = replay.FrameDraws(P, C, d, P)
    for counts, (E, N, U) in zip(frames, want):
        assert np.array_equal(fd.switch(), E)
        assert np.array_equal(fd.dynamics(counts), N)
        assert np.array_equal(fd.resample(), U)
    with pytest.raises(ValueError):
        fd.dynamics([1, 2, 3])


def test_rccl_is_not_a_load_time_dependency():
    """RCCL is resolved at run time by the communicator calls only: a
    single-GPU user's process never needs librccl to load the library."""
    import subprocess
    from gpmdm_amd import _lib as L
    out = subprocess.run(["readelf", "-d", str(L.LIB_PATH)], capture_output=True, text=True).stdout
    needed = [ln for ln in out.splitlines() if "NEEDED" in ln]
    assert needed and not any("rccl" in ln for ln in needed), needed
