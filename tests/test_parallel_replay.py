"""CPU: the parallel replay draws (replay.ParallelFrameDraws over gpmdm_rng_walk) are bit for
bit torch's serial draws in the reference's order (gpmdm_pf.py:137-213), and leave torch's
global generator where the serial draws leave it -- including classes of fewer than 16
normals (torch's serial path with its normal cache), empty classes, odd lengths, and a
caller's own draws between frames (which invalidate the draws made ahead)."""
import numpy as np
import pytest
import torch

from gpmdm_amd import _lib
from gpmdm_amd.replay import STATE_BYTES, FrameDraws, ParallelFrameDraws, _Walk


def test_walk_states_are_torch_states():
    """The walk's state after n draws is torch's own state after torch.rand(n, float64)."""
    torch.manual_seed(3)
    torch.randn(3, dtype=torch.float64)           # odd serial normals: a cached normal in the state
    s0 = torch.get_rng_state()
    w = _Walk().reset(s0.numpy().copy(), 5000)
    g = torch.Generator()
    for n in (0, 1, 2, 311, 312, 313, 623, 624, 625, 1248, 4999, 5000):
        g.set_state(s0)
        torch.rand(n, dtype=torch.float64, generator=g)
        assert torch.equal(w.state(n), g.get_state()), n
    with pytest.raises(ValueError):
        w.state(5001 + 312)
    bad = s0.numpy().copy()
    bad[8:12] = 0                                  # left = 0: not a generator state
    with pytest.raises(ValueError):
        _Walk().reset(bad, 10)
    assert s0.numel() == STATE_BYTES


def test_walk_states_batch_is_walk_state():
    torch.manual_seed(4)
    s0 = torch.get_rng_state().numpy().copy()
    w = _Walk().reset(s0, 3000)
    offs = np.array([0, 5, 311, 312, 2999, 7], dtype=np.int64)
    cache = s0.copy()
    cache[5016:] = 7
    got = w.states(offs, cache)
    for k, o in enumerate(offs):
        assert np.array_equal(got[k], w.state(int(o), cache).numpy()), o


def _frames(P, C, d, counts_list, interleave, threads, native=None):
    torch.manual_seed(5)
    ref = FrameDraws(P, C, d, P)
    outs = []
    for k, counts in enumerate(counts_list):
        outs.append((ref.switch().copy(), ref.dynamics(counts).copy(), ref.resample().copy(),
                     torch.get_rng_state().clone()))
        if interleave and k == 1:
            torch.randn(7)
    torch.manual_seed(5)
    par = ParallelFrameDraws(P, C, d, P, threads=threads, native=native)
    par.record = True
    for k, counts in enumerate(counts_list):
        par.begin()
        par.dynamics(counts)
        par.resample()
        e, n, u, s = outs[k]
        assert np.array_equal(par.last_E, e), (k, "E")
        assert np.array_equal(par.last_N, n), (k, "normals", int(np.sum(par.last_N != n)))
        assert np.array_equal(par.last_U, u), (k, "U")
        assert torch.equal(torch.get_rng_state(), s), (k, "generator state")
        if interleave and k == 1:
            torch.randn(7)
    hits, misses = par.prefetch_hits, par.prefetch_misses
    par.close()
    return hits, misses


@pytest.mark.parametrize("P,C,d,counts_list", [
    (1000, 3, 3, [[500, 499, 1], [0, 1000, 0], [998, 1, 1], [333, 333, 334], [2, 3, 995]]),
    (20000, 5, 8, [[4000] * 5, [1, 1, 1, 1, 19996], [19999, 0, 0, 0, 1], [2, 19990, 3, 2, 3]]),
    (50001, 2, 3, [[25001, 25000], [50001, 0], [5, 49996], [0, 50001]]),
])
@pytest.mark.parametrize("interleave", [False, True])
@pytest.mark.parametrize("native", [True, False], ids=["native", "pythonpool"])
def test_parallel_draws_are_the_serial_draws(P, C, d, counts_list, interleave, native):
    """The chunks run by libgpmdm_replay.so (csrc/replay_draws.cpp: torch's samplers on its
    native thread pool) and on the Python thread pool."""
    hits, misses = _frames(P, C, d, counts_list, interleave, threads=4, native=native)
    assert misses == (2 if interleave else 1)    # the first frame, and the frame after a caller's draw
    assert hits == len(counts_list) - misses


def test_library_declares_the_walk():
    lib = _lib.load()
    for name in ("gpmdm_rng_walk_create", "gpmdm_rng_walk_reset", "gpmdm_rng_walk_state", "gpmdm_rng_walk_states",
                 "gpmdm_rng_walk_destroy"):
        assert hasattr(lib, name)


def test_native_runner_exports_and_rejects_bad_arguments():
    """libgpmdm_replay.so (built by gpmdm_amd.build): its entry points, and argument checks
    that return an error instead of drawing (no GPU)."""
    import ctypes
    from gpmdm_amd.replay import _Native
    lib = _Native.load()
    if lib is None:
        pytest.skip("GPMDM_REPLAY_PY_CHUNKS set or the runner is not built")
    for name in ("gpmdm_replay_draw_chunks", "gpmdm_replay_warm", "gpmdm_replay_last_error"):
        assert hasattr(lib, name)
    buf = np.zeros(64)
    states = np.zeros((1, STATE_BYTES), dtype=np.uint8)
    bad = np.array([10, 5], dtype=np.int64)                     # end before begin
    assert lib.gpmdm_replay_draw_chunks(1, buf.ctypes.data, bad.ctypes.data, states.ctypes.data, 1, 2) == -1
    assert b"bounds" in lib.gpmdm_replay_last_error()
    ok = np.array([0, 64], dtype=np.int64)
    assert lib.gpmdm_replay_draw_chunks(7, buf.ctypes.data, ok.ctypes.data, states.ctypes.data, 1, 2) == -1   # kind
    assert lib.gpmdm_replay_warm(4, 100) == 0
    assert lib.gpmdm_replay_warm(4, -1) == 0                    # ignored
    # a real draw from torch's state: the values of a generator in that state
    torch.manual_seed(8)
    st = torch.get_rng_state().numpy().copy()[None, :]
    assert lib.gpmdm_replay_draw_chunks(2, buf.ctypes.data, ok.ctypes.data, st.ctypes.data, 1, 1) == 0
    g = torch.Generator()
    g.set_state(torch.from_numpy(st[0].copy()))
    assert np.array_equal(buf, torch.empty(64, dtype=torch.float64).uniform_(0, 1, generator=g).numpy())
