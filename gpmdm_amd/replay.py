"""Replay of the reference's random-number consumption (``rng='torch'`` mode).

The reference draws everything from torch's global CPU generator, in a fixed order
(verified bitwise against the unmodified reference):

1. ``GPMDM_PF._sample_particles_from_training_data`` (`gpmdm_pf.py:106-115`): for each
   class ``c`` in order, ``torch.randint(0, |X_c|, (P_c,))``;
2. per frame, ``_propogate_markov_switching`` (`gpmdm_pf.py:137-151`):
   ``torch.multinomial(probs, 1)`` draws ``empty_like(probs).exponential_(1)`` on a
   ``P x C`` float64 tensor and takes ``argmax(probs / E)``;
3. ``_propogate_dynamics`` (`gpmdm_pf.py:153-168`): for each class in order,
   ``torch.normal(mean, std)`` draws ``normal_(0, 1)`` on a ``P_c x d`` float64 tensor
   (``P_c`` counted after the switch) and returns ``eps * std + mean``;
4. ``_resample`` (`gpmdm_pf.py:206-213`): ``torch.multinomial(w, P, True)`` draws one
   float64 uniform per sample, i.e. the stream of ``torch.rand(P, dtype=float64)``.

Drawing the same shapes from the same generator in the same order therefore gives
the exact streams the reference would consume; the HIP kernels then consume them
through the C ABI.  torch's CPU ``normal_`` takes a size-dependent vectorised path,
so each class is drawn with its own ``(P_c, d)`` shape, never as one long tensor.

torch is used here as the reference's random-number generator, nothing else.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch


def init_draws(class_sizes, counts, generator: Optional[torch.Generator] = None):
    """randint draws of `gpmdm_pf.py:113`, one int64 array per class."""
    out = []
    for n_c, p_c in zip(class_sizes, counts):
        idx = torch.randint(0, int(n_c), (int(p_c),), generator=generator)
        out.append(idx.numpy().astype(np.int64))
    return out


def switch_draws(P: int, C: int, generator: Optional[torch.Generator] = None) -> np.ndarray:
    """Exp(1) draws of ``torch.multinomial(probs, 1)`` (P x C float64)."""
    e = torch.empty((P, C), dtype=torch.float64).exponential_(1, generator=generator)
    return e.numpy()


def dynamics_draws(counts, d: int, generator: Optional[torch.Generator] = None) -> np.ndarray:
    """Standard normals of ``torch.normal(mean, std)`` per class, concatenated in class
    order ((sum P_c) x d float64).  Empty classes draw nothing."""
    parts = []
    for p_c in counts:
        p_c = int(p_c)
        if p_c == 0:
            continue
        parts.append(torch.empty((p_c, d), dtype=torch.float64).normal_(0, 1, generator=generator).numpy())
    if not parts:
        return np.zeros((0, d))
    return np.concatenate(parts, 0)


def resample_draws(P: int, generator: Optional[torch.Generator] = None) -> np.ndarray:
    """Uniforms of ``torch.multinomial(w, P, replacement=True)`` (P float64)."""
    return torch.rand((P,), dtype=torch.float64, generator=generator).numpy()


class FrameDraws:
    """The per-frame streams of ``switch_draws`` / ``dynamics_draws`` /
    ``resample_draws`` drawn in place into buffers allocated once (the notebook's
    per-frame host cost is mostly torch's per-call overhead, not the draws).  A
    contiguous block of rows draws exactly what a fresh tensor of its shape draws, so
    the streams are unchanged (tests/test_abi_and_replay.py).  The returned arrays are
    overwritten by the next frame's draws."""

    def __init__(self, P: int, C: int, d: int, n_uniform: int,
                 generator: Optional[torch.Generator] = None):
        self._gen = generator
        self._E = torch.empty((P, C), dtype=torch.float64)
        self._N = torch.empty((P, d), dtype=torch.float64)
        self._U = torch.empty((n_uniform,), dtype=torch.float64)
        self.E, self.N, self.U = self._E.numpy(), self._N.numpy(), self._U.numpy()

    def switch(self) -> np.ndarray:
        self._E.exponential_(1, generator=self._gen)
        return self.E

    def dynamics(self, counts) -> np.ndarray:
        off = 0
        for p_c in counts:
            p_c = int(p_c)
            if p_c:
                self._N[off:off + p_c].normal_(0, 1, generator=self._gen)
                off += p_c
        if off != self._N.shape[0]:
            raise ValueError(f"class counts sum to {off}, not {self._N.shape[0]}")
        return self.N

    def resample(self) -> np.ndarray:
        self._U.uniform_(0, 1, generator=self._gen)
        return self.U


# ---- parallel replay (large filters) ---------------------------------------------------
STATE_BYTES = 5056                    # torch CPU generator state (GPMDM_TORCH_GEN_STATE_BYTES)
_CACHE = slice(5016, 5056)            # the normal-sample caches of that state (double and float)


def host_threads() -> int:
    """Cores this process may really use: the CPU affinity capped by the cgroup's CPU quota
    (a GPU box shows 256 CPUs and grants 16) and by OMP_NUM_THREADS when set."""
    import os
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(np.ceil(int(q) / int(per)))))
    except Exception:
        pass
    v = os.environ.get("OMP_NUM_THREADS", "")
    if v.isdigit() and int(v) > 0:
        n = min(n, int(v))
    return max(1, n)


class _Walk:
    """gpmdm_rng_walk: generator states at draw offsets of one stretch of the stream."""

    def __init__(self):
        import ctypes
        from . import _lib
        self._lib, self._ct = _lib, ctypes
        self._h = None
        self.n_draws = 0

    def reset(self, state: np.ndarray, n_draws: int) -> "_Walk":
        ct, lib = self._ct, self._lib.load()
        buf = ct.c_void_p(state.ctypes.data)
        if self._h is None:
            h = ct.c_void_p()
            self._lib.check(lib.gpmdm_rng_walk_create(buf, int(n_draws), ct.byref(h)), "rng walk")
            self._h = h
        else:
            self._lib.check(lib.gpmdm_rng_walk_reset(self._h, buf, int(n_draws)), "rng walk")
        self.n_draws = int(n_draws)
        return self

    def state(self, draws: int, cache_from: Optional[np.ndarray] = None) -> torch.Tensor:
        out = torch.empty(STATE_BYTES, dtype=torch.uint8)
        cf = None if cache_from is None else cache_from.ctypes.data
        self._lib.check(self._lib.load().gpmdm_rng_walk_state(self._h, int(draws), cf, out.data_ptr()), "rng walk")
        return out

    def states(self, draws: np.ndarray, cache_from: Optional[np.ndarray] = None) -> np.ndarray:
        """The states at every offset of ``draws`` (int64), one row each (n x STATE_BYTES)."""
        draws = np.ascontiguousarray(draws, dtype=np.int64)
        out = np.empty((draws.size, STATE_BYTES), dtype=np.uint8)
        cf = None if cache_from is None else cache_from.ctypes.data
        self._lib.check(self._lib.load().gpmdm_rng_walk_states(self._h, draws.size, draws.ctypes.data, cf,
                                                               out.ctypes.data), "rng walk")
        return out

    def __del__(self):
        try:
            if self._h:
                self._lib.load().gpmdm_rng_walk_destroy(self._h)
                self._h = None
        except Exception:
            pass


_EXPONENTIAL, _NORMAL, _UNIFORM = 0, 1, 2
_OPS = {_EXPONENTIAL: lambda x, g: x.exponential_(1, generator=g),
        _NORMAL: lambda x, g: x.normal_(0, 1, generator=g),
        _UNIFORM: lambda x, g: x.uniform_(0, 1, generator=g)}


class _Native:
    """libgpmdm_replay.so (csrc/replay_draws.cpp, built by gpmdm_amd/build.py): all chunks of
    a draw run by torch's samplers on a native thread pool in one call, the GIL released.
    ``None`` when the library is absent or GPMDM_REPLAY_PY_CHUNKS is set (the chunks then
    run on a Python thread pool: the same samplers and values, ~15 us more per chunk)."""
    _lib = None
    _tried = False

    @classmethod
    def load(cls):
        import ctypes
        import os
        from pathlib import Path
        if not cls._tried:
            cls._tried = True
            path = Path(__file__).resolve().parent / "libgpmdm_replay.so"
            if path.exists() and not os.environ.get("GPMDM_REPLAY_PY_CHUNKS"):
                lib = ctypes.CDLL(str(path))
                lib.gpmdm_replay_draw_chunks.restype = ctypes.c_int
                lib.gpmdm_replay_draw_chunks.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                         ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
                lib.gpmdm_replay_last_error.restype = ctypes.c_char_p
                lib.gpmdm_replay_warm.restype = ctypes.c_int
                lib.gpmdm_replay_warm.argtypes = [ctypes.c_int, ctypes.c_int64]
                cls._lib = lib
        return cls._lib


class ParallelFrameDraws:
    """The per-frame streams of FrameDraws (the reference's order: E_k, per-class normals,
    U_k; gpmdm_pf.py:137-213) bit for bit, with torch's own samplers run as parallel chunks.

    torch's CPU samplers are serial: ~13 ms per frame at P = 100k on one core, twice the GPU
    frame.  Each chunk here runs the same sampler (exponential_, normal_, uniform_) on a
    private generator placed at the exact state the serial draw would have reached at that
    chunk (gpmdm_rng_walk, torch_rng.cpp).  exponential_ and uniform_ take one random64 per
    value; normal_ on n >= 16 values fills n uniforms and Box-Mullers blocks of 16
    (recomputing the last 16 with 16 fresh uniforms when 16 does not divide n), so the chunks
    of a class start at multiples of 16 values and the last chunk carries the class's tail; a
    class of fewer than 16 values takes torch's serial path (pairs, with the generator's
    normal cache), run on one private generator whose cache then carries on.  The global
    generator ends each frame where the serial draws would leave it.

    What does not depend on the device's results is drawn ahead, on a background thread,
    while the GPU runs the frame: as soon as a frame's last draw is placed (``resample``),
    the walk over the next frame's stretch, its Exp(1) switch draws, and the normals of its
    first non-empty class -- that class's values start at a fixed place of the stream (right
    after E) and its blocks of 16 do not depend on its length, so the normals are drawn for
    the longest length it can have and only its last 16 (when 16 does not divide its length)
    are drawn again once the switch's counts are known.  ``begin()`` uses them only if the
    global generator still stands where the frame ended (any other draw in between
    invalidates them, and they are drawn again there and then), so the streams are the
    reference's whatever the caller does between frames."""

    def __init__(self, P: int, C: int, d: int, n_uniform: int, threads: Optional[int] = None,
                 chunk: Optional[int] = None, buffers=None, wait_free=None, native: Optional[bool] = None):
        """``buffers``: (E, N, U) float64 numpy arrays to draw into (e.g. the library's
        pinned staging buffers, gpmdm_pf_draw_buffers), else own ones; ``wait_free(k)``
        (k = 0 E, 1 N, 2 U) returns once buffer k may be rewritten (gpmdm_pf_draws_free).
        ``chunk``: the least values per chunk (default 2048 with the native runner, 8192 on
        the Python pool).  ``native``: run the chunks through libgpmdm_replay.so (True; an
        error if it is absent), on the Python pool (False), or the former when present."""
        from concurrent.futures import ThreadPoolExecutor
        self.P, self.C, self.d, self.nu = int(P), int(C), int(d), int(n_uniform)
        self.threads = threads or host_threads()
        self._native = _Native.load() if native is not False else None
        if native and self._native is None:
            raise RuntimeError("libgpmdm_replay.so is not built (python -m gpmdm_amd.build)")
        self._pool = None if self._native is not None else ThreadPoolExecutor(max_workers=self.threads)
        self._bg = ThreadPoolExecutor(max_workers=1)
        self._chunk = int(chunk or (2048 if self._native is not None else 8192))
        if buffers is None:
            buffers = (np.empty((P, C)), np.empty((P, d)), np.empty((self.nu,)))
        self.E, self.N, self.U = (np.asarray(b, dtype=np.float64) for b in buffers)
        assert self.E.shape == (P, C) and self.N.shape == (P, d) and self.U.shape == (self.nu,)
        self._E, self._N, self._U = (torch.from_numpy(b) for b in (self.E, self.N, self.U))
        self._wait_free = wait_free or (lambda k: None)
        self._walks = (_Walk(), _Walk())   # this frame's and the next frame's (buffers reused)
        self._wi = 0
        self._walk = None
        self._cache = None              # a state holding the stream's current normal-cache bytes
        self._spec = False              # N holds the first class's normals drawn ahead
        self._pos = 0                   # draws consumed in the frame so far
        self._expect = None             # global state the last frame ended in
        self._pending = None            # background future (the next frame's walk, E, first normals)
        self.prefetch_hits = 0
        self.prefetch_misses = 0
        self.last_hit = False           # the last begin() used the draws made ahead
        self.ahead_valid = 0            # leading values of N the last dynamics() kept from the ahead draw
        self.record = False             # keep copies of the frame's draws (last_E/N/U; tests): E
                                        # and N are refilled ahead for the next frame

    # draws of one frame at most: E, the normals (+16 per class for a tail, a small class
    # at most 16), U
    def _frame_draws(self) -> int:
        return self.P * self.C + self.P * self.d + 16 * self.C + self.nu

    def _draw(self, kind: int, flat: torch.Tensor, walk: _Walk, cache: np.ndarray, spans):
        """Run the chunks ``spans`` = [(a, b, draw offset)] of one sampler: flat[a:b] drawn
        from the walk's state at that offset (normal caches of ``cache``), in parallel."""
        if not spans:
            return
        offs = np.array([o for _, _, o in spans], dtype=np.int64)
        states = walk.states(offs, cache)
        if self._native is not None:
            bounds = np.array([(a, b) for a, b, _ in spans], dtype=np.int64)
            if self._native.gpmdm_replay_draw_chunks(kind, flat.data_ptr(), bounds.ctypes.data, states.ctypes.data,
                                                     len(spans), self.threads) != 0:
                raise RuntimeError("replay draws: " + self._native.gpmdm_replay_last_error().decode())
            return
        op = _OPS[kind]
        st = [torch.from_numpy(states[k].copy()) for k in range(len(spans))]   # (set_state of a row view faults)
        tasks = [lambda a=a, b=b, k=k: op(flat[a:b], self._gen(st[k])) for k, (a, b, _) in enumerate(spans)]
        futs = [self._pool.submit(f) for f in tasks[1:]]
        tasks[0]()
        for f in futs:
            f.result()

    @staticmethod
    def _gen(state: torch.Tensor) -> torch.Generator:
        g = torch.Generator()
        g.set_state(state)
        return g

    def _normal_spans(self, off: int, n: int, pos: int, spans: list):
        """Chunks of one class's normal_ (n >= 16 values at flat[off:], from draw ``pos``)."""
        step = max(16 * -(-self._chunk // 16), 16 * -(-n // (16 * self.threads)))
        a = 0
        while a < n:
            b = n if n - a < step + 16 else a + step   # the last chunk: >= 16 values, the tail
            spans.append((off + a, off + b, pos + a))
            a = b

    def _plain_spans(self, n: int, pos: int):
        step = max(self._chunk, -(-n // self.threads))
        return [(a, min(n, a + step), pos + a) for a in range(0, n, step)]

    def _ahead(self, walk: _Walk, state: np.ndarray):
        """The frame's draws that need no device result: E, and the first class's normals
        for the longest length (all P particles)."""
        walk.reset(state, self._frame_draws())
        self._wait_free(0)
        self._wait_free(1)
        flat = self._E.view(-1)
        self._draw(_EXPONENTIAL, flat, walk, state, self._plain_spans(flat.numel(), 0))
        spec = self.P * self.d >= 16
        if spec:
            spans = []
            self._normal_spans(0, self.P * self.d, self.P * self.C, spans)
            self._draw(_NORMAL, self._N.view(-1), walk, state, spans)
        return walk, state, spec

    def ahead_ready(self) -> bool:
        """Wait for the next frame's draws ahead (if any are being made); True if there are."""
        if self._pending is None:
            return False
        self._pending.result()
        return True

    def begin(self) -> np.ndarray:
        """The frame's Exp(1) switch draws (P x C), from the global generator's state."""
        if self._native is not None:    # the pool polls until the frame's normals (dynamics())
            self._native.gpmdm_replay_warm(self.threads, 400)
        cur = torch.get_rng_state()
        got = None
        if self._pending is not None:
            got = self._pending.result()
            self._pending = None
        self.last_hit = got is not None and self._expect is not None and torch.equal(cur, self._expect)
        if self.last_hit:
            self._walk, self._cache, self._spec = got
            self.prefetch_hits += 1
        else:
            self._wi ^= 1 if got is None else 0
            self._walk, self._cache, self._spec = self._ahead(self._walks[self._wi], cur.numpy().copy())
            self.prefetch_misses += 1
        self._pos = self.P * self.C
        if self.record:
            self.last_E = self.E.copy()
        return self.E

    switch = begin                      # FrameDraws' name for the frame's first draw

    def dynamics(self, counts) -> np.ndarray:
        """Per-class standard normals (sum_c P_c) x d in class order."""
        walk, d = self._walk, self.d
        flat = self._N.view(-1)
        spans, row, first = [], 0, True
        self.ahead_valid = 0
        if int(sum(int(c) for c in counts)) != self.P:
            raise ValueError(f"class counts sum to {sum(counts)}, not {self.P}")
        for p_c in counts:
            p_c = int(p_c)
            if p_c == 0:
                continue
            n = p_c * d
            off = row * d
            if n < 16:                  # torch's serial path: pairs and the normal cache
                self._draw(_NORMAL, flat, walk, self._cache, spans)   # (the chunks before it
                spans = []                                            # do not depend on it)
                g = self._gen(walk.state(self._pos, self._cache))
                flat[off:off + n].normal_(0, 1, generator=g)
                after = g.get_state().numpy()
                self._cache = self._cache.copy()
                self._cache[_CACHE] = after[_CACHE]
                self._pos += _consumed(after, walk, self._pos)
            elif first and self._spec:  # drawn ahead; only a tail's last 16 are drawn again
                if n % 16:
                    spans.append((off + n - 16, off + n, self._pos + n))
                self.ahead_valid = n - 16 if n % 16 else n
                self._pos += n + (16 if n % 16 else 0)
            else:
                self._normal_spans(off, n, self._pos, spans)
                self._pos += n + (16 if n % 16 else 0)
            first = False
            row += p_c
        self._draw(_NORMAL, flat, walk, self._cache, spans)
        if self.record:
            self.last_N = self.N.copy()
        return self.N

    def resample(self) -> np.ndarray:
        """The resampling uniforms; the global generator then stands where the serial
        frame would leave it, and the next frame's draws ahead start in the background."""
        walk, n = self._walk, self.nu
        self._wait_free(2)
        self._draw(_UNIFORM, self._U, walk, self._cache, self._plain_spans(n, self._pos))
        if self.record:
            self.last_U = self.U.copy()
        self._pos += n
        end = walk.state(self._pos, self._cache)
        torch.set_rng_state(end)
        self._expect = end
        self._wi ^= 1
        self._pending = self._bg.submit(self._ahead, self._walks[self._wi], end.numpy().copy())
        return self.U

    def close(self):
        if self._pending is not None:
            self._pending.result()
            self._pending = None
        if self._pool is not None:
            self._pool.shutdown(wait=True)
        self._bg.shutdown(wait=True)


def _consumed(state_after: np.ndarray, walk: _Walk, pos: int) -> int:
    """Draws between ``pos`` and a state reached from it by a short serial draw (< 32)."""
    for k in range(0, 34):
        if np.array_equal(walk.state(pos + k).numpy()[8:24 + 8 * 624], state_after[8:24 + 8 * 624]):
            return k
    raise RuntimeError("could not place a serial normal draw on the generator's stream")
