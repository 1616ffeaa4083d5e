"""GPMDM_PF -- drop-in mirror of ``/root/reference/gpmdm/gpmdm_pf.py`` on libgpmdm_hip.

Same constructor, methods and properties as the reference class (gpmdm_pf.py:47-312);
every per-frame computation runs in the HIP library.  Extra keyword options:

* ``rng='torch'`` (default): the random draws come from torch's global CPU generator in
  exactly the reference's order (``gpmdm_amd.replay``), so ``torch.manual_seed(s)``
  reproduces the reference's sampling; ``rng='philox'`` draws on the device (no host
  work per frame; the bench mode);
* ``seed``: Philox key (default: drawn from torch's generator);
* ``resample='multinomial'`` (reference, gpmdm_pf.py:211) or ``'systematic'``;
* ``process_group``: a ``torch.distributed`` group to shard particles over (one process
  per GPU; per frame, the new {class, state} rows are all-gathered while the observation GP
  runs and the likelihoods after it).  The Philox seed and
  the initial particles are broadcast from the group's rank 0, so every rank holds the
  same replicated filter whatever its local torch RNG state; replay mode (``rng='torch'``)
  consumes the host generator on every rank and therefore requires identical torch RNG
  states on all ranks (checked at construction: ``ValueError`` otherwise);
* ``devices=[d0, d1, ...]``: one process drives one rank per GPU (SURVEY §5's config row;
  a notebook uses several GPUs without torchrun): a library handle per device on the
  model's image there (``GPMDM.handle_on``), communicators made together
  (``gpmdm_comm_init_all``), and per frame every rank's stages with their all-gathers grouped
  (``gpmdm_pf_propagate_multi``); rank r owns ``device_shard_plan``'s particle range.  The
  read-outs and exports come from rank 0 (the filter is replicated).  ``devices=[0]`` is the
  plain filter bit for bit.  ``transport='loopback'`` (tests) swaps RCCL for the library's
  in-process loopback communicators (``gpmdm_comm_init_loopback``), which also accept a
  device repeated, e.g. ``devices=[0] * 8``: the multi-rank exchange on one GPU;
* ``shard=(world, rank)``: sharding with a caller-driven exchange (``exchange=`` or the
  staged calls); a Philox filter then needs an explicit ``seed`` (nothing to broadcast).
  ``exchange(recv, send)`` is called twice per frame: with the (P x (d+1)) / (P_r x (d+1))
  ``{class, state[d]}`` rows after the dynamics GP, then with the (P x 1) / (P_r x 1)
  ``{ll}`` column after the observation GP;
* ``dedup`` (default True): evaluate the dynamics GP once per distinct (resampling
  ancestor, new class) pair -- offspring of one ancestor hold bit-identical states -- and
  share the result; bitwise identical to ``dedup=False`` (every particle evaluated) with
  the same dynamics tile shape (``dyn_tiles``).
* ``shard_order`` (default True; multi-rank philox filters): each rank evaluates a slice of
  the particles ordered by resampling ancestor rather than a slice of particle indices, so
  de-duplication keeps ~1/R of the distinct keys per rank; bitwise identical either way.
* ``set_comm(comm)``: hand the library an RCCL communicator (``gpmdm_amd.RcclComm`` or
  any ncclComm_t of ``shard=(world, rank)``'s ranks); ``update`` then exchanges the rows
  itself (``gpmdm_pf_set_comm``: both all-gathers on a library-owned stream, the first
  overlapping the observation GP), the native hosts' path -- no torch.distributed.
* ``dyn_tiles`` (``'auto'``): tile shape of the dynamics-GP pass (``gpmdm_pf_set_dyn_tiles``):
  narrow tiles for de-duplicated rows, wide ones when every particle is evaluated; for
  d <= 12 the two are bitwise identical, above it they differ in summation order only.

Reference quirks kept for parity: log variance counted twice in the
log-likelihood, float32 ``ln 2pi``, non-recursive weights, read-outs pairing
post-resample classes/states with pre-resample weights, ``ll + log_w`` in the posterior,
``log_likelihood()`` returning a sum of exponentials, ``dyn_target`` ignored.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib, replay
from .model import GPMDM


# Replay filters from this many particles draw torch's streams as parallel chunks
# (replay.ParallelFrameDraws); below it the serial draws cost less than the threads' hand-offs.
PARALLEL_REPLAY_P = 16384


def device_shard_plan(P: int, devices, repeat: bool = False) -> list:
    """(device, rank, lo, hi) of a one-process multi-device filter (GPMDM_PF(devices=...)):
    rank r runs on devices[r] and owns particles [r P / R, (r + 1) P / R) -- the library's
    own shard rule (gpmdm_pf_create), so the filter is bitwise the one-rank filter's.
    ``repeat``: a device may hold several ranks (the loopback transport; tests)."""
    devs = [int(x) for x in devices]
    if not devs:
        raise ValueError("devices must name at least one GPU")
    if not repeat and len(set(devs)) != len(devs):
        raise ValueError(f"devices must be distinct (one rank per GPU; RCCL refuses two on one device): {devs}")
    if any(x < 0 for x in devs):
        raise ValueError(f"bad device index in {devs}")
    R = len(devs)
    return [(dev, r, P * r // R, P * (r + 1) // R) for r, dev in enumerate(devs)]


def _as_f64_vector(z) -> np.ndarray:
    """The observation as a contiguous float64 vector (the reference casts it with
    torch.tensor(z, dtype=float64), gpmdm_pf.py:123; float32 -> float64 is exact)."""
    if isinstance(z, np.ndarray):
        return np.ascontiguousarray(z, dtype=np.float64).reshape(-1)
    return np.ascontiguousarray(torch.as_tensor(z, dtype=torch.float64).cpu().numpy().reshape(-1))


class GPMDM_PF:
    def __init__(self, gpmdm: GPMDM, markov_switching_model, num_particles: int, *,
                 rng: str = "torch", seed=None, resample: str = "multinomial", process_group=None,
                 shard=None, exchange=None, dedup: bool = True, shard_order: bool = True,
                 dyn_tiles: str = "auto", devices=None, obs_cutoff: bool = False, transport: str = "rccl"):
        self._gpmdm = gpmdm
        self._gpmdm.set_evaluation_mode()
        self._markov_switching_model = torch.as_tensor(markov_switching_model).type(self.dtype)
        self._num_particles = int(num_particles)
        if self._gpmdm.n_classes != self._markov_switching_model.size(0):
            raise ValueError("Number of classes in the GPMDM model and the Markov model do not match")
        if rng not in ("torch", "philox"):
            raise ValueError("rng must be 'torch' or 'philox'")
        if resample not in ("multinomial", "systematic"):
            raise ValueError("resample must be 'multinomial' or 'systematic'")
        self._rng = rng
        self._draws = None                      # replay.FrameDraws (rng='torch'), made on first use
        self._pre_sw = False                    # a replay pre-switch with the draws made ahead is pending
        self._n_staged = False                  # ... and the normals drawn ahead are on the device
        self._resample_mode = resample
        self._group = process_group
        self._exchange_fn = exchange
        self._devices = None
        if devices is not None:                 # one process, one handle per device (device_shard_plan)
            if process_group is not None or shard is not None or exchange is not None:
                raise ValueError("devices= drives every rank itself: no process_group, shard or exchange")
            if transport not in ("rccl", "loopback"):
                raise ValueError("transport must be 'rccl' or 'loopback'")
            self._devices = [p[0] for p in device_shard_plan(self._num_particles, devices,
                                                             repeat=transport == "loopback")]
            self._world, self._rank = len(self._devices), 0
        elif process_group is not None:
            import torch.distributed as dist
            self._world, self._rank = dist.get_world_size(process_group), dist.get_rank(process_group)
        elif shard is not None:                 # (world, rank) with a caller-driven exchange
            self._world, self._rank = int(shard[0]), int(shard[1])
            if self._world > 1 and rng == "philox" and seed is None:
                raise ValueError("shard= with rng='philox' needs an explicit seed (identical on every rank)")
        else:
            self._world, self._rank = 1, 0
        self._collective = process_group is not None and self._world > 1
        if self._collective and rng == "torch":
            from .distributed import identical_on_all_ranks
            if not identical_on_all_ranks(torch.get_rng_state().numpy().tobytes(), process_group, self.device):
                raise ValueError("rng='torch' on several ranks needs identical torch RNG states "
                                 "(torch.manual_seed with the same seed on every rank)")
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if rng == "philox" else 0
        if self._collective and rng == "philox":
            from .distributed import broadcast_array
            seed = int(broadcast_array(np.array([seed], dtype=np.int64), process_group, self.device)[0])
        self._seed = int(seed)
        lib = _lib.load()
        T = np.ascontiguousarray(self._markov_switching_model.numpy(), dtype=np.float64)
        if dyn_tiles not in _lib.DYN_TILES:
            raise ValueError("dyn_tiles must be 'auto', 'narrow' or 'wide'")

        if isinstance(obs_cutoff, str) and obs_cutoff != "auto":
            raise ValueError("obs_cutoff: True, False or 'auto'")
        self._obs_cutoff = 3 if obs_cutoff == "auto" else (1 if obs_cutoff else 0)
        if obs_cutoff:
            gpmdm.enable_obs_cutoff(True)       # the model's cutoff image (built once)

        def create(model_handle, rank):
            h = ctypes.c_void_p()
            _lib.check(lib.gpmdm_pf_create(
                model_handle, _lib.dptr(T), self._num_particles,
                _lib.GPMDM_RNG_REPLAY if rng == "torch" else _lib.GPMDM_RNG_PHILOX,
                ctypes.c_uint64(self._seed & (2 ** 64 - 1)),
                _lib.GPMDM_RESAMPLE_MULTINOMIAL if resample == "multinomial" else _lib.GPMDM_RESAMPLE_SYSTEMATIC,
                self._world, rank, ctypes.byref(h)), "GPMDM_PF")
            _lib.check(lib.gpmdm_pf_set_dedup(h, 1 if dedup else 0), "dedup")
            _lib.check(lib.gpmdm_pf_set_shard_order(h, 1 if shard_order else 0), "shard_order")
            _lib.check(lib.gpmdm_pf_set_dyn_tiles(h, _lib.DYN_TILES[dyn_tiles]), "dyn_tiles")
            if self._obs_cutoff:
                _lib.check(lib.gpmdm_pf_set_obs_cutoff(h, self._obs_cutoff), "obs_cutoff")
            return h

        self._peers = []                        # devices=: ranks 1.. as (handle, device index)
        self._comms = []
        if self._devices is None:
            self._h = create(gpmdm.handle, self._rank)
            self._dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        else:
            hs = [create(gpmdm.handle_on(dev), r) for r, dev in enumerate(self._devices)]
            self._h, self._dev_index = hs[0], self._devices[0]
            self._peers = list(zip(hs[1:], self._devices[1:]))
            # one communicator per device, made together (ncclCommInitAll); rank r on devices[r]
            # (transport='loopback': the library's in-process test transport, several ranks
            # per device allowed -- gpmdm_comm_init_loopback)
            n = len(self._devices)
            comms = (ctypes.c_void_p * n)()
            init = lib.gpmdm_comm_init_loopback if transport == "loopback" else lib.gpmdm_comm_init_all
            _lib.check(init(n, (ctypes.c_int * n)(*self._devices), comms), "gpmdm_comm_init")
            self._comms = [ctypes.c_void_p(c) for c in comms]
            for h, c in zip(hs, self._comms):
                _lib.check(lib.gpmdm_pf_set_comm(h, c, 0), "set_comm")
        self._model_gen = gpmdm.generation
        self._readout = None
        self._comm = self._comms[0] if self._comms else None
        # read-out landing buffers and their pointers, made once (read per frame)
        C, d = self.num_classes, self.latent_dim
        self._ro = (np.zeros(C), np.zeros(d), np.zeros(1))
        self._ro_ptr = tuple(_lib.dptr(a) for a in self._ro)
        if self._world > 1 and self._devices is None:
            h = self._h
            w, lo, hi = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
            lib.gpmdm_pf_exchange_width(h, ctypes.byref(w), ctypes.byref(lo), ctypes.byref(hi))
            dev = self.device
            n_loc, P = hi.value - lo.value, self._num_particles
            self._send = torch.empty((n_loc, w.value), dtype=torch.float64, device=dev)
            self._recv = torch.empty((P, w.value), dtype=torch.float64, device=dev)
            # the split exchange: {class, state} during the observation GP, then {ll}
            self._send_s = torch.empty((n_loc, w.value - 1), dtype=torch.float64, device=dev)
            self._recv_s = torch.empty((P, w.value - 1), dtype=torch.float64, device=dev)
            self._send_l = torch.empty((n_loc, 1), dtype=torch.float64, device=dev)
            self._recv_l = torch.empty((P, 1), dtype=torch.float64, device=dev)
        self._init_particles()

    def __del__(self):
        try:
            dr = getattr(self, "_draws", None)
            if dr is not None and hasattr(dr, "close"):
                dr.close()                      # draws ahead write into the handle's buffers: join them
            for h, _ in getattr(self, "_peers", []):
                _lib.load().gpmdm_pf_destroy(h)
            self._peers = []
            if getattr(self, "_h", None) is not None and self._h.value:
                _lib.load().gpmdm_pf_destroy(self._h)
                self._h = None
            for c in getattr(self, "_comms", []):   # after the filters using them
                _lib.load().gpmdm_comm_destroy(c)
            self._comms = []
        except Exception:
            pass

    # ---- helpers --------------------------------------------------------------
    def _stream(self):
        # the raw handle of the device's current stream (torch.cuda.current_stream builds a
        # Stream object per call: ~5 us, a visible share of a 0.12 ms notebook frame)
        return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(self._dev_index))

    def _sync_model(self):
        """The reference filter reads its GPMDM's current state on every call
        (gpmdm_pf.py:164, 183): after the model was rebuilt (set_latents, train_adam,
        a reload into the same object) rebind the device filter to the new image."""
        self._gpmdm._refresh()                  # parameters changed in place (an optimiser step)?
        if self._gpmdm.generation != self._model_gen:
            lib = _lib.load()
            if self._devices is None:
                _lib.check(lib.gpmdm_pf_set_model(self._h, self._gpmdm.handle), "rebind to the rebuilt model")
            else:
                for h, dev in [(self._h, self._devices[0])] + self._peers:
                    _lib.check(lib.gpmdm_pf_set_model(h, self._gpmdm.handle_on(dev)), "rebind to the rebuilt model")
            self._model_gen = self._gpmdm.generation

    def _all(self):
        """(handle, raw stream) of every rank this process drives (devices=: all of them)."""
        out = [(self._h, self._stream())]
        for h, dev in self._peers:
            out.append((h, ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(dev))))
        return out

    def _each(self, fn_name, *args, what=""):
        """The same library call (handle, *args, stream) on every rank this process drives."""
        lib = _lib.load()
        for h, s in self._all():
            _lib.check(getattr(lib, fn_name)(h, *args, s), what or fn_name)

    def _divide_into_n_parts(self, x: int, n: int) -> list:
        """gpmdm_pf.py:287-292."""
        g, r = divmod(x, n)
        return [g + (1 if i < r else 0) for i in range(n)]

    # ---- reference API ----------------------------------------------------------
    def _init_particles(self):
        """gpmdm_pf.py:87-115: P_c particles per class drawn from that class's latents."""
        counts = self._divide_into_n_parts(self._num_particles, self.num_classes)
        sizes = [self._gpmdm.get_X_for_class(c).shape[0] for c in range(self.num_classes)]
        idx = replay.init_draws(sizes, counts)
        states = np.concatenate([self._gpmdm.get_X_for_class(c).detach().cpu().numpy()[idx[c]] for c in range(self.num_classes)], 0)
        classes = np.concatenate([np.full(counts[c], c, dtype=np.int64) for c in range(self.num_classes)])
        states = np.ascontiguousarray(states, dtype=np.float64)
        if self._collective:                    # one replicated filter: rank 0's particles
            from .distributed import broadcast_array
            states = np.ascontiguousarray(broadcast_array(states, self._group, self.device))
            classes = np.ascontiguousarray(broadcast_array(classes, self._group, self.device))
        self._sync_model()
        for h in [self._h] + [p[0] for p in self._peers]:
            _lib.check(_lib.load().gpmdm_pf_init(h, _lib.dptr(states), _lib.i64ptr(classes)), "init")
        self._readout = None

    def reset(self):
        self._init_particles()

    def update(self, z):
        """gpmdm_pf.py:117-135: switch classes, propagate dynamics, weight, resample."""
        z = _as_f64_vector(z)
        if z.shape[0] != self.observation_dim:
            raise ValueError(f"observation must have {self.observation_dim} values, got {z.shape[0]}")
        self._sync_model()
        lib, h, s = _lib.load(), self._h, self._stream()
        P, C, d = self._num_particles, self.num_classes, self.latent_dim
        if self._rng == "torch":
            if self._draws is None:
                nu = P if self._resample_mode == "multinomial" else 1
                if P >= PARALLEL_REPLAY_P and replay.host_threads() > 1:
                    # torch's own samplers in parallel chunks, bit for bit the serial streams,
                    # drawn straight into the library's pinned staging buffers (no copy)
                    pe, pn, pu = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
                    _lib.check(lib.gpmdm_pf_draw_buffers(h, ctypes.byref(pe), ctypes.byref(pn), ctypes.byref(pu)),
                               "draw buffers")
                    bufs = (np.ctypeslib.as_array(ctypes.cast(pe, ctypes.POINTER(ctypes.c_double)), (P, C)),
                            np.ctypeslib.as_array(ctypes.cast(pn, ctypes.POINTER(ctypes.c_double)), (P, d)),
                            np.ctypeslib.as_array(ctypes.cast(pu, ctypes.POINTER(ctypes.c_double)), (nu,)))
                    hh = self._h
                    self._draws = replay.ParallelFrameDraws(
                        P, C, d, nu, buffers=bufs,
                        wait_free=lambda k: _lib.check(_lib.load().gpmdm_pf_draws_free(hh, k), "draw buffer"))
                else:
                    self._draws = replay.FrameDraws(P, C, d, nu)
                self._counts = np.zeros(C, dtype=np.int64)
                dr = self._draws           # the draws land in place: their pointers are fixed
                self._draw_ptr = (_lib.dptr(dr.E), _lib.i64ptr(self._counts), _lib.dptr(dr.N), _lib.dptr(dr.U))
            dr, counts = self._draws, self._counts
            pE, pC, pN, pU = self._draw_ptr
            dr.switch()
            if self._pre_sw and not dr.last_hit:
                # the caller drew from the generator since the pre-switch: its E is stale
                _lib.check(lib.gpmdm_pf_preswitch(h, pE, s), "preswitch")
            self._pre_sw = False
            _lib.check(lib.gpmdm_pf_switch(h, pE, pC, s), "switch")
            for hp, sp in self._all()[1:]:      # devices=: every rank switches all P (replay)
                _lib.check(lib.gpmdm_pf_switch(hp, pE, None, sp), "switch")
            dr.dynamics(counts)
            if self._n_staged:
                # the first class's normals drawn ahead went to the device behind the last
                # read-out; copy what dynamics() drew (everything if the ahead draw was stale)
                v = dr.ahead_valid if dr.last_hit else 0
                _lib.check(lib.gpmdm_pf_stage_normals(h, pN, v, P * d, s), "stage normals")
                self._n_staged = False
            self._propagate(z, dr.N, s, pN)
            dr.resample()
            self._each("gpmdm_pf_resample", pU, what="resample")
            if self._replay_preswitch() and dr.ahead_ready():
                # the next frame's E and first-class normals are drawn ahead (they need no
                # device result): its switch and dynamics tiles go behind this read-out
                # (gpmdm_pf_preswitch), and the normals to the device (gpmdm_pf_stage_normals)
                _lib.check(lib.gpmdm_pf_preswitch(h, pE, s), "preswitch")
                _lib.check(lib.gpmdm_pf_stage_normals(h, pN, 0, P * d, s), "stage normals")
                self._pre_sw = self._n_staged = True
        else:
            self._each("gpmdm_pf_switch", None, None, what="switch")
            self._propagate(z, None, s)
            self._each("gpmdm_pf_resample", None, what="resample")
        self._readout = None

    step = update    # north-star name (BASELINE.json): one filter step

    def _replay_preswitch(self) -> bool:
        """Replay filters whose draws are made ahead (ParallelFrameDraws), on one handle and
        one rank, launch the next switch between frames (GPMDM_NO_PRESWITCH=1: not, A/B)."""
        return (isinstance(self._draws, replay.ParallelFrameDraws) and not self._peers and self._world == 1
                and not os.environ.get("GPMDM_NO_PRESWITCH"))

    def update_with_draws(self, z, exp_draws, normals, uniforms):
        """One update with explicit random draws in the reference's order (replay: see
        gpmdm_amd.replay): exp_draws P x C, normals (sum_c P_c) x d grouped by class,
        uniforms P (multinomial) or 1 (systematic).  Requires rng='torch'."""
        if self._rng != "torch":
            raise ValueError("explicit draws need rng='torch' (replay mode)")
        z = _as_f64_vector(z)
        self._sync_model()
        lib, h, s = _lib.load(), self._h, self._stream()
        P, C, d = self._num_particles, self.num_classes, self.latent_dim
        E = np.ascontiguousarray(exp_draws, dtype=np.float64).reshape(P, C)
        self._each("gpmdm_pf_switch", _lib.dptr(E), None, what="switch")
        nrm = np.ascontiguousarray(normals, dtype=np.float64).reshape(P, d)
        self._propagate(z, nrm, s)
        U = np.ascontiguousarray(uniforms, dtype=np.float64).reshape(-1)
        self._each("gpmdm_pf_resample", _lib.dptr(U), what="resample")
        self._readout = None

    def set_comm(self, comm, pad_rows: bool = False):
        """Let the library run the per-frame exchange over an RCCL communicator
        (``gpmdm_pf_set_comm``; ``comm``: an ``RcclComm`` or a raw ncclComm_t address of
        this filter's (world, rank), on the model's device; ``None`` detaches).
        ``pad_rows`` forces the uneven-shard gather path (tests).  The communicator must
        outlive the filter's use of it."""
        if self._devices is not None:
            raise ValueError("a devices= filter holds its own communicators")
        ptr = getattr(comm, "ptr", comm)
        _lib.check(_lib.load().gpmdm_pf_set_comm(self._h, ctypes.c_void_p(ptr) if ptr else None,
                                                 _lib.GPMDM_COMM_PAD_ROWS if pad_rows else 0), "set_comm")
        self._comm = comm

    def _propagate(self, z, normals, s, normals_ptr=None):
        """gpmdm_pf.py:153-192 for this rank's particles, and on several ranks the exchange:
        the new {class, state} rows are all-gathered while the observation GP runs (they are
        final once the dynamics GP is done), the likelihoods after it -- by the library over
        its communicator (set_comm), or here over the process group / exchange callback."""
        lib, h = _lib.load(), self._h
        nrm = normals_ptr if normals_ptr is not None else (None if normals is None else _lib.dptr(normals))
        if self._devices is not None:
            # one thread drives every rank: the library stages them and groups the collectives
            hs = self._all()
            n = len(hs)
            _lib.check(lib.gpmdm_pf_propagate_multi((ctypes.c_void_p * n)(*[x[0] for x in hs]), n, _lib.dptr(z), nrm,
                                                    (ctypes.c_void_p * n)(*[x[1] for x in hs])), "propagate")
            return
        if self._world == 1 or self._comm is not None:
            _lib.check(lib.gpmdm_pf_propagate(h, _lib.dptr(z), nrm, s), "propagate")
            return
        _lib.check(lib.gpmdm_pf_propagate_dynamics(h, nrm, s), "propagate_dynamics")
        _lib.check(lib.gpmdm_pf_pack_part(h, self._send_s.data_ptr(), _lib.GPMDM_PACK_STATES, s), "pack")
        states_done = self._gather(self._recv_s, self._send_s)
        _lib.check(lib.gpmdm_pf_weigh(h, _lib.dptr(z), s), "weigh")
        _lib.check(lib.gpmdm_pf_pack_part(h, self._send_l.data_ptr(), _lib.GPMDM_PACK_LL, s), "pack")
        self._gather(self._recv_l, self._send_l)()
        states_done()
        _lib.check(lib.gpmdm_pf_unpack_part(h, self._recv_s.data_ptr(), _lib.GPMDM_PACK_STATES, s), "unpack")
        _lib.check(lib.gpmdm_pf_unpack_part(h, self._recv_l.data_ptr(), _lib.GPMDM_PACK_LL, s), "unpack")

    def _gather(self, recv, send):
        """Start the all-gather of recv <- send; returns the function that completes it."""
        if self._exchange_fn is not None:
            self._exchange_fn(recv, send)
            return lambda: None
        from .distributed import allgather_rows_start
        return allgather_rows_start(recv, send, self._group)

    # staged update for callers that drive the exchange themselves (tests, schedulers)
    def _stage_propagate(self, z):
        z = np.ascontiguousarray(torch.as_tensor(z, dtype=torch.float64).cpu().numpy().reshape(-1))
        self._sync_model()
        lib, h, s = _lib.load(), self._h, self._stream()
        _lib.check(lib.gpmdm_pf_switch(h, None, None, s), "switch")
        _lib.check(lib.gpmdm_pf_propagate(h, _lib.dptr(z), None, s), "propagate")
        _lib.check(lib.gpmdm_pf_pack(h, self._send.data_ptr(), s), "pack")
        return self._send

    def _stage_resample(self):
        lib, h, s = _lib.load(), self._h, self._stream()
        _lib.check(lib.gpmdm_pf_unpack(h, self._recv.data_ptr(), s), "unpack")
        _lib.check(lib.gpmdm_pf_resample(h, None, s), "resample")
        self._readout = None

    def _read(self):
        if self._readout is None:
            post, mean, lik = self._ro           # reused buffers: callers get copies
            _lib.check(_lib.load().gpmdm_pf_read(self._h, *self._ro_ptr, self._stream()), "read")
            self._readout = (post, mean, float(lik[0]))
        return self._readout

    def log_likelihood(self) -> float:
        """gpmdm_pf.py:215-222 (as in the reference: sum exp(ll + log_w - max), not a log)."""
        return self._read()[2]

    def class_probabilities(self) -> torch.Tensor:
        """gpmdm_pf.py:224-248."""
        return torch.from_numpy(self._read()[0].copy())

    def get_most_likely_class(self) -> int:
        """gpmdm_pf.py:250-254 (argmax, first maximum as torch.argmax; numpy on the cached
        read-out: no tensor round trip in the per-frame loop)."""
        return int(np.argmax(self._read()[0]))

    def current_state_mean(self) -> torch.Tensor:
        """gpmdm_pf.py:256-262."""
        return torch.from_numpy(self._read()[1].copy())

    def predict(self) -> torch.Tensor:
        """Dynamics-only one-step prediction of the latent mean: the average over the
        current particles of each particle's class dynamics-GP mean (gpmdm.py:1032-1068),
        computed on the device (gpmdm_pf_predict: class grouping, the dynamics GP tiles,
        a fixed-order mean).  Does not change the filter state and draws no random numbers."""
        self._sync_model()
        out = np.zeros(self.latent_dim)
        _lib.check(_lib.load().gpmdm_pf_predict(self._h, _lib.dptr(out), self._stream()), "predict")
        return torch.from_numpy(out)

    @property
    def frame(self) -> int:
        """Resamples done so far: the Philox counter of the next step's draws."""
        f = np.zeros(1, dtype=np.int64)
        _lib.check(_lib.load().gpmdm_pf_frame(self._h, _lib.i64ptr(f)), "frame")
        return int(f[0])

    def health(self, reset: bool = False) -> dict:
        """Failure counters since creation (or the last reset), per particle and step
        (SURVEY.md §5): non-positive observation / dynamics variances and non-finite
        log-likelihoods / states.  The arithmetic is the reference's (NaN propagates);
        these counts say when it happened."""
        n = np.zeros(len(_lib.HEALTH), dtype=np.int64)
        for h, s in self._all():                # devices=: each rank counts its own slice's events
            m = np.zeros(len(_lib.HEALTH), dtype=np.int64)
            _lib.check(_lib.load().gpmdm_pf_health(h, _lib.i64ptr(m), 1 if reset else 0, s), "health")
            n += m
        return {k: int(v) for k, v in zip(_lib.HEALTH, n)}

    # ---- introspection (tests, checkpoint of the filter state) --------------------
    def export_state(self) -> dict:
        P, d = self._num_particles, self.latent_dim
        out = dict(states=np.zeros((P, d)), classes=np.zeros(P, dtype=np.int64), ll=np.zeros(P),
                   log_w=np.zeros(P), w=np.zeros(P), resample_idx=np.zeros(P, dtype=np.int64))
        _lib.check(_lib.load().gpmdm_pf_export(
            self._h, _lib.dptr(out["states"]), _lib.i64ptr(out["classes"]), _lib.dptr(out["ll"]),
            _lib.dptr(out["log_w"]), _lib.dptr(out["w"]), _lib.i64ptr(out["resample_idx"]), self._stream()),
            "export")
        out["frame"] = self.frame
        out["seed"] = self._seed
        return out

    def load_state(self, states, classes, *, ll=None, log_w=None, w=None, resample_idx=None, frame=None):
        """Set the particle state.  With ``states``/``classes`` only: those particles with the
        reference's initial weights (ll = log_w = 0, w = 1/P; gpmdm_pf.py:100-104), e.g. a
        reference pre-step state.  With ``ll``, ``log_w`` and ``w`` as well (all three): the
        full filter state of ``export_state`` (gpmdm_pf.py:78-82) -- the read-outs right
        after are the exporter's, and the next updates continue its trajectory bit for bit
        (``resample_idx``: the ancestors of the last resample, optional; ``frame``: the
        Philox counter, optional; a replay filter's torch RNG state is the caller's to
        restore).  ``gpmdm_pf_import``."""
        self._sync_model()
        P = self._num_particles
        states = np.ascontiguousarray(states, dtype=np.float64).reshape(P, self.latent_dim)
        classes = np.ascontiguousarray(classes, dtype=np.int64).reshape(P)
        full = (ll, log_w, w)
        if all(x is None for x in full) and resample_idx is None and frame is None:
            for h in [self._h] + [p[0] for p in self._peers]:
                _lib.check(_lib.load().gpmdm_pf_init(h, _lib.dptr(states), _lib.i64ptr(classes)), "load_state")
        else:
            if any(x is None for x in full):
                raise ValueError("a full state import needs ll, log_w and w together")
            ll, log_w, w = (np.ascontiguousarray(x, dtype=np.float64).reshape(P) for x in full)
            ridx = None if resample_idx is None else np.ascontiguousarray(resample_idx, dtype=np.int64).reshape(P)
            for h in [self._h] + [p[0] for p in self._peers]:
                _lib.check(_lib.load().gpmdm_pf_import(
                    h, _lib.dptr(states), _lib.i64ptr(classes), _lib.dptr(ll), _lib.dptr(log_w), _lib.dptr(w),
                    _lib.i64ptr(ridx), -1 if frame is None else int(frame)), "load_state")
        self._readout = None

    def import_state(self, st: dict):
        """Restore an ``export_state()`` dict (a checkpoint of this filter or of one with
        the same configuration): ``load_state`` with every field it holds.  A Philox filter
        must have been built with the exporter's seed (checked)."""
        if self._rng == "philox" and "seed" in st and int(st["seed"]) != self._seed:
            raise ValueError("the state was exported by a filter with another Philox seed")
        self.load_state(st["states"], st["classes"], ll=st["ll"], log_w=st["log_w"], w=st["w"],
                        resample_idx=st.get("resample_idx"), frame=st.get("frame"))

    _CUT_SPLIT = {"auto": 0, "none": 1, "all": 2, "tail": 3, "chunks": 4}

    def set_obs_cutoff(self, on=True, stats: bool = False, split: str | None = None):
        """Run the observation GP with the model's kernel-value cutoff (GPMDM.enable_obs_cutoff,
        built here if needed) or the dense kernel; ``on="auto"``: per frame, the cutoff while
        the reach it measured on its last frame is below its break-even against the dense
        kernel, else the dense kernel (re-measured at least every 8 frames; one-rank filters,
        gpmdm_pf_set_obs_cutoff mode 3); ``stats`` also counts the MFMA groups run
        (obs_cutoff_stats; not with "auto"); ``split`` ("auto" default, "none", "all", "tail", "chunks")
        schedules the particle tiles run as two workgroups each (gpmdm_pf_set_obs_cutoff_split;
        the same results under every policy).  Between frames only."""
        if split is not None and split not in self._CUT_SPLIT:
            raise ValueError(f"split: one of {sorted(self._CUT_SPLIT)}")
        if isinstance(on, str) and on != "auto":
            raise ValueError("on: True, False or 'auto'")
        if on == "auto" and stats:
            raise ValueError("stats count the cutoff's work of every frame: not with on='auto'")
        if on:
            self._gpmdm.enable_obs_cutoff(True)
            self._sync_model()
        mode = 3 if on == "auto" else ((2 if stats else 1) if on else 0)
        lib = _lib.load()
        for h in [self._h] + [p[0] for p in self._peers]:
            _lib.check(lib.gpmdm_pf_set_obs_cutoff(h, mode), "set_obs_cutoff")
            if split is not None:
                _lib.check(lib.gpmdm_pf_set_obs_cutoff_split(h, self._CUT_SPLIT[split]), "set_obs_cutoff")
        self._obs_cutoff = mode

    def obs_cutoff_auto(self) -> dict:
        """AUTO cutoff state: whether the last frame ran the cutoff kernel, and the fraction of
        the dense MFMA work it ran on its last cutoff frame (None: not measured yet)."""
        last, frac = ctypes.c_int(), ctypes.c_double()
        _lib.check(_lib.load().gpmdm_pf_obs_cutoff_auto(self._h, ctypes.byref(last), ctypes.byref(frac)),
                   "obs_cutoff_auto")
        return {"last_frame_cutoff": bool(last.value), "fraction_run": frac.value if frac.value >= 0 else None}

    def obs_cutoff_stats(self, reset: bool = True) -> dict:
        """MFMA groups (16-particle x 16-column tile x 16-row K-step) the cutoff kernel ran since
        the last reset, against the dense kernel's count for the same launches."""
        lib = _lib.load()
        run, dense = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(lib.gpmdm_pf_obs_cutoff_stats(self._h, ctypes.byref(run), ctypes.byref(dense), 1 if reset else 0,
                                                 self._stream()), "obs_cutoff_stats")
        return {"run": run.value, "dense": dense.value,
                "fraction_run": run.value / dense.value if dense.value else None}

    def dynamics_rows(self) -> int:
        """Rows the last dynamics-GP pass evaluated (distinct ancestor/class keys when
        de-duplicating; this rank's particle count otherwise)."""
        r = np.zeros(1, dtype=np.int64)
        _lib.check(_lib.load().gpmdm_pf_dyn_rows(self._h, _lib.i64ptr(r), self._stream()), "dyn_rows")
        return int(r[0])

    def enable_timing(self, on: bool = True, stages=None):
        """Record per-stage HIP events (``stages``: names from ``_lib.STAGES``; default all).
        Each recorded stage adds two event records to the stream."""
        lib = _lib.load()
        names = _lib.STAGES if stages is None else tuple(stages)
        mask = 0
        for n in names:
            mask |= 1 << _lib.STAGES.index(n)
        _lib.check(lib.gpmdm_pf_timing_stages(self._h, mask))
        _lib.check(lib.gpmdm_pf_enable_timing(self._h, 1 if on else 0))

    def stage_times(self) -> dict:
        ms = np.zeros(len(_lib.STAGES))
        n = np.zeros(len(_lib.STAGES), dtype=np.int64)
        _lib.check(_lib.load().gpmdm_pf_stage_times(self._h, _lib.dptr(ms), _lib.i64ptr(n)))
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(_lib.STAGES)}

    # ---- properties (gpmdm_pf.py:267-285) ------------------------------------------
    @property
    def latent_dim(self):
        return self._gpmdm.d

    @property
    def observation_dim(self):
        return self._gpmdm.D

    @property
    def num_classes(self):
        return self._gpmdm.n_classes

    @property
    def dtype(self):
        return self._gpmdm.dtype

    @property
    def device(self):
        return self._gpmdm.device
