"""GPMDM_PF_Bank -- many independent particle filters sharing one GPMDM.

The reference runs one ``GPMDM_PF`` per observation stream, one after another (the 39
trials of ``test_gpmdm_pf.ipynb`` cell 4, each a fresh filter over the same model;
SURVEY.md §8(f) row 3).  A bank runs F such filters as one device computation: the
dynamics and observation GP tile kernels see all F x P particles at once (filling the
GPU at the notebooks' P = 100), while normalisation, resampling and the read-outs run
per filter.  Every filter keeps the reference's per-filter semantics
(``gpmdm_pf.py:117-262``).

Draws come from the device (Philox).  Filter f is keyed with ``seed + f``, so its
trajectory is bit-identical to a single ``GPMDM_PF(..., rng='philox', seed=seed + f)``
started from the same particles; the bank changes the schedule, not the numbers.

With a ``process_group`` the filters are sharded over ranks (rank r owns filters
``[r F / R, (r + 1) F / R)``, the particle-shard rule of ``gpmdm_pf_create``).  Filters
are independent, so the step needs no collective at all; ``gather_readouts()`` is the
only exchange and is optional.  ``shard=(world, rank)`` selects the same slice without a
process group.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib, replay
from .distributed import shard_range
from .model import GPMDM


class GPMDM_PF_Bank:
    def __init__(self, gpmdm: GPMDM, markov_switching_model, num_filters: int, num_particles: int, *,
                 seed=None, resample: str = "multinomial", process_group=None, shard=None,
                 dedup: bool = True, dyn_tiles: str = "auto", obs_cutoff: bool = False):
        self._gpmdm = gpmdm
        self._gpmdm.set_evaluation_mode()
        self._T = torch.as_tensor(markov_switching_model).type(torch.float64)
        if self._gpmdm.n_classes != self._T.size(0):
            raise ValueError("Number of classes in the GPMDM model and the Markov model do not match")
        if resample not in ("multinomial", "systematic"):
            raise ValueError("resample must be 'multinomial' or 'systematic'")
        self._num_filters = int(num_filters)
        self._num_particles = int(num_particles)
        if self._num_filters < 1 or self._num_particles < 1:
            raise ValueError("num_filters and num_particles must be positive")
        self._group = process_group
        if process_group is not None:
            import torch.distributed as dist
            world, rank = dist.get_world_size(process_group), dist.get_rank(process_group)
        elif shard is not None:                   # (world, rank) without a process group
            world, rank = int(shard[0]), int(shard[1])
            if world > 1 and seed is None:
                raise ValueError("shard= needs an explicit seed (identical on every rank)")
        else:
            world, rank = 1, 0
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        if process_group is not None and world > 1:   # one seed for the whole bank: rank 0's
            from .distributed import broadcast_array
            seed = int(broadcast_array(np.array([seed], dtype=np.int64), process_group, self.device)[0])
        self._seed = int(seed)
        self._world, self._rank = world, rank
        self._f_lo, self._f_hi = shard_range(self._num_filters, world, rank)
        self._h = None
        self._readout = None
        if obs_cutoff:
            gpmdm.enable_obs_cutoff(True)     # the model's cutoff image (built once)
        if self.local_filters > 0:
            T = np.ascontiguousarray(self._T.numpy(), dtype=np.float64)
            h = ctypes.c_void_p()
            _lib.check(_lib.load().gpmdm_bank_create(
                gpmdm.handle, _lib.dptr(T), self.local_filters, self._num_particles,
                ctypes.c_uint64((self._seed + self._f_lo) & (2 ** 64 - 1)),
                _lib.GPMDM_RESAMPLE_MULTINOMIAL if resample == "multinomial" else _lib.GPMDM_RESAMPLE_SYSTEMATIC,
                ctypes.byref(h)), "GPMDM_PF_Bank")
            self._h = h
            self._model_gen = gpmdm.generation
            _lib.check(_lib.load().gpmdm_pf_set_dedup(h, 1 if dedup else 0), "dedup")
            if dyn_tiles not in _lib.DYN_TILES:
                raise ValueError("dyn_tiles must be 'auto', 'narrow' or 'wide'")
            _lib.check(_lib.load().gpmdm_pf_set_dyn_tiles(h, _lib.DYN_TILES[dyn_tiles]), "dyn_tiles")
            if obs_cutoff:                    # the observation GP's kernel-value cutoff (GPMDM_PF's)
                _lib.check(_lib.load().gpmdm_pf_set_obs_cutoff(h, 1), "obs_cutoff")
            self._init_particles()

    def __del__(self):
        try:
            if getattr(self, "_h", None) is not None and self._h.value:
                _lib.load().gpmdm_pf_destroy(self._h)
                self._h = None
        except Exception:
            pass

    def _stream(self):
        dev = self.device
        return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(dev.index if dev.index is not None
                                                                   else torch.cuda.current_device()))

    def _sync_model(self):
        """Rebind to the GPMDM's current device image (see GPMDM_PF._sync_model)."""
        self._gpmdm._refresh()
        if self._h is not None and self._gpmdm.generation != self._model_gen:
            _lib.check(_lib.load().gpmdm_pf_set_model(self._h, self._gpmdm.handle), "rebind to the rebuilt model")
            self._model_gen = self._gpmdm.generation

    # ---- state ----------------------------------------------------------------------
    def _init_particles(self):
        """gpmdm_pf.py:87-115 for every local filter.  Filter f's initial draws come from a
        generator seeded with seed + f, so they do not depend on the rank count."""
        C, P = self.num_classes, self._num_particles
        g, r = divmod(P, C)
        counts = [g + (1 if i < r else 0) for i in range(C)]
        Xc = [self._gpmdm.get_X_for_class(c).detach().cpu().numpy() for c in range(C)]
        sizes = [x.shape[0] for x in Xc]
        states, classes = [], []
        for f in range(self._f_lo, self._f_hi):
            gen = torch.Generator().manual_seed(self._seed + f)
            idx = replay.init_draws(sizes, counts, generator=gen)
            states.append(np.concatenate([Xc[c][idx[c]] for c in range(C)], 0))
            classes.append(np.concatenate([np.full(counts[c], c, dtype=np.int64) for c in range(C)]))
        self.load_state(np.stack(states), np.stack(classes))

    def reset(self):
        if self._h is not None:
            self._init_particles()

    def load_state(self, states, classes, *, ll=None, log_w=None, w=None, resample_idx=None, frame=None):
        """states (F_local, P, d), classes (F_local, P); with ll / log_w / w (F_local, P) the
        full state of ``export_state`` (GPMDM_PF.load_state; gpmdm_pf_import)."""
        Fl, P, d = self.local_filters, self._num_particles, self.latent_dim
        states = np.ascontiguousarray(states, dtype=np.float64).reshape(Fl * P, d)
        classes = np.ascontiguousarray(classes, dtype=np.int64).reshape(Fl * P)
        self._sync_model()
        full = (ll, log_w, w)
        if all(x is None for x in full) and resample_idx is None and frame is None:
            _lib.check(_lib.load().gpmdm_pf_init(self._h, _lib.dptr(states), _lib.i64ptr(classes)), "load_state")
        else:
            if any(x is None for x in full):
                raise ValueError("a full state import needs ll, log_w and w together")
            ll, log_w, w = (np.ascontiguousarray(x, dtype=np.float64).reshape(Fl * P) for x in full)
            ridx = None if resample_idx is None else np.ascontiguousarray(resample_idx, dtype=np.int64).reshape(Fl * P)
            _lib.check(_lib.load().gpmdm_pf_import(
                self._h, _lib.dptr(states), _lib.i64ptr(classes), _lib.dptr(ll), _lib.dptr(log_w), _lib.dptr(w),
                _lib.i64ptr(ridx), -1 if frame is None else int(frame)), "load_state")
        self._readout = None

    def import_state(self, st: dict):
        """Restore an ``export_state()`` dict (same filters, same seed: checked)."""
        if "seed" in st and int(st["seed"]) != self._seed:
            raise ValueError("the state was exported by a bank with another seed")
        self.load_state(st["states"], st["classes"], ll=st["ll"], log_w=st["log_w"], w=st["w"],
                        resample_idx=st.get("resample_idx"), frame=st.get("frame"))

    def export_state(self) -> dict:
        Fl, P, d = self.local_filters, self._num_particles, self.latent_dim
        n = Fl * P
        out = dict(states=np.zeros((n, d)), classes=np.zeros(n, dtype=np.int64), ll=np.zeros(n),
                   log_w=np.zeros(n), w=np.zeros(n), resample_idx=np.zeros(n, dtype=np.int64))
        _lib.check(_lib.load().gpmdm_pf_export(
            self._h, _lib.dptr(out["states"]), _lib.i64ptr(out["classes"]), _lib.dptr(out["ll"]),
            _lib.dptr(out["log_w"]), _lib.dptr(out["w"]), _lib.i64ptr(out["resample_idx"]), self._stream()),
            "export")
        out["states"] = out["states"].reshape(Fl, P, d)
        for k in ("classes", "ll", "log_w", "w", "resample_idx"):
            out[k] = out[k].reshape(Fl, P)
        out["frame"] = self.frame
        out["seed"] = self._seed
        return out

    # ---- per-frame ------------------------------------------------------------------
    def update(self, Z):
        """One frame for every filter.  Z: (F, D) (all filters; each rank takes its rows)
        or (F_local, D)."""
        Z = np.asarray(torch.as_tensor(Z, dtype=torch.float64).cpu().numpy(), dtype=np.float64)
        Z = Z.reshape(-1, self.observation_dim)
        if Z.shape[0] == self._num_filters and self.local_filters != self._num_filters:
            Z = Z[self._f_lo:self._f_hi]
        if Z.shape[0] != self.local_filters:
            raise ValueError(f"expected {self._num_filters} (or {self.local_filters} local) observations, "
                             f"got {Z.shape[0]}")
        self._readout = None
        if self._h is None:
            return
        Z = np.ascontiguousarray(Z)
        self._sync_model()
        lib, h, s = _lib.load(), self._h, self._stream()
        _lib.check(lib.gpmdm_pf_switch(h, None, None, s), "switch")
        _lib.check(lib.gpmdm_pf_propagate(h, _lib.dptr(Z), None, s), "propagate")
        _lib.check(lib.gpmdm_pf_resample(h, None, s), "resample")

    step = update

    def _read(self):
        if self._readout is None:
            Fl, C, d = self.local_filters, self.num_classes, self.latent_dim
            post, mean, lik = np.zeros((Fl, C)), np.zeros((Fl, d)), np.zeros(Fl)
            if self._h is not None:
                _lib.check(_lib.load().gpmdm_pf_read(self._h, _lib.dptr(post), _lib.dptr(mean), _lib.dptr(lik),
                                                     self._stream()), "read")
            self._readout = (post, mean, lik)
        return self._readout

    def class_probabilities(self) -> torch.Tensor:
        """(F_local, C): gpmdm_pf.py:224-248 per filter."""
        return torch.tensor(self._read()[0], dtype=torch.float64)

    def get_most_likely_class(self) -> torch.Tensor:
        """(F_local,): gpmdm_pf.py:250-254 per filter (first maximum)."""
        return torch.argmax(self.class_probabilities(), dim=1)

    def current_state_mean(self) -> torch.Tensor:
        """(F_local, d): gpmdm_pf.py:256-262 per filter."""
        return torch.tensor(self._read()[1], dtype=torch.float64)

    def log_likelihood(self) -> torch.Tensor:
        """(F_local,): gpmdm_pf.py:215-222 per filter (a sum of exponentials, as there)."""
        return torch.tensor(self._read()[2], dtype=torch.float64)

    def predict(self) -> torch.Tensor:
        """(F_local, d): GPMDM_PF.predict per filter (gpmdm_pf_predict)."""
        out = np.zeros((self.local_filters, self.latent_dim))
        if self._h is not None:
            self._sync_model()
            _lib.check(_lib.load().gpmdm_pf_predict(self._h, _lib.dptr(out), self._stream()), "predict")
        return torch.from_numpy(out)

    def gather_readouts(self) -> dict:
        """All filters' read-outs on every rank (one all-gather of F x (C + d + 1))."""
        post, mean, lik = self._read()
        rows = np.concatenate([post, mean, lik[:, None]], 1)
        if self._group is None:
            full = rows
        else:
            import torch.distributed as dist
            from .distributed import allgather_rows
            dev = self.device if dist.get_backend(self._group) != "gloo" else torch.device("cpu")
            send = torch.as_tensor(rows, dtype=torch.float64, device=dev)
            recv = torch.empty((self._num_filters, rows.shape[1]), dtype=torch.float64, device=dev)
            allgather_rows(recv, send, self._group)
            full = recv.cpu().numpy()
        C, d = self.num_classes, self.latent_dim
        return dict(class_probabilities=torch.tensor(full[:, :C]),
                    current_state_mean=torch.tensor(full[:, C:C + d]),
                    log_likelihood=torch.tensor(full[:, C + d]))

    # ---- properties -----------------------------------------------------------------
    @property
    def frame(self) -> int:
        """Resamples done so far (every filter of the bank steps together)."""
        f = np.zeros(1, dtype=np.int64)
        if self._h is not None:
            _lib.check(_lib.load().gpmdm_pf_frame(self._h, _lib.i64ptr(f)), "frame")
        return int(f[0])

    @property
    def num_filters(self):
        return self._num_filters

    @property
    def local_filters(self):
        return self._f_hi - self._f_lo

    @property
    def filter_range(self):
        return self._f_lo, self._f_hi

    @property
    def num_particles(self):
        return self._num_particles

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
