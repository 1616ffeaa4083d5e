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
