"""CPU restatement of the device random draws of ``rng='philox'`` filters.

TEST INFRASTRUCTURE ONLY (like ``gpmdm_oracle``): imported by ``tests/`` and
``__graft_entry__.smoke()`` as the checker, never by the product path.

The reference draws from torch's CPU generator (``gpmdm_pf.py:150, 167-168, 211``); a
Philox filter replaces that generator with counter-based draws made on the GPU, so each
particle's numbers depend only on (seed, filter, frame, particle index, stream) and not on
how particles are sharded or grouped.  The transforms are the ones torch applies to its own
uniforms, so the sampling *semantics* of the reference are unchanged:

* class switch: ``torch.multinomial(p, 1)`` = ``argmax(p / E)`` with ``E ~ Exp(1)``;
  ``E = -log(u)``, ``u`` in (0, 1)  (``gpmdm_amd/csrc/pf_kernels.hip`` ``k_switch``);
* dynamics: ``torch.normal(mu, std)`` = ``mu + std * eps``; ``eps`` by Box-Muller from a
  (0, 1) and a [0, 1) uniform (``k_dyn_finish``);
* multinomial resample: one [0, 1) uniform per output slot (``k_resample``);
* systematic resample: one [0, 1) uniform per frame, ``u_s = (s + u0) / P``.

Philox4x32-10 is Salmon, Moraes, Dror & Shaw, "Parallel random numbers: as easy as 1, 2,
3" (SC'11): multipliers 0xD2511F53 / 0xCD9E8D57, Weyl key increments 0x9E3779B9 /
0xBB67AE85, ten rounds.  Counter layout (``gpmdm_amd/csrc/common.h``):
``(in-filter particle index, frame, stream, sub)`` with key = seed + filter index (64-bit,
split lo/hi), streams 0 switch, 1 dynamics, 2 resample, 3 systematic.  ``frame`` is the
number of resamples the handle has done (``gpmdm_pf_frame``).
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

STREAM_SWITCH, STREAM_DYN, STREAM_RESAMPLE, STREAM_SYSTEMATIC = 0, 1, 2, 3


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 over uint32 arrays (broadcasting); returns (x, y, z, w)."""
    c0, c1, c2, c3 = (np.asarray(v, dtype=np.uint32) for v in (c0, c1, c2, c3))
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & MASK32).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & MASK32).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = np.uint32(k0 + W0)
            k1 = np.uint32(k1 + W1)
    return c0, c1, c2, c3


def _u53(hi, lo):
    return ((hi.astype(np.uint64) << np.uint64(32)) | lo.astype(np.uint64)) >> np.uint64(11)


def u01_co(hi, lo):
    """[0, 1) from two 32-bit words (53 bits, exact in fp64)."""
    return _u53(hi, lo).astype(np.float64) * 2.0 ** -53


def u01_oo(hi, lo):
    """(0, 1) from two 32-bit words."""
    return (_u53(hi, lo).astype(np.float64) + 0.5) * 2.0 ** -53


def filter_key(seed: int, f: int = 0):
    """Key of filter f of a handle seeded with `seed` (a bank's filter f = seed + f)."""
    k = (int(seed) + int(f)) & (2 ** 64 - 1)
    return k & 0xFFFFFFFF, k >> 32


def switch_draws(seed: int, frame: int, P: int, C: int, f: int = 0) -> np.ndarray:
    """P x C Exp(1) draws of frame `frame` (k_switch): pair j//2 of particle p."""
    k0, k1 = filter_key(seed, f)
    p = np.arange(P, dtype=np.uint32)[:, None]
    sub = np.arange((C + 1) // 2, dtype=np.uint32)[None, :]
    x, y, z, w = philox4x32_10(p, np.uint32(frame), np.uint32(STREAM_SWITCH), sub, k0, k1)
    E = np.empty((P, 2 * sub.shape[1]))
    E[:, 0::2] = -np.log(u01_oo(x, y))
    E[:, 1::2] = -np.log(u01_oo(z, w))
    return E[:, :C]


def dynamics_normals(seed: int, frame: int, P: int, d: int, f: int = 0) -> np.ndarray:
    """P x d standard normals by particle index (k_dyn_finish's Box-Muller)."""
    k0, k1 = filter_key(seed, f)
    p = np.arange(P, dtype=np.uint32)[:, None]
    sub = np.arange((d + 1) // 2, dtype=np.uint32)[None, :]
    x, y, z, w = philox4x32_10(p, np.uint32(frame), np.uint32(STREAM_DYN), sub, k0, k1)
    u1, u2 = u01_oo(x, y), u01_co(z, w)
    rr = np.sqrt(-2.0 * np.log(u1))
    t = 6.283185307179586476925 * u2
    out = np.empty((P, 2 * sub.shape[1]))
    out[:, 0::2] = rr * np.cos(t)
    out[:, 1::2] = rr * np.sin(t)
    return out[:, :d]


def grouped_normals(normals_by_particle: np.ndarray, classes_switched: np.ndarray, C: int) -> np.ndarray:
    """Reorder per-particle draws into the class-grouped order ``propagate_dynamics``
    consumes (class by class, ascending particle index inside a class)."""
    order = np.concatenate([np.nonzero(classes_switched == c)[0] for c in range(C)])
    return normals_by_particle[order]


def resample_uniforms(seed: int, frame: int, P: int, f: int = 0) -> np.ndarray:
    """P [0, 1) uniforms of a multinomial resample (k_resample): one per output slot."""
    k0, k1 = filter_key(seed, f)
    s = np.arange(P, dtype=np.uint32)
    x, y, _, _ = philox4x32_10(s, np.uint32(frame), np.uint32(STREAM_RESAMPLE), np.uint32(0), k0, k1)
    return u01_co(x, y)


def systematic_u0(seed: int, frame: int, f: int = 0) -> float:
    """The single [0, 1) offset of a systematic resample."""
    k0, k1 = filter_key(seed, f)
    x, y, _, _ = philox4x32_10(np.uint32(0), np.uint32(frame), np.uint32(STREAM_SYSTEMATIC), np.uint32(0), k0, k1)
    return float(u01_co(np.atleast_1d(x), np.atleast_1d(y))[0])
