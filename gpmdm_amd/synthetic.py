"""Synthetic GPMDM workloads of the shape BASELINE.json names.

There is no network and the CMU mocap set is not shipped with the reference
(`/root/reference/README.md` "mocap: Not included"), so every model and observation
stream here is synthetic:

* per class ``c`` there are ``S`` sequences of length ``L`` (``N = C*S*L``);
* latent phase ``t_k = k * 0.1 * (1 + c) + phi_s`` with ``phi_s ~ U(0, 2*pi)``;
* features ``F = [sin(t + j)]_{j < 2d}``, observations ``Y = tanh(F W) + 0.05 eps``
  with ``W ~ N(0, 1)^{2d x D}``, cast to float32 as the notebooks feed them
  (`notebooks/test_gpmdm_pf.ipynb`, ``to_numpy(dtype=np.float32)``);
* the observation stream is ``z_f = Y_seq0[f mod L] + 0.05 N(0, 1)``.

Hyperparameters follow SURVEY §8(d): unit lengthscales, lambdas and linear
coefficients, ``sigma_n = 0.1`` for both GPs, ``sigma_n_num = 0``, ``dyn_target='full'``,
``dyn_back_step=1``; the Markov matrix has 0.9 on the diagonal.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

# The five workloads of BASELINE.json "configs" (S sequences of length L per class).
CONFIGS = {
    1: dict(C=2, S=5, L=50, D=62, d=3, P=100, frames=200),
    2: dict(C=2, S=5, L=200, D=62, d=3, P=100_000, frames=500),
    3: dict(C=5, S=5, L=400, D=128, d=8, P=100_000, frames=500),
    4: dict(C=2, S=5, L=200, D=62, d=3, P=1_000_000, frames=500),
    5: dict(C=8, S=5, L=500, D=256, d=16, P=1_000_000, frames=500),
}


@dataclass
class SyntheticData:
    sequences: list          # sequences[c] = list of (L, D) float32 arrays
    D: int
    d: int
    n_classes: int

    def observation_stream(self, frames: int, seed: int = 1, noise: float = 0.05) -> np.ndarray:
        """``z_f = Y_seq0[f mod L] + noise * N(0,1)`` as float32 (frames x D)."""
        rng = np.random.RandomState(seed)
        y0 = self.sequences[0][0]
        L = y0.shape[0]
        idx = np.arange(frames) % L
        z = y0[idx].astype(np.float64) + noise * rng.randn(frames, self.D)
        return z.astype(np.float32)


def make_sequences(C: int, S: int, L: int, D: int, d: int, seed: int = 0) -> SyntheticData:
    rng = np.random.RandomState(seed)
    W = rng.randn(2 * d, D)
    seqs = []
    for c in range(C):
        cls = []
        for _ in range(S):
            phi = rng.uniform(0.0, 2.0 * np.pi)
            t = np.arange(L) * 0.1 * (1 + c) + phi
            F = np.sin(t[:, None] + np.arange(2 * d)[None, :])
            Y = np.tanh(F @ W) + 0.05 * rng.randn(L, D)
            cls.append(Y.astype(np.float32))
        seqs.append(cls)
    return SyntheticData(seqs, D, d, C)


def markov_matrix(C: int, stay: float = 0.9) -> np.ndarray:
    if C == 1:
        return np.ones((1, 1))
    T = np.full((C, C), (1.0 - stay) / (C - 1))
    np.fill_diagonal(T, stay)
    return T


def default_hyperparameters(D: int, d: int, sigma_n: float = 0.1) -> dict:
    """Constructor initialisers of the reference GPMDM (`gpmdm.py:96-109`)."""
    return dict(
        y_lambdas_init=np.ones(D),
        y_lengthscales_init=np.ones(d),
        y_sigma_n_init=sigma_n,
        x_lambdas_init=np.ones(d),
        x_lengthscales_init=np.ones(d),
        x_sigma_n_init=sigma_n,
        x_lin_coeff_init=np.ones(d + 1),
    )
