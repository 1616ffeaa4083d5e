import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def load_fixture(name):
    return dict(np.load(GOLDEN / f"{name}.npz", allow_pickle=False))


def seq_lengths(f):
    return [list(map(int, r)) for r in f["seq_lengths"]]


def oracle_model(f):
    from oracle import gpmdm_oracle as O
    return O.OracleModel(
        X=f["X"], Y=f["Y"].astype(np.float64), seq_lengths=seq_lengths(f),
        y_log_lengthscales=f["y_log_lengthscales"], y_log_lambdas=f["y_log_lambdas"],
        y_log_sigma_n=float(f["y_log_sigma_n"]), x_log_lengthscales=f["x_log_lengthscales"],
        x_log_lambdas=f["x_log_lambdas"], x_log_sigma_n=float(f["x_log_sigma_n"]),
        x_log_lin_coeff=f["x_log_lin_coeff"], sigma_n_num_X=float(f["sigma_n_num_X"]),
        sigma_n_num_Y=float(f["sigma_n_num_Y"])).precompute()


def y_sequences(f):
    Y = f["Y"]
    out, s = [], 0
    for lens in seq_lengths(f):
        cls = []
        for L in lens:
            cls.append(Y[s:s + L])
            s += L
        out.append(cls)
    return out


def product_model(f):
    from gpmdm_amd import GPMDM
    return GPMDM.from_arrays(
        f["X"], y_sequences(f), f["y_log_lengthscales"], f["y_log_lambdas"], float(f["y_log_sigma_n"]),
        f["x_log_lengthscales"], f["x_log_lambdas"], float(f["x_log_sigma_n"]), f["x_log_lin_coeff"],
        sigma_n_num_X=float(f["sigma_n_num_X"]), sigma_n_num_Y=float(f["sigma_n_num_Y"]))


def synthetic_model(C, d, D, L, S=3, seed=9):
    """A small random-hyperparameter GPMDM (C classes x S sequences x L frames), its Markov
    matrix and the stacked observations Y (host arrays)."""
    import torch
    from gpmdm_amd import GPMDM, synthetic
    data = synthetic.make_sequences(C=C, S=S, L=L, D=D, d=d, seed=seed)
    rng = np.random.RandomState(seed + 1)
    N = C * S * L
    X = rng.randn(N, d)
    lp = dict(y_log_lengthscales=np.log(rng.uniform(1.0, 2.5, d)), y_log_lambdas=np.log(rng.uniform(0.5, 2, D)),
              y_log_sigma_n=np.log(0.15), x_log_lengthscales=np.log(rng.uniform(1.0, 2.5, d)),
              x_log_lambdas=np.log(rng.uniform(0.5, 2, d)), x_log_sigma_n=np.log(0.12),
              x_log_lin_coeff=np.log(rng.uniform(0.2, 0.8, d + 1)))
    m = GPMDM.from_arrays(X, data.sequences, **lp)
    Y = np.concatenate([y for c in data.sequences for y in c]).astype(np.float64)
    return m, torch.tensor(synthetic.markov_matrix(C)), Y


def nrel(a, b):
    """max |a - b| / max |b| (normwise relative error)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


@pytest.fixture(scope="session")
def fx_config1():
    return load_fixture("config1_n500_p100_f200")


@pytest.fixture(scope="session")
def fx_config2():
    return load_fixture("config2_n2000_p1000")


@pytest.fixture(scope="session")
def fx_stress():
    return load_fixture("stress_n500_sigma001")
