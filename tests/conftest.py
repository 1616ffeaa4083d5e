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


# Resample-index ties observed against the oracle's search (how many of
# the allowed <= 2 last-ulp CDF ties actually occur): every comparison is recorded and the
# session writes them to gpurun_out/resample_ties.json (the GPU box's output directory).
TIE_LOG = []


def record_ties(what, P, n):
    TIE_LOG.append({"test": what, "P": int(P), "ties": int(n)})


def pytest_sessionfinish(session, exitstatus):
    if TIE_LOG:
        import json
        out = ROOT / "gpurun_out"
        out.mkdir(exist_ok=True)
        (out / "resample_ties.json").write_text(json.dumps(
            {"comparisons": len(TIE_LOG), "with_ties": sum(1 for t in TIE_LOG if t["ties"]),
             "max_ties": max(t["ties"] for t in TIE_LOG), "records": TIE_LOG}, indent=1))


def assert_step_matches(post, r, gpu_post, gpu_mean, u, resample="multinomial", what="", w_tol=1e-5):
    """A GPU filter step (``post`` = export after it, read-outs ``gpu_post``/``gpu_mean``)
    against the oracle's step ``r`` from the same pre-step particles and draws.

    Every stage is compared given the previous one: weights against the oracle's (1e-5
    normwise); the resample indices against the oracle's inverse-CDF search of the GPU's
    own weights with the same uniforms (exact up to 2 last-ulp CDF ties: the device scans
    in another association order than numpy's cumsum); post-resample states / classes and
    the read-outs against the oracle's propagated states, switched classes and read-out
    formulas at the GPU's indices.  (Comparing indices searched in two independently
    computed CDFs is not a parity statement at large P: a 1e-12 relative weight
    difference moves ~P^2 x 1e-12 / 2 slots across a boundary.)"""
    from oracle import gpmdm_oracle as O
    idx = post["resample_idx"]
    assert nrel(post["w"], r.w) < w_tol, (what, nrel(post["w"], r.w))
    if resample == "multinomial":
        ref_idx = O.multinomial_resample_indices(post["w"], u)
    else:
        ref_idx = O.systematic_resample_indices(post["w"], float(np.asarray(u).reshape(-1)[0]))
    ties = int(np.sum(ref_idx != idx))
    record_ties(what or "assert_step_matches", len(idx), ties)
    assert ties <= 2, (what, ties)
    assert np.array_equal(post["classes"], r.classes_switched[idx]), what
    assert nrel(post["states"], r.states_propagated[idx]) < 1e-6, what
    C = len(r.posterior)
    ref_post = O.class_probabilities(r.ll, r.log_w, r.classes_switched[idx], C)
    ref_mean = O.current_state_mean(r.states_propagated[idx], r.w)
    assert np.max(np.abs(gpu_post - ref_post)) < 1e-6, what
    assert nrel(gpu_mean, ref_mean) < 1e-6, what
    return int(np.sum(r.resample_idx != idx))
