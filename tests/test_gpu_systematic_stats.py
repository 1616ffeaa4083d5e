"""GPU: the device's systematic resampler against its multinomial one,
statistically, on real filter weights.

Two banks of F filters x P = 10^4 particles (one multinomial, one systematic) follow the
same observation streams for a few frames.  For a function f of the particle index that
is uncorrelated with the particles' order (a hash), the last resample's mean
(1/P) sum_s f(a_s) estimates sum_i w_i f(i) of its own pre-resample weights; over the F
filters the multinomial resampler's squared error must match the iid value Var_w(f) / P,
and the systematic resampler's (relative to its own iid value) must be well below it.
The CPU counterpart on the oracle's resamplers is tests/test_systematic_stats.py."""
import numpy as np
import pytest
import torch

from conftest import load_fixture

pytestmark = pytest.mark.gpu

F, P, STEPS = 96, 10_000, 4


def _f(i):
    v = np.sin(12.9898 * i.astype(np.float64) + 78.233) * 43758.5453
    return v - np.floor(v)                    # in [0, 1), no relation to the index order


def test_systematic_moment_error_on_device_weights():
    from gpmdm_amd import GPMDM, GPMDM_PF_Bank
    from conftest import y_sequences
    fx = load_fixture("config1_n500_p100_f200")
    # the config-1 model with output scales exp(y_log_lambdas) x 0.05 (bench.py's spread line):
    # a less peaked likelihood, so one step leaves a cloud with an ESS worth resampling
    m = GPMDM.from_arrays(
        fx["X"], y_sequences(fx), fx["y_log_lengthscales"], fx["y_log_lambdas"] + np.log(0.05),
        float(fx["y_log_sigma_n"]), fx["x_log_lengthscales"], fx["x_log_lambdas"], float(fx["x_log_sigma_n"]),
        fx["x_log_lin_coeff"], sigma_n_num_X=float(fx["sigma_n_num_X"]), sigma_n_num_Y=float(fx["sigma_n_num_Y"]))
    T = torch.tensor(fx["T"])
    Y = m.get_Y()
    n = Y.shape[0]
    out = {}
    for mode in ("multinomial", "systematic"):
        bank = GPMDM_PF_Bank(m, T, F, P, seed=77, resample=mode)
        for k in range(STEPS):                 # filter f follows the training frames from 5 f
            bank.update(np.stack([np.asarray(Y[(5 * f + k) % n], dtype=np.float64) + 0.05 for f in range(F)]))
        out[mode] = bank.export_state()
    fi = _f(np.arange(P))
    # squared error of the resampled mean of f over the filters, and the iid (multinomial)
    # value Var_w(f) / P of each filter's own weights
    err, iid, ess = {}, {}, {}
    for mode in ("multinomial", "systematic"):
        e, v = [], []
        for k in range(F):
            w = out[mode]["w"][k]
            idx = out[mode]["resample_idx"][k]
            mu = float(w @ fi)
            e.append(float(np.mean(fi[idx])) - mu)
            v.append(float(w @ (fi - mu) ** 2) / P)
        err[mode], iid[mode] = float(np.mean(np.square(e))), float(np.mean(v))
        ess[mode] = float(np.mean([1.0 / np.sum(w * w) for w in out[mode]["w"]]))
    rel = {k: err[k] / iid[k] for k in err}
    print(f"ESS {ess}; squared error of the resampled mean / iid value: {rel}; "
          f"ratio systematic / multinomial {rel['systematic'] / rel['multinomial']:.3f}")
    assert min(ess.values()) > 2, ess         # a cloud with something to resample
    assert 0.6 < rel["multinomial"] < 1.6, (err, iid)
    assert rel["systematic"] < 0.5 * rel["multinomial"], (rel, ess)
