"""GPU: the device's systematic resampler against its multinomial one,
statistically, on real filter weights.

Two banks of F filters x P = 10^4 particles with the same seeds take one step from the
same initial particles: their switch and dynamics draws are the same Philox streams, so
their pre-resample weights are bit-identical and only the resampler differs.  For a
function f of the particle index that is uncorrelated with the particles' order (a hash),
the resampled mean (1/P) sum_s f(a_s) estimates sum_i w_i f(i); over the F filters the
systematic resampler's squared error must be well below the multinomial one's, which must
match the iid value Var_w(f) / P.  The CPU counterpart on the oracle's resamplers is
tests/test_systematic_stats.py."""
import numpy as np
import pytest
import torch

from conftest import load_fixture

pytestmark = pytest.mark.gpu

F, P = 96, 10_000


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
    Z = np.stack([np.asarray(Y[(7 * f) % Y.shape[0]], dtype=np.float64) + 0.05 for f in range(F)])
    out = {}
    for mode in ("multinomial", "systematic"):
        bank = GPMDM_PF_Bank(m, T, F, P, seed=77, resample=mode)
        bank.update(Z)
        out[mode] = bank.export_state()
    wm, ws = out["multinomial"]["w"], out["systematic"]["w"]
    assert np.array_equal(wm, ws)             # same draws before the resampler
    fi = _f(np.arange(P))
    err = {}
    var_ratio = []
    for mode in ("multinomial", "systematic"):
        e = []
        for k in range(F):
            w = out[mode]["w"][k]
            idx = out[mode]["resample_idx"][k]
            mu = float(w @ fi)
            e.append(float(np.mean(fi[idx])) - mu)
            if mode == "multinomial":
                var_ratio.append(float(w @ (fi - mu) ** 2) / P)
        err[mode] = float(np.mean(np.square(e)))
    iid = float(np.mean(var_ratio))
    ess = float(np.mean([1.0 / np.sum(w * w) for w in wm]))
    assert ess > 20, ess                      # a cloud with something to resample
    assert 0.6 < err["multinomial"] / iid < 1.6, (err, iid)
    assert err["systematic"] < 0.5 * err["multinomial"], (err, ess)
    print(f"ESS {ess:.1f}; squared error of the resampled mean: multinomial {err['multinomial']:.3e} "
          f"(iid {iid:.3e}), systematic {err['systematic']:.3e}, ratio {err['systematic'] / err['multinomial']:.3f}")
