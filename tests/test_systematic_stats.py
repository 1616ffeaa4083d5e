"""Systematic resampling statistics: over many seeds at P = 10^4, the
error of the resampled moments (mean and variance of the states) against the weighted
moments they estimate, systematic versus the reference's multinomial resampling
(gpmdm_pf.py:211), on the oracle's resamplers (CPU).  The device's resamplers are checked
the same way in tests/test_gpu_systematic_stats.py."""
import numpy as np

from oracle import gpmdm_oracle as O

P, D_LAT, SEEDS = 10_000, 3, 200


def moment_errors(x, w, idx):
    m = w @ x
    v = w @ (x - m) ** 2
    xs = x[idx]
    mh = xs.mean(0)
    vh = ((xs - mh) ** 2).mean(0)
    return mh - m, vh - v


def resampled_mse(x, w, mode):
    em, ev = [], []
    for s in range(SEEDS):
        r = np.random.RandomState(1000 + s)
        if mode == "multinomial":
            idx = O.multinomial_resample_indices(w, r.rand(P))
        else:
            idx = O.systematic_resample_indices(w, r.rand())
        a, b = moment_errors(x, w, idx)
        em.append(a)
        ev.append(b)
    return float(np.mean(np.square(em))), float(np.mean(np.square(ev)))


def weighted_cloud(seed=0, sigma=0.3):
    """States of a cloud and likelihood weights of one observation (ESS ~ 5% of P)."""
    rng = np.random.RandomState(seed)
    x = rng.randn(P, D_LAT)
    ll = -0.5 * np.sum((x - np.array([0.5, -0.3, 0.2])) ** 2, 1) / sigma ** 2
    w = np.exp(ll - ll.max())
    return x, w / w.sum()


def test_systematic_moment_error_below_multinomial():
    x, w = weighted_cloud()
    mult = resampled_mse(x, w, "multinomial")
    sys_ = resampled_mse(x, w, "systematic")
    m = w @ x
    var_w = float(np.mean(w @ (x - m) ** 2))
    # multinomial: the resampled mean's error variance is Var_w(x) / P (iid draws)
    assert 0.8 < mult[0] / (var_w / P) < 1.25, (mult[0], var_w / P)
    # systematic (one uniform, stratified slots): measured 0.09 (mean) and 0.17 (variance)
    # of multinomial's squared error on this cloud
    assert sys_[0] < 0.2 * mult[0], (sys_, mult)
    assert sys_[1] < 0.35 * mult[1], (sys_, mult)


def test_systematic_offspring_bounds():
    """Each particle gets floor(P w_i) or ceil(P w_i) offspring (up to the CDF's last-ulp
    rounding at a boundary), every seed."""
    x, w = weighted_cloud(seed=1)
    for s in range(20):
        idx = O.systematic_resample_indices(w, np.random.RandomState(s).rand())
        n = np.bincount(idx, minlength=P)
        assert np.all(n >= np.floor(P * w) - 1) and np.all(n <= np.ceil(P * w) + 1)
        assert int(np.sum(n)) == P
