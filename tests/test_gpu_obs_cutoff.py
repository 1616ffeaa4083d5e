"""The observation GP's opt-in kernel-value cutoff (``GPMDM_PF(..., obs_cutoff=True)``,
DESIGN.md §3 "Kernel-value cutoff"): kernel values k_i = exp(-|x - X_i|^2 / l^2) below the
model's tau are flushed to exactly 0 and the MFMAs of the 16-row K-steps a particle tile
cannot reach are skipped (gpmdm.py:923-963 / gpmdm_pf.py:170-192 otherwise unchanged).

Checked at the dense filter's tolerances:
  * the reference's golden vectors: config-1 per-step parity over 200 frames, the 200-frame
    torch-seeded trajectory, the N = 2000 per-step fixture (tests/golden, make_golden.py);
  * the oracle: three resynced Philox steps at the benchmarked P = 100k (config 2);
  * tiling / shard invariance: 4 and 8 logical shards bitwise equal one rank (the flush is
    per value, and a skipped K-step or column tile contributes only exact zeros);
  * against the dense kernel from the same state with the same draws (the two evaluate
    k^T K^-1 k in different associations: symmetric K^-1 vs |R^T k|^2);
  * tau equals the bound restated here (host_image.h obs_cutoff_tau), and the kernel skips
    work on the benchmark's collapsed cloud.
"""
import numpy as np
import pytest
import torch

from conftest import assert_step_matches, nrel, oracle_model, product_model

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def m1c(fx_config1):
    m = product_model(fx_config1)
    m.enable_obs_cutoff(True)
    return m


@pytest.fixture(scope="module")
def m2c(fx_config2):
    m = product_model(fx_config2)
    m.enable_obs_cutoff(True)
    return m


def _tau_bound(m):
    """host_image.h obs_cutoff_tau restated: min(tau_q, tau_mu)."""
    Y = np.asarray(m.get_Y(), dtype=np.float64)
    N = Y.shape[0]
    sigma2 = float(torch.exp(m.y_log_sigma_n.detach().cpu())) ** 2 + m.sigma_n_num_Y ** 2
    vc_min = sigma2 / (N + sigma2)
    h = 0.5 * (np.nextafter(vc_min, 1.0) - vc_min)
    tau = np.sqrt(sigma2) * h / (2.001 * np.sqrt(N))
    X = m.X.detach().cpu().numpy()
    ls = np.exp(m.y_log_lengthscales.detach().cpu().numpy())
    from oracle import gpmdm_oracle as O
    K = O.rbf_kernel(X, X, np.log(ls), float(m.y_log_sigma_n.detach().cpu()), m.sigma_n_num_Y, noise=True)
    beta = np.linalg.solve(K, Y)
    for j in range(Y.shape[1]):
        m1 = np.sum(np.abs(beta[:, j]))
        y = np.max(np.abs(Y[:, j]))
        tau = min(tau, 0.5 * (np.nextafter(y, np.inf) - y) / m1)
    return tau


def test_tau_is_the_bound(m2c):
    # beta from a fresh solve here, the library's from the precompute: the mean bound moves
    # with |beta_j|_1 at the 1e-9 level
    t = m2c.obs_cutoff_tau
    assert t > 0
    assert abs(t - _tau_bound(m2c)) <= 1e-6 * t, (t, _tau_bound(m2c))


def _per_step_cutoff(m, f, pre, z_offset=0):
    from gpmdm_amd import GPMDM_PF
    P = f[pre + "E"].shape[1]
    pf = GPMDM_PF(m, torch.tensor(f["T"]), P, rng="torch", obs_cutoff=True)
    worst = {}
    for k in range(f[pre + "E"].shape[0]):
        pf.load_state(f[pre + "pre_states"][k], f[pre + "pre_classes"][k])
        pf.update_with_draws(f["z"][k + z_offset], f[pre + "E"][k], f[pre + "normals"][k], f[pre + "u"][k])
        st = pf.export_state()
        assert np.array_equal(st["classes"], f[pre + "classes"][k].reshape(-1)), f"frame {k}: classes"
        err = {"states": nrel(st["states"], f[pre + "states"][k]), "w": nrel(st["w"], f[pre + "w"][k]),
               "post": float(np.max(np.abs(pf.class_probabilities().numpy() - f[pre + "posterior"][k]))),
               "mean": nrel(pf.current_state_mean().numpy(), f[pre + "mean"][k]),
               "lik": abs(pf.log_likelihood() - f[pre + "lik"][k]) / abs(f[pre + "lik"][k])}
        assert pf.get_most_likely_class() == int(f[pre + "most_likely"][k])
        for key, v in err.items():
            worst[key] = max(worst.get(key, 0.0), v)
    assert worst["states"] < 1e-6, worst
    assert worst["w"] < 1e-5, worst
    assert worst["post"] < 1e-6, worst
    assert worst["mean"] < 1e-6, worst
    assert worst["lik"] < 1e-5, worst
    return worst


def test_step_parity_config1_cutoff(m1c, fx_config1):
    _per_step_cutoff(m1c, fx_config1, "traj_")


def test_step_parity_config2_p1000_cutoff(m2c, fx_config2):
    f = fx_config2
    _per_step_cutoff(m2c, f, "step_", z_offset=f["z"].shape[0] - f["step_E"].shape[0])


def test_trajectory_config1_cutoff(m1c, fx_config1):
    """The 200-frame torch-seeded trajectory of the reference (test_gpu_parity.py's dense
    test) with the cutoff: same classes, posterior and mean to 1e-5."""
    from gpmdm_amd import GPMDM_PF
    f = fx_config1
    torch.manual_seed(11)
    pf = GPMDM_PF(m1c, torch.tensor(f["T"]), 100, obs_cutoff=True)
    wp = wm = 0.0
    for k in range(200):
        pf.update(f["z"][k])
        assert pf.get_most_likely_class() == int(f["traj_most_likely"][k])
        wp = max(wp, float(np.max(np.abs(pf.class_probabilities().numpy() - f["traj_posterior"][k]))))
        wm = max(wm, nrel(pf.current_state_mean().numpy(), f["traj_mean"][k]))
    assert wp < 1e-5 and wm < 1e-5, (wp, wm)


def test_philox_steps_cutoff_vs_oracle(m2c, fx_config2):
    """The benchmarked configuration (config-2 model, P = 100k, Philox, multinomial): three
    resynced steps after a warm-up step against the oracle (conftest.assert_step_matches:
    weights 1e-5, indices of the GPU's weights exact up to 2 ties, states / read-outs 1e-6)."""
    from gpmdm_amd import GPMDM_PF
    from oracle import gpmdm_oracle as O
    from oracle import philox as X
    om = oracle_model(fx_config2)
    T = np.asarray(fx_config2["T"], dtype=np.float64)
    P, seed = 100_000, 11
    pf = GPMDM_PF(m2c, torch.tensor(T), P, rng="philox", seed=seed, obs_cutoff=True)
    Y = m2c.get_Y()
    pf.update(Y[10])
    for k in range(3):
        pre = pf.export_state()
        frame = pf.frame
        z = Y[11 + k] + 0.01
        pf.update(z)
        post = pf.export_state()
        E = X.switch_draws(seed, frame, P, 2)
        nrm = X.dynamics_normals(seed, frame, P, 3)
        u = X.resample_uniforms(seed, frame, P)
        r = O.step(om, T, pre["states"], pre["classes"], z, E, nrm, u, normals_by_particle=True)
        assert_step_matches(post, r, pf.class_probabilities().numpy(), pf.current_state_mean().numpy(), u,
                            "multinomial", ("cutoff", k))
        assert pf.health() == {h: 0 for h in pf.health()}


def test_cutoff_vs_dense_same_state(m2c, fx_config2):
    """The cutoff and the dense kernel from one state with the same draws agree at the
    filter's tolerances: log-likelihoods 1e-5 normwise, weights 1e-5 (the flushed values
    move q by less than half an ulp of 1 - q by construction; what remains is the two
    associations of k^T K^-1 k -- the reference's symmetric K^-1 against |R^T k|^2 --, whose
    cancellation at cond(K_y) ~ 1e6 gives ~1e-6 relative in ll here)."""
    from gpmdm_amd import GPMDM_PF
    T = torch.tensor(fx_config2["T"])
    P = 20_000
    Y = m2c.get_Y()
    torch.manual_seed(3)
    a = GPMDM_PF(m2c, T, P, rng="torch")
    a.update(Y[30])
    st = a.export_state()
    b = GPMDM_PF(m2c, T, P, rng="torch", obs_cutoff=True)
    b.load_state(st["states"], st["classes"], ll=st["ll"], log_w=st["log_w"], w=st["w"],
                 resample_idx=st["resample_idx"], frame=st.get("frame"))
    rng = np.random.RandomState(5)
    E, nrm, u = rng.exponential(size=(P, 2)), rng.randn(P, 3), rng.rand(P)
    a.update_with_draws(Y[31], E, nrm, u)
    b.update_with_draws(Y[31], E, nrm, u)
    sa, sb = a.export_state(), b.export_state()
    assert np.array_equal(sa["classes"], sb["classes"])
    assert nrel(sb["ll"], sa["ll"]) < 1e-5, nrel(sb["ll"], sa["ll"])
    assert nrel(sb["w"], sa["w"]) < 1e-5, nrel(sb["w"], sa["w"])


@pytest.mark.parametrize("world,P", [(4, 10_007), (8, 100_000)])
def test_cutoff_logical_shards_match_one_rank(m2c, world, P):
    """R logical shards of a cutoff filter (ancestor-ordered shards: another particle tiling
    than one rank's) are bitwise the one-rank cutoff filter over 3 frames."""
    from gpmdm_amd import GPMDM_PF
    T = torch.tensor([[0.9, 0.1], [0.1, 0.9]])
    Y = m2c.get_Y()
    torch.manual_seed(4)
    ref = GPMDM_PF(m2c, T, P, rng="philox", seed=91, obs_cutoff=True)
    ranks = []
    for r in range(world):
        torch.manual_seed(4)
        ranks.append(GPMDM_PF(m2c, T, P, rng="philox", seed=91, shard=(world, r), obs_cutoff=True))
    for k in range(3):
        z = np.ascontiguousarray(np.asarray(Y[60 + 3 * k], dtype=np.float64))
        ref.update(z)
        full = torch.cat([pf._stage_propagate(z) for pf in ranks], 0)
        for pf in ranks:
            pf._recv.copy_(full)
            pf._stage_resample()
        a = ref.export_state()
        for pf in ranks:
            b = pf.export_state()
            for key in ("states", "classes", "ll", "resample_idx"):
                assert np.array_equal(a[key], b[key]), (k, key)
            assert np.array_equal(ref.class_probabilities().numpy(), pf.class_probabilities().numpy())


@pytest.mark.parametrize("P", [100_000, 20_000])
def test_cutoff_split_policies_bitwise(m2c, P):
    """The cutoff kernel's tile scheduling (set_obs_cutoff(split=...)): whole tiles, the grid's
    tail as two workgroups per tile, every tile as two, the default's choice -- the same states,
    classes, log-likelihoods and ancestors bit for bit over 4 frames of the bench's stream: the
    second workgroup's per-tile partials, chained on in list order by the likelihood finish,
    are the whole tile's running sums."""
    from gpmdm_amd import GPMDM_PF, synthetic
    data = synthetic.make_sequences(2, 5, 200, 62, 3, seed=0)
    zs = data.observation_stream(6, seed=1)
    T = torch.tensor(synthetic.markov_matrix(2))
    out = {}
    for split in ("none", "tail", "all", "auto", "chunks"):
        torch.manual_seed(4)                 # (the initial cloud)
        pf = GPMDM_PF(m2c, T, P, rng="philox", seed=11, obs_cutoff=True)
        pf.set_obs_cutoff(True, split=split)
        out[split] = []
        for k in range(4):
            pf.update(zs[k])
            out[split].append(pf.export_state())
    with pytest.raises(ValueError):
        pf.set_obs_cutoff(True, split="half")
    for split in ("tail", "all", "auto", "chunks"):
        for k in range(4):
            for key in ("states", "classes", "ll", "log_w", "resample_idx"):
                assert np.array_equal(out["none"][k][key], out[split][k][key]), (split, k, key)


def test_cutoff_chunk_grid_on_a_spread_cloud_bitwise(m2c):
    """A cloud of 2000 distinct ancestors (the bench's --cutoff-spread cloud, 0.2 l): the
    default split policy measures the reach on its first frame (mode 1 counts like AUTO) and
    takes the chunk grid on the second (reach >= 0.5; the resampled cloud then collapses and
    the third frame goes back to whole tiles); every frame is bitwise the whole-tile
    scheduling's (split="none") and the explicit chunk grid's (split="chunks")."""
    from gpmdm_amd import GPMDM_PF, synthetic
    P = 100_000
    data = synthetic.make_sequences(2, 5, 200, 62, 3, seed=0)
    zs = data.observation_stream(6, seed=1)
    T = torch.tensor(synthetic.markov_matrix(2))
    X = m2c.X.detach().cpu().numpy()
    N, d = X.shape
    ell = np.exp(m2c.y_log_lengthscales.detach().cpu().numpy())
    cls_of = np.concatenate([np.full(m2c.get_X_for_class(c).shape[0], c) for c in range(2)])
    g = np.random.RandomState(23)
    anc = np.sort(g.choice(N, 2000, replace=False))
    g.shuffle(anc)
    owner = anc[(np.arange(P) * anc.size) // P]
    states = np.ascontiguousarray(X[owner] + 0.2 * ell[None, :] * g.randn(P, d))
    classes = cls_of[owner].astype(np.int64)
    zero, unif = np.zeros(P), np.full(P, 1.0 / P)
    out, fr = {}, {}
    for split in ("none", "auto", "chunks"):
        pf = GPMDM_PF(m2c, T, P, rng="philox", seed=11, obs_cutoff=True)
        pf.set_obs_cutoff(True, split=split)
        pf.load_state(states, classes, ll=zero, log_w=zero, w=unif, frame=7)
        out[split] = []
        for k in range(3):
            pf.update(zs[k])
            pf.class_probabilities()
            out[split].append(pf.export_state())
            if k == 0:              # the reach the second frame's split choice reads
                fr[split] = pf.obs_cutoff_auto()["fraction_run"]
    assert fr["auto"] is not None and fr["auto"] >= 0.5, fr
    for split in ("auto", "chunks"):
        for k in range(3):
            for key in ("states", "classes", "ll", "log_w", "resample_idx"):
                assert np.array_equal(out["none"][k][key], out[split][k][key]), (split, k, key)


def test_cutoff_skips_work_on_the_benchmark_cloud(m2c):
    """The bench's workload (config-2 model, P = 100k, the mocap-surrogate stream): the
    cutoff kernel runs a fraction of the dense kernel's MFMA groups."""
    from gpmdm_amd import GPMDM_PF, synthetic
    data = synthetic.make_sequences(2, 5, 200, 62, 3, seed=0)
    zs = data.observation_stream(8, seed=1)
    pf = GPMDM_PF(m2c, torch.tensor(synthetic.markov_matrix(2)), 100_000, rng="philox", seed=11)
    pf.set_obs_cutoff(True, stats=True)
    for k in range(6):
        pf.update(zs[k])
    pf.obs_cutoff_stats(reset=True)
    pf.update(zs[6])
    st = pf.obs_cutoff_stats()
    assert st["dense"] > 0 and 0 < st["run"] < st["dense"], st


def test_cutoff_far_cloud_has_no_reachable_kstep(m2c):
    """A cloud far from every training latent: every K-step is out of reach (the kernel runs
    the mean tiles only, with V = 0), and the likelihoods equal the dense kernel's, whose
    kernel values underflow to 0 there, to the rounding of the S sum's association."""
    from gpmdm_amd import GPMDM_PF
    T = torch.tensor([[0.9, 0.1], [0.1, 0.9]])
    P = 1000
    X = m2c.X.detach().cpu().numpy()
    rng = np.random.RandomState(7)
    far = X.max(0) + 50.0 * np.exp(m2c.y_log_lengthscales.detach().cpu().numpy()) + rng.rand(P, X.shape[1])
    cls = rng.randint(0, 2, size=P)
    Y = m2c.get_Y()
    E, nrm, u = rng.exponential(size=(P, 2)), np.zeros((P, X.shape[1])), rng.rand(P)
    out = {}
    for cut in (False, True):
        pf = GPMDM_PF(m2c, T, P, rng="torch", obs_cutoff=cut)
        pf.load_state(far, cls)
        if cut:
            pf.set_obs_cutoff(True, stats=True)
            pf.obs_cutoff_stats(reset=True)
        pf.update_with_draws(Y[5], E, nrm, u)
        out[cut] = pf.export_state()
        if cut:
            st = pf.obs_cutoff_stats()
    a, b = out[False], out[True]
    assert np.array_equal(a["classes"], b["classes"])
    # the propagated cloud (the dynamics GP's linear kernel extrapolates the far states) stays
    # out of reach: only the mean tiles ran
    assert st["dense"] > 0 and st["run"] < 0.05 * st["dense"], st
    assert np.max(np.abs(a["ll"] - b["ll"]) / np.maximum(np.abs(a["ll"]), 1.0)) < 1e-12


@pytest.fixture(scope="module", params=[5, 12])
def synth_cut(request):
    """Synthetic models at d = 5 (the 32 x 512 cutoff tile with the particle coordinates read
    from LDS, d = 4..8) and d = 12 (the 8-wave 64 x 512 tile of 9 <= d <= 16), N = 3000."""
    from conftest import synthetic_model
    m, T, Y = synthetic_model(C=2, d=request.param, D=24, L=500, S=3, seed=31 + request.param)
    return request.param, m, T, Y


def test_cutoff_vs_dense_other_latent_dims(synth_cut):
    """the cutoff kernel's d = 4..7 LDS-coordinate path and its 64-particle
    instantiations (9 <= d <= 15) against the dense kernel from one state with the same draws:
    classes exact, log-likelihoods and weights 1e-5 normwise (gpmdm.py:923-963,
    gpmdm_pf.py:170-204), one step from each of two states of the dense filter's trajectory
    (b is reloaded with a's state before each step: a flipped resampling index would otherwise
    compare different clouds)."""
    from gpmdm_amd import GPMDM_PF
    d, m, T, Y = synth_cut
    P = 5000
    torch.manual_seed(3)
    a = GPMDM_PF(m, T, P, rng="torch")
    a.update(Y[40])
    b = GPMDM_PF(m, T, P, rng="torch", obs_cutoff=True)
    b.set_obs_cutoff(True, stats=True)
    rng = np.random.RandomState(5)
    for k in range(2):
        st = a.export_state()
        b.load_state(st["states"], st["classes"], ll=st["ll"], log_w=st["log_w"], w=st["w"],
                     resample_idx=st["resample_idx"], frame=st.get("frame"))
        E, nrm, u = rng.exponential(size=(P, 2)), rng.randn(P, d), rng.rand(P)
        a.update_with_draws(Y[41 + k], E, nrm, u)
        b.update_with_draws(Y[41 + k], E, nrm, u)
        sa, sb = a.export_state(), b.export_state()
        assert np.array_equal(sa["classes"], sb["classes"]), (d, k)
        assert nrel(sb["ll"], sa["ll"]) < 1e-5, (d, k, nrel(sb["ll"], sa["ll"]))
        assert nrel(sb["w"], sa["w"]) < 1e-5, (d, k, nrel(sb["w"], sa["w"]))
    st = b.obs_cutoff_stats()
    assert st["dense"] > 0 and 0 < st["run"] <= st["dense"], st


def test_cutoff_logical_shards_other_latent_dims(synth_cut):
    """4 logical shards of a d = 5 / d = 12 cutoff filter (another particle tiling; shards 0 and
    2 with every list chunk its own workgroup, split="chunks") are bitwise the one-rank cutoff
    filter over 3 frames."""
    from gpmdm_amd import GPMDM_PF
    d, m, T, Y = synth_cut
    P, world = 6_007, 4
    torch.manual_seed(4)
    ref = GPMDM_PF(m, T, P, rng="philox", seed=91, obs_cutoff=True)
    ranks = []
    for r in range(world):
        torch.manual_seed(4)
        ranks.append(GPMDM_PF(m, T, P, rng="philox", seed=91, shard=(world, r), obs_cutoff=True))
        if r % 2 == 0:
            ranks[-1].set_obs_cutoff(True, split="chunks")
    for k in range(3):
        z = np.ascontiguousarray(np.asarray(Y[60 + 3 * k], dtype=np.float64))
        ref.update(z)
        full = torch.cat([pf._stage_propagate(z) for pf in ranks], 0)
        for pf in ranks:
            pf._recv.copy_(full)
            pf._stage_resample()
        a = ref.export_state()
        for pf in ranks:
            b = pf.export_state()
            for key in ("states", "classes", "ll", "resample_idx"):
                assert np.array_equal(a[key], b[key]), (d, k, key)


@pytest.mark.parametrize("which", ["config1", "config2"])
def test_device_cutoff_image_is_byte_equal_to_the_host_packer(fx_config1, fx_config2, which):
    """the cutoff image built on the device (gpmdm_model_build_obs_cutoff: R and
    K_y^-1 Y read back out of the device image, K_y^-1 = R R^T by dsyrk, the tile-major
    packing by a kernel) is byte for byte the host packer's image (host_image.h CutoffPacker,
    gpmdm_model_set_obs_cutoff) of the same K_y^-1 and K_y^-1 Y, with the same tau; the
    K_y^-1 it formed is the reference's U^-1 U^-T (gpmdm.py:1286-1290) to rounding."""
    import ctypes
    from gpmdm_amd import _lib
    m = product_model(fx_config1 if which == "config1" else fx_config2)
    lib = _lib.load()
    h = m.handle
    N, D = m.X.shape[0], m.D
    y_absmax = np.ascontiguousarray(np.max(np.abs(np.asarray(m.get_Y(), dtype=np.float64)), axis=0))
    sigma2 = float(torch.exp(m.y_log_sigma_n.detach().cpu())) ** 2 + m.sigma_n_num_Y ** 2
    K = np.zeros((N, N))
    M = np.zeros((N, D))
    _lib.check(lib.gpmdm_model_build_obs_cutoff(h, ctypes.c_double(sigma2), _lib.dptr(y_absmax), _lib.dptr(K),
                                                _lib.dptr(M)), "build")
    tau_dev = m.obs_cutoff_tau
    n = ctypes.c_int64()
    _lib.check(lib.gpmdm_model_obs_cutoff_image(h, ctypes.byref(n), None), "image size")
    img_dev = np.zeros(n.value)
    _lib.check(lib.gpmdm_model_obs_cutoff_image(h, ctypes.byref(n), _lib.dptr(img_dev)), "image")
    _lib.check(lib.gpmdm_model_set_obs_cutoff(h, _lib.dptr(K), _lib.dptr(M), ctypes.c_double(sigma2),
                                              _lib.dptr(y_absmax)), "host packer")
    img_host = np.zeros(n.value)
    _lib.check(lib.gpmdm_model_obs_cutoff_image(h, ctypes.byref(n), _lib.dptr(img_host)), "image")
    assert m.obs_cutoff_tau == tau_dev
    assert img_dev.tobytes() == img_host.tobytes()
    # K^-1 against the oracle's explicit inverse of K_y (the reference's recipe)
    om = oracle_model(fx_config1 if which == "config1" else fx_config2)
    assert np.max(np.abs(K - om.Ky_inv)) <= 1e-6 * np.max(np.abs(om.Ky_inv))
    assert np.array_equal(K, K.T)
    _lib.check(lib.gpmdm_model_set_obs_cutoff(h, None, None, ctypes.c_double(0.0), None), "remove")


def _auto_vs_hand_switched(m, T, P, zs, init=None, seed=11):
    """Run an AUTO filter (obs_cutoff="auto") beside a mode-1 filter switched by hand
    (set_obs_cutoff) through the AUTO filter's per-frame choices: every choice must follow the
    rule (a cutoff frame when no fraction is known, 8 frames after the last cutoff frame, or
    when the last measured fraction is <= 0.75) and every frame must be bitwise equal."""
    from gpmdm_amd import GPMDM_PF
    filters = []
    for mode in ("auto", True):
        torch.manual_seed(4)
        pf = GPMDM_PF(m, T, P, rng="philox", seed=seed, obs_cutoff=mode)
        if init is not None:
            pf.load_state(*init[:2], ll=init[2], log_w=init[2], w=init[3], frame=0)
        filters.append(pf)
    a, b = filters
    choices, fracs = [], []
    last_probe, frac = None, None
    for k, z in enumerate(zs):
        a.update(z)
        cut = a.obs_cutoff_auto()["last_frame_cutoff"]
        expect = frac is None or k - last_probe >= 8 or frac <= 0.75
        assert cut == expect, (k, cut, frac, last_probe)
        if cut:
            last_probe = k
            frac = a.obs_cutoff_auto()["fraction_run"]
        choices.append(cut)
        fracs.append(frac)
        b.set_obs_cutoff(bool(cut))
        b.update(z)
        sa, sb = a.export_state(), b.export_state()
        for key in ("states", "classes", "ll", "resample_idx"):
            assert np.array_equal(sa[key], sb[key]), (k, key, choices)
    return choices, fracs


def test_cutoff_auto_on_the_benchmark_stream(m2c):
    """AUTO (gpmdm_pf_set_obs_cutoff mode 3) on the bench's stream: the initial cloud (drawn
    from every training latent) reaches every K-step, so after the first probe the dense kernel
    runs; the next probe (frame 8) finds the collapsed cloud's low reach and the cutoff runs
    from there on."""
    from gpmdm_amd import synthetic
    data = synthetic.make_sequences(2, 5, 200, 62, 3, seed=0)
    zs = data.observation_stream(12, seed=1)
    T = torch.tensor(synthetic.markov_matrix(2))
    choices, fracs = _auto_vs_hand_switched(m2c, T, 100_000, zs)
    assert choices[0] and not all(choices[1:8]), (choices, fracs)
    assert all(choices[8:]) and fracs[-1] < 0.75, (choices, fracs)


def test_cutoff_auto_on_a_spread_cloud(m2c):
    """AUTO from a cloud spread over the training set (2000 ancestors, 0.5 l): the probe's
    reach is above the break-even, so the dense kernel runs until the next probe or until the
    cloud has collapsed; bitwise a hand-switched filter through the same choices."""
    T = torch.tensor([[0.9, 0.1], [0.1, 0.9]])
    P = 20_000
    X = m2c.X.detach().cpu().numpy()
    g = np.random.RandomState(23)
    anc = g.choice(X.shape[0], 2000, replace=False)
    owner = anc[(np.arange(P) * anc.size) // P]
    cls_of = np.concatenate([np.full(m2c.get_X_for_class(c).shape[0], c) for c in range(2)])
    states = np.ascontiguousarray(X[owner] + 0.5 * g.randn(P, X.shape[1]))
    classes = cls_of[owner].astype(np.int64)
    Y = m2c.get_Y()
    zs = [np.asarray(Y[100 + 5 * k], dtype=np.float64) for k in range(12)]
    choices, fracs = _auto_vs_hand_switched(m2c, T, P, zs, init=(states, classes, np.zeros(P), np.full(P, 1.0 / P)),
                                            seed=5)
    assert choices[0] and fracs[0] > 0.75 and not all(choices), (choices, fracs)
