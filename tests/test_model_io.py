"""Model I/O on the host (no GPU): the reference checkpoint format and our .npz."""
import numpy as np
import torch

from gpmdm_amd import GPMDM
from gpmdm_amd.model import read_reference_checkpoint


def _reference_style_checkpoint(path):
    """A file in the exact layout GPMDM.save writes (gpmdm.py:1316-1345): state_dict of
    log-parameters and X, config_dict holding numpy observation arrays."""
    rng = np.random.RandomState(0)
    obs = [[rng.randn(6, 4).astype(np.float32), rng.randn(5, 4).astype(np.float32)],
           [rng.randn(7, 4).astype(np.float32)]]
    sd = {"y_log_lengthscales": torch.log(torch.tensor([1.1, 0.9], dtype=torch.float64)),
          "y_log_lambdas": torch.zeros(4, dtype=torch.float64),
          "y_log_sigma_n": torch.log(torch.tensor(0.1, dtype=torch.float64)),
          "x_log_lengthscales": torch.zeros(2, dtype=torch.float64),
          "x_log_lambdas": torch.zeros(2, dtype=torch.float64),
          "x_log_sigma_n": torch.log(torch.tensor(0.2, dtype=torch.float64)),
          "x_log_lin_coeff": torch.zeros(3, dtype=torch.float64),
          "X": torch.tensor(rng.randn(18, 2))}
    cfg = {"class_aware_observations_list": obs, "dyn_target": "full", "dyn_back_step": 1, "D": 4, "d": 2,
           "n_classes": 2, "sigma_n_num_X": 0.0, "sigma_n_num_Y": 0.0, "dtype": "torch.float64",
           "device": "cpu", "y_lengthscales_init": [1.1, 0.9], "y_lambdas_init": [1.0] * 4,
           "y_sigma_n_init": 0.1, "x_lengthscales_init": [1.0, 1.0], "x_lambdas_init": [1.0, 1.0],
           "x_sigma_n_init": 0.2, "x_lin_coeff_init": [1.0, 1.0, 1.0]}
    torch.save({"state_dict": sd, "config_dict": cfg}, path)
    return sd, cfg


def test_reference_pth_loads_with_weights_only(tmp_path):
    p = tmp_path / "model.pth"
    sd, cfg = _reference_style_checkpoint(p)
    cfg2, sd2 = read_reference_checkpoint(p)
    assert cfg2["D"] == 4 and len(cfg2["class_aware_observations_list"][0]) == 2
    assert np.array_equal(cfg2["class_aware_observations_list"][1][0], cfg["class_aware_observations_list"][1][0])
    m = GPMDM.load(p, upload=False)
    assert torch.equal(m.X, sd["X"])
    assert torch.equal(m.y_log_lengthscales, sd["y_log_lengthscales"])
    Xin, Xout, starts = m.get_Xin_Xout_matrices()
    assert Xin.shape == (15, 2) and starts == [0, 6, 11]
    assert torch.equal(m.get_X_for_class(1), sd["X"][11:])


def test_npz_round_trip(tmp_path):
    p = tmp_path / "model.pth"
    _reference_style_checkpoint(p)
    m = GPMDM.load(p, upload=False)
    q = tmp_path / "model.npz"
    m.save(q)
    m2 = GPMDM.load(q, upload=False)
    assert torch.equal(m2.X, m.X)
    for k in ("y_log_lengthscales", "y_log_lambdas", "x_log_lin_coeff", "x_log_sigma_n"):
        assert torch.equal(getattr(m2, k), getattr(m, k)), k
    assert np.array_equal(m2.get_Y(), m.get_Y())


def test_reference_written_checkpoint_loads(tmp_path):
    """A checkpoint written by the reference's own GPMDM.save after 20 steps of its own
    train_adam (tests/golden/make_checkpoint.py): the safe loader reproduces every saved
    parameter bit for bit and the observation sequences; the .npz round trip keeps them."""
    from conftest import GOLDEN
    f = np.load(GOLDEN / "ref_checkpoint_config1.npz", allow_pickle=False)
    m = GPMDM.load(GOLDEN / "ref_checkpoint_config1.pth", upload=False)
    assert np.array_equal(m.X.detach().numpy(), f["X"])
    for k in ("y_log_lengthscales", "y_log_lambdas", "x_log_lengthscales", "x_log_lambdas", "x_log_lin_coeff"):
        assert np.array_equal(getattr(m, k).detach().numpy(), f[k]), k
    for k in ("y_log_sigma_n", "x_log_sigma_n"):
        assert float(getattr(m, k)) == float(f[k]), k
    assert np.array_equal(m.get_Y(), f["Y"])
    assert [[len(s) for s in c] for c in m.class_aware_observations_list] == f["seq_lengths"].tolist()
    assert (m.D, m.d, m.n_classes, m.dyn_target, m.dyn_back_step) == (62, 3, 2, "full", 1)
    q = tmp_path / "m.npz"
    m.save(q)
    m2 = GPMDM.load(q, upload=False)
    assert np.array_equal(m2.X.detach().numpy(), f["X"]) and np.array_equal(m2.get_Y(), f["Y"])


def test_kernel_helpers_match_reference():
    """GPMDM's kernel helpers (gpmdm.py:311-548, 965-991, 1070-1101) on the reference-trained
    checkpoint against the reference's own values (tests/golden/make_map_performance.py);
    host tensors, no device model."""
    from pathlib import Path
    golden = Path(__file__).resolve().parent / "golden"
    g = dict(np.load(golden / "ref_map_performance_config1.npz", allow_pickle=False))
    m = GPMDM.load(golden / "ref_checkpoint_config1.pth", upload=False)
    Xin, _, _ = m.get_Xin_Xout_matrices()
    xq = torch.tensor(g["alldyn_xs"])
    close = lambda a, b: np.testing.assert_allclose(a.detach().numpy(), b, rtol=1e-12, atol=1e-13)
    close(m.get_x_kernel(Xin[:7], Xin[3:10]), g["k_x_noise"])
    close(m.get_x_kernel(Xin[:7], xq[:4], False), g["k_x"])
    close(m.get_y_kernel(m.X[:6], m.X[2:8]), g["k_y_noise"])
    close(m.get_x_diag_kernel(xq, True), g["kd_x"])
    close(m.get_y_diag_kernel(xq, True), g["kd_y"])
    close(m.get_M().sum(1), g["M_rowsums"])
    close(m.get_M_for_class(1).sum(1), g["M1_rowsums"])


def test_state_dict_matches_reference_checkpoint():
    """state_dict()/named_parameters() carry the reference nn.Module's parameter names in its
    registration order (gpmdm.py:201-230, 773) and the values GPMDM.save stored."""
    from pathlib import Path
    pth = Path(__file__).resolve().parent / "golden" / "ref_checkpoint_config1.pth"
    _, ref_sd = read_reference_checkpoint(pth)
    m = GPMDM.load(pth, upload=False)
    sd = m.state_dict()
    assert list(sd.keys()) == list(ref_sd.keys())
    for k, v in ref_sd.items():
        assert torch.equal(sd[k], v.to(torch.float64)), k
    assert [k for k, _ in m.named_parameters()] == list(sd.keys())
    assert len(list(m.parameters())) == len(sd)
    try:
        m.load_state_dict({"X": sd["X"]})
    except RuntimeError as e:
        assert "missing keys" in str(e)
    else:
        raise AssertionError("strict load_state_dict accepted a partial state")


def test_load_state_dict_rejects_before_installing():
    """A size mismatch names its key and, like a strict key mismatch, leaves the model as
    it was (nothing is installed before the whole dict is checked)."""
    from pathlib import Path
    import pytest
    pth = Path(__file__).resolve().parent / "golden" / "ref_checkpoint_config1.pth"
    m = GPMDM.load(pth, upload=False)
    before = {k: v.clone() for k, v in m.state_dict().items()}
    bad = dict(before)
    bad["y_log_lambdas"] = before["y_log_lambdas"] + 1.0
    bad["X"] = before["X"][:-3]                      # fewer latents than the model holds
    with pytest.raises(RuntimeError, match="size mismatch for X"):
        m.load_state_dict(bad)
    bad2 = dict(before, y_log_lambdas=before["y_log_lambdas"] + 1.0, extra=torch.zeros(1))
    with pytest.raises(RuntimeError, match="unexpected keys"):
        m.load_state_dict(bad2)
    for k, v in m.state_dict().items():
        assert torch.equal(v, before[k]), k


def test_save_warns_on_an_unusual_suffix(tmp_path):
    import warnings
    from pathlib import Path
    pth = Path(__file__).resolve().parent / "golden" / "ref_checkpoint_config1.pth"
    m = GPMDM.load(pth, upload=False)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        m.save(tmp_path / "model.bin")
        m.save(tmp_path / "model.pth")
    assert len(w) == 1 and "pickle" in str(w[0].message)
    assert (tmp_path / "model.bin").exists() and (tmp_path / "model.pth").exists()


def _structure(cfg, sd):
    """Keys, types, dtypes and shapes of a checkpoint (values aside)."""
    def desc(v):
        if isinstance(v, torch.Tensor):
            return ("tensor", str(v.dtype), tuple(v.shape))
        if isinstance(v, np.ndarray):
            return ("ndarray", str(v.dtype), v.ndim)
        if isinstance(v, list):
            return ("list", desc(v[0]) if v else None)
        return (type(v).__name__,)
    return ([(k, desc(v)) for k, v in sd.items()],
            [(k, desc(v)) for k, v in cfg.items() if k not in ("class_aware_observations_list", "device")],
            [[desc(s) for s in c] for c in cfg["class_aware_observations_list"]])


def test_pth_round_trip_exact_path(tmp_path):
    """save("m.pth") writes the reference's torch layout to exactly that path (gpmdm.py:
    1307-1345) and load("m.pth") gives X, the log-parameters and the observations back bit
    for bit (train_gpmdm.ipynb:366 -> test_gpmdm_pf.ipynb:38)."""
    from conftest import GOLDEN
    m = GPMDM.load(GOLDEN / "ref_checkpoint_config1.pth", upload=False)
    p = tmp_path / "gpmdm_4d_30fps.pth"
    m.save(str(p))
    assert p.exists() and not (tmp_path / "gpmdm_4d_30fps.pth.npz").exists()
    assert not GPMDM._is_npz(p)
    m2 = GPMDM.load(p, upload=False)
    assert torch.equal(m2.X, m.X)
    for k, v in m.state_dict().items():
        assert torch.equal(m2.state_dict()[k], v), k
    assert (m2.D, m2.d, m2.n_classes, m2.dyn_target, m2.dyn_back_step) == (m.D, m.d, m.n_classes, "full", 1)
    for c1, c2 in zip(m.class_aware_observations_list, m2.class_aware_observations_list):
        assert len(c1) == len(c2)
        for a, b in zip(c1, c2):
            assert a.dtype == b.dtype and np.array_equal(a, b)
    # .npz stays the pickle-free option, written to exactly its path, also found by content
    q = tmp_path / "m.npz"
    m.save(q)
    assert GPMDM._is_npz(q)
    r = tmp_path / "renamed.pth"
    q.rename(r)
    m3 = GPMDM.load(r, upload=False)
    assert torch.equal(m3.X, m.X) and np.array_equal(m3.get_Y(), m.get_Y())


def test_pth_layout_matches_reference_written_file(tmp_path):
    """Our .pth and the reference-written checkpoint have the same keys (in order), types,
    dtypes and shapes, read with the same safe loader; the config values the reference
    derives from the parameters agree."""
    from conftest import GOLDEN
    ref = GOLDEN / "ref_checkpoint_config1.pth"
    cfg_r, sd_r = read_reference_checkpoint(ref)
    m = GPMDM.load(ref, upload=False)
    p = tmp_path / "ours.pth"
    m.save(p)
    cfg_o, sd_o = read_reference_checkpoint(p)
    assert list(cfg_o.keys()) == list(cfg_r.keys())
    assert list(sd_o.keys()) == list(sd_r.keys())
    assert _structure(cfg_o, sd_o) == _structure(cfg_r, sd_r)
    assert getattr(sd_o, "_metadata", None) == getattr(sd_r, "_metadata", None)
    for k in ("y_lengthscales_init", "y_lambdas_init", "y_sigma_n_init", "x_lengthscales_init",
              "x_lambdas_init", "x_sigma_n_init", "x_lin_coeff_init", "dtype", "D", "d", "n_classes",
              "dyn_target", "dyn_back_step", "sigma_n_num_X", "sigma_n_num_Y"):
        assert cfg_o[k] == cfg_r[k], k


def test_gpmdm_is_an_nn_module_with_the_reference_parameters():
    """GPMDM is a torch.nn.Module like the reference's (gpmdm.py:18): nn.Parameters in the
    reference's registration order, requires_grad from the flg_train_* flags and from
    set_training_mode / set_evaluation_mode (gpmdm.py:239-279), train()/eval(), and
    parameter versions that tell the model its device factors are stale after an in-place
    update (an optimiser step)."""
    from conftest import GOLDEN
    m = GPMDM.load(GOLDEN / "ref_checkpoint_config1.pth", upload=False)
    assert isinstance(m, torch.nn.Module)
    names = [n for n, _ in m.named_parameters()]
    assert names == ["y_log_lengthscales", "y_log_lambdas", "y_log_sigma_n", "x_log_lengthscales",
                     "x_log_lambdas", "x_log_sigma_n", "x_log_lin_coeff", "X"]
    assert all(isinstance(p, torch.nn.Parameter) and p.requires_grad for p in m.parameters())
    m.set_training_mode("latent")
    assert m.y_log_lambdas.requires_grad and not m.x_log_lambdas.requires_grad and m.X.requires_grad
    m.set_training_mode("dynamics")
    assert not m.y_log_lambdas.requires_grad and m.x_log_lin_coeff.requires_grad
    m.set_evaluation_mode()
    assert not any(p.requires_grad for p in m.parameters())
    assert m.eval() is m and not m.training and m.train().training
    # constructor flags are requires_grad flags
    m2 = GPMDM(D=4, d=2, n_classes=1, dyn_target="full", dyn_back_step=1, y_lambdas_init=np.ones(4),
               y_lengthscales_init=np.ones(2), y_sigma_n_init=0.1, x_lambdas_init=np.ones(2),
               x_lengthscales_init=np.ones(2), x_sigma_n_init=0.1, x_lin_coeff_init=np.ones(3),
               flg_train_y_lambdas=False, device="cuda:0")
    assert not m2.y_log_lambdas.requires_grad and m2.y_log_lengthscales.requires_grad
    assert m2.X is None and "X" not in m2.state_dict()
    # an optimiser step over parameters() changes the parameter versions the device model
    # was built from (GPMDM._refresh rebuilds it on the next use)
    m.set_training_mode("all")
    before = m._param_versions()
    opt = torch.optim.SGD(m.parameters(), lr=1e-3)
    loss = (m.y_log_lambdas ** 2).sum() + (m.X ** 2).sum()
    loss.backward()
    opt.step()
    assert m._param_versions() != before
