"""GPU: a native host drives the whole path through the C ABI alone.

``examples/c_host/pf_main`` (plain C, built by ``gpmdm_amd.build``) reads the model's raw
training data, factors the kernel matrices on the device (gpmdm_gp_factor), builds the
model and a Philox filter, and steps it frame by frame (gpmdm_pf_step / gpmdm_pf_read):
what a notebook does with the reference (gpmdm_pf.py:47-262), with no Python or torch in
the process.  Its per-frame read-outs must be bitwise those of the Python mirror on the
same model (device precompute), the same initial particles and the same seed.
"""
import struct
import subprocess

import numpy as np
import pytest
import torch

from conftest import product_model

pytestmark = pytest.mark.gpu


def _write_input(path, m, T, st, Z, P, seed, resample):
    C, d, D = m.n_classes, m.d, m.D
    X = m.X.detach().numpy()
    Y = np.asarray(m.get_Y(), dtype=np.float64)
    Xin, Xout, _ = m.get_Xin_Xout_matrices(X=m.X)
    Nc = np.asarray(m._class_dynamics_rows(), dtype=np.int64)
    sy2 = float(torch.exp(m.y_log_sigma_n)) ** 2
    sx2 = float(torch.exp(m.x_log_sigma_n)) ** 2
    f64 = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64)).tobytes()  # noqa: E731
    with open(path, "wb") as fh:
        fh.write(struct.pack("<8q", X.shape[0], D, d, C, P, Z.shape[0], seed, resample))
        fh.write(Nc.tobytes())
        for a in (X, Y, np.asarray(Xin), np.asarray(Xout),
                  torch.exp(m.y_log_lengthscales).detach().numpy(), (torch.exp(m.y_log_lambdas) ** -2).detach().numpy(),
                  torch.exp(m.x_log_lengthscales).detach().numpy(), (torch.exp(m.x_log_lin_coeff) ** 2).detach().numpy(),
                  (torch.exp(m.x_log_lambdas) ** -2).detach().numpy(),
                  [sy2, m.sigma_n_num_Y ** 2, sx2, m.sigma_n_num_X ** 2], T, st["states"]):
            fh.write(f64(a))
        fh.write(np.ascontiguousarray(st["classes"], dtype=np.int64).tobytes())
        fh.write(f64(Z))


@pytest.mark.parametrize("resample,ranks", [(0, 0), (1, 0), (0, 1)])
def test_native_c_host_matches_python(fx_config2, tmp_path, resample, ranks):
    """ranks=1: the host's --ranks mode (RCCL communicator through gpmdm_comm_init, the
    library's own exchange, gpmdm_pf_set_comm) on this box's one GPU."""
    from gpmdm_amd import GPMDM_PF, build
    exe = build.build_c_host()
    m = product_model(fx_config2)
    m._precompute_device = "device"          # the factors the C host computes with gpmdm_gp_factor
    m._precompute_kernel_inverses()
    T = np.asarray(fx_config2["T"], dtype=np.float64)
    P, F, seed = 20_011, 6, 77
    torch.manual_seed(3)
    pf = GPMDM_PF(m, torch.tensor(T), P, rng="philox", seed=seed,
                  resample="multinomial" if resample == 0 else "systematic")
    st = pf.export_state()
    Y = m.get_Y()
    Z = np.stack([np.asarray(Y[40 + 3 * k], dtype=np.float64) for k in range(F)])
    _write_input(tmp_path / "in.bin", m, T, st, Z, P, seed, resample)
    extra = ["--ranks", str(ranks), "--rank", "0", "--id", str(tmp_path / "rccl.id")] if ranks else []
    r = subprocess.run([str(exe), str(tmp_path / "in.bin"), str(tmp_path / "out.bin"), *extra],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    C, d = m.n_classes, m.d
    got = np.fromfile(tmp_path / "out.bin", dtype=np.float64).reshape(F, C + d + 1)
    for k in range(F):
        pf.update(Z[k])
        assert np.array_equal(got[k, :C], pf.class_probabilities().numpy()), k
        assert np.array_equal(got[k, C:C + d], pf.current_state_mean().numpy()), k
        assert got[k, C + d] == pf.log_likelihood(), k
