"""Generate the UNMODIFIED reference's map-performance read-outs for the trained config-1
model of ``make_checkpoint.py`` (train_gpmdm.ipynb's evaluation calls, gpmdm.py:1147-1273):

    python tests/golden/make_map_performance.py

The model is rebuilt and trained exactly as ``make_checkpoint.py`` does (20 reference
``train_adam`` steps, seed 0) and checked against the committed checkpoint arrays
(``ref_checkpoint_config1.npz``: X and the log hyperparameters bit for bit), so the outputs
below belong to ``ref_checkpoint_config1.pth``.  Written (numbers only):
``ref_map_performance_config1.npz`` with, per class c, the reference's
``get_dynamics_map_performance_for_class(c)`` (means, variances, NMSE; Xin/Xout once) and
``get_latent_map_performance_for_class(c)`` (NMSE and its row range: its means and variances
are those rows of the all-rows read-out to 1e-10, asserted here) and once ``get_latent_map_performance()``
(means, variances, NMSE).  The reference computes NMSE with floor division,
``(Y - mu) ** 2 // var``.  Also: the all-class ``map_x_dynamics`` at 32 fixed points and a few
kernel-helper values (get_x/y_kernel with and without noise, the diagonal kernels, row sums of
get_M / get_M_for_class).
Run here only: the reference never travels to the GPU box.
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
import make_golden as G  # noqa: E402  (imports the reference with its two stand-ins)

OUT = Path(__file__).resolve().parent


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    cfg = G.synthetic.CONFIGS[1]
    m, _ = G.build_reference_model(cfg["C"], cfg["S"], cfg["L"], cfg["D"], cfg["d"], 0.1)
    torch.manual_seed(0)
    m.train_adam(20, num_print_steps=0, lr=0.01)
    ck = np.load(OUT / "ref_checkpoint_config1.npz")
    for k, v in G.model_arrays(m).items():
        if k in ck.files and k != "seq_lengths":
            assert np.array_equal(np.asarray(v, dtype=np.float64), ck[k]), f"retrained model differs from the checkpoint: {k}"
    m.set_evaluation_mode()
    arr = {}
    mu, var, Y, nmse = m.get_latent_map_performance()
    arr.update({"obs_mu": mu, "obs_var": var, "obs_nmse": np.float64(nmse)})
    off = 0
    for c in range(cfg["C"]):
        mu_d, var_d, Xout, Xin, nmse_d = m.get_dynamics_map_performance_for_class(c)
        arr.update({f"dyn{c}_mu": mu_d, f"dyn{c}_var": var_d, f"dyn{c}_nmse": np.float64(nmse_d),
                    "dyn_Xout": Xout, "dyn_Xin": Xin})
        mu_c, var_c, Y_c, nmse_c = m.get_latent_map_performance_for_class(c)
        n = mu_c.shape[0]
        # the class read-out is the class's rows of the all-rows one up to BLAS blocking
        # (stored once)
        assert np.allclose(mu_c, mu[off:off + n], rtol=1e-10, atol=1e-12)
        assert np.allclose(var_c, var[off:off + n], rtol=1e-10, atol=1e-12)
        arr[f"obs{c}_nmse"] = np.float64(nmse_c)
        arr[f"obs{c}_rows"] = np.array([off, off + n])
        off += n
    # the all-class dynamics map and the kernel helpers at fixed query points
    rng = np.random.RandomState(21)
    Xin_t, _, _ = m.get_Xin_Xout_matrices()
    xq = torch.tensor(rng.randn(32, cfg["d"]), dtype=torch.float64)
    with torch.no_grad():
        mu, var = m.map_x_dynamics(xq)
        arr.update({"alldyn_xs": xq.numpy(), "alldyn_mu": mu.numpy(), "alldyn_var": var.numpy(),
                    "k_x_noise": m.get_x_kernel(Xin_t[:7], Xin_t[3:10]).numpy(),
                    "k_x": m.get_x_kernel(Xin_t[:7], xq[:4], False).numpy(),
                    "k_y_noise": m.get_y_kernel(m.X[:6], m.X[2:8]).numpy(),
                    "kd_x": m.get_x_diag_kernel(xq, True).numpy(),
                    "kd_y": m.get_y_diag_kernel(xq, True).numpy(),
                    "M_rowsums": m.get_M().sum(1).numpy(),
                    "M1_rowsums": m.get_M_for_class(1).sum(1).numpy()})
    np.savez_compressed(OUT / "ref_map_performance_config1.npz", **arr)
    print("wrote ref_map_performance_config1.npz:",
          {k: float(v) for k, v in arr.items() if k.endswith("nmse")})


if __name__ == "__main__":
    main()
