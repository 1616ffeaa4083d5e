"""Training goldens from the UNMODIFIED reference (run here only; the reference never travels).

    python tests/golden/make_golden_training.py

For the config-1 model (N=500, D=62, d=3, C=2, sigma_n=0.1, PCA-initialised latents) the
reference's ``GPMDM.gpdm_loss`` (gpmdm.py:721-760) and its parameter gradients at the
initial point, the two loss terms (gpmdm.py:550-628), and five steps of
``GPMDM.train_adam(5, lr=0.01)`` (gpmdm.py:817-885): the per-step losses and the trained
parameters.  Only numbers are stored.
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
import make_golden as mg  # noqa: E402  (imports the reference with the two stand-in modules)

from gpmdm_amd import synthetic  # noqa: E402

PARAMS = ("y_log_lengthscales", "y_log_lambdas", "y_log_sigma_n", "x_log_lengthscales",
          "x_log_lambdas", "x_log_sigma_n", "x_log_lin_coeff", "X")


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    cfg = synthetic.CONFIGS[1]
    m, _ = mg.build_reference_model(cfg["C"], cfg["S"], cfg["L"], cfg["D"], cfg["d"], 0.1)
    arr = mg.model_arrays(m)
    Y = m.get_Y()
    N = Y.shape[0]
    Yt = torch.tensor(Y, dtype=torch.float64)
    m.set_training_mode("all")
    Xin, Xout, _ = m.get_Xin_Xout_matrices()
    arr["loss_y0"] = np.float64(m.get_y_neg_log_likelihood(Yt, m.X, N).item())
    arr["loss_x0"] = np.float64(m.get_x_neg_log_likelihood(Xout, Xin).item())
    loss = m.gpdm_loss(Yt, N, None)
    loss.backward()
    arr["loss0"] = np.float64(loss.item())
    for p in PARAMS:
        arr[f"grad0_{p}"] = getattr(m, p).grad.detach().numpy().astype(np.float64).reshape(-1)

    m2, _ = mg.build_reference_model(cfg["C"], cfg["S"], cfg["L"], cfg["D"], cfg["d"], 0.1)
    losses = m2.train_adam(5, num_print_steps=0, lr=0.01, balance=1)
    arr["adam_losses"] = np.asarray(losses, dtype=np.float64)
    for p in PARAMS:
        arr[f"adam5_{p}"] = getattr(m2, p).detach().numpy().astype(np.float64).reshape(-1)
    mg.save("training_n500.npz", arr)


if __name__ == "__main__":
    main()
