"""Generate a checkpoint written by the UNMODIFIED reference's ``GPMDM.save``
(gpmdm.py:1307-1346) and the reference's outputs for it.

Run here only (the reference never travels to the GPU box):

    python tests/golden/make_checkpoint.py

The config-1 model shape (N=500, D=62, d=3, C=2, sigma_n=0.1, tests/golden/make_golden.py)
is trained for 20 Adam steps with the reference's own ``train_adam`` (gpmdm.py:817-885),
so every saved parameter differs from its initial value, then saved with ``GPMDM.save``:
``torch.save({'state_dict', 'config_dict'})``, whose config holds the observation
sequences as numpy arrays.  Written next to it (numbers only):

* ``ref_checkpoint_config1.pth``  -- the reference's file, byte for byte as it wrote it;
* ``ref_checkpoint_config1.npz``  -- the parameters it holds (X and the log
  hyperparameters as float64) and the reference's predictive maps of the trained model
  at fixed query points (map_x_dynamics_for_class per class, map_x_to_y).

``gpmdm_amd.GPMDM.load`` must read the .pth with the safe loader only
(``torch.load(weights_only=True)`` with numpy arrays allow-listed; the reference's own
``GPMDM.load`` fails under torch >= 2.6) and reproduce both.
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
    losses = m.train_adam(20, num_print_steps=0, lr=0.01)
    pth = OUT / "ref_checkpoint_config1.pth"
    m.save(str(pth))
    arr = {k: np.asarray(v, dtype=np.float64) for k, v in G.model_arrays(m).items() if k != "seq_lengths"}
    arr["seq_lengths"] = G.model_arrays(m)["seq_lengths"]
    arr["losses"] = np.asarray(losses)
    arr.update(G.op_goldens(m, 64, 128, seed=15))
    np.savez_compressed(OUT / "ref_checkpoint_config1.npz", **arr)
    print(f"wrote {pth} ({pth.stat().st_size / 1e3:.0f} kB) and ref_checkpoint_config1.npz; "
          f"loss {losses[0]:.6g} -> {losses[-1]:.6g}")


if __name__ == "__main__":
    main()
