"""Time the UNMODIFIED reference's train_adam per step on this container's CPU (configs 1, 2).

Run here only (imports /root/reference through tests/golden/make_golden.py's stand-ins;
the reference never travels to the GPU box).  Output recorded in profiles/.
"""
import os
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests" / "golden"))
import make_golden as mg  # noqa: E402
from gpmdm_amd import synthetic  # noqa: E402

torch.set_num_threads(min(8, os.cpu_count() or 1))
for cfg in (1, 2):
    c = synthetic.CONFIGS[cfg]
    m, _ = mg.build_reference_model(c["C"], c["S"], c["L"], c["D"], c["d"], 0.1)
    m.train_adam(1, lr=0.01)
    steps = 5 if cfg == 1 else 2
    t0 = time.perf_counter()
    m.train_adam(steps, lr=0.01)
    s = (time.perf_counter() - t0) / steps
    print(f"reference train_adam config {cfg} (N={m.X.shape[0]}): {s:.4f} s per Adam step "
          f"(CPU, torch threads {torch.get_num_threads()})", flush=True)
