"""Bank throughput on the config-1 model (N = 500) at F x P = 1000 x 1000: the per-filter
16 x 256 observation image (default for P <= 1024) against the 32 x 512 image
(GPMDM_OBS_IMAGE16=0; run once per setting, the switch is read when the model is built)."""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from conftest import load_fixture, product_model  # noqa: E402
from gpmdm_amd import GPMDM_PF_Bank  # noqa: E402

f = load_fixture("config1_n500_p100_f200")
m = product_model(f)
T = torch.tensor(np.asarray(f["T"], dtype=np.float64))
Y = m.get_Y()
F, P = int(sys.argv[1]), int(sys.argv[2])
bank = GPMDM_PF_Bank(m, T, F, P, seed=5)
Z = [np.stack([Y[(7 * i + k) % Y.shape[0]] for i in range(F)]) for k in range(30)]
for k in range(5):
    bank.update(Z[k])
    bank.class_probabilities()
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(5, 30):
    bank.update(Z[k])
    bank.class_probabilities()
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / 25 * 1e3
print(f"F={F} P={P} image16={os.environ.get('GPMDM_OBS_IMAGE16', 'default')}: {ms:.3f} ms/frame, "
      f"{F * P / ms * 1e3:.3e} particle-steps/s")
