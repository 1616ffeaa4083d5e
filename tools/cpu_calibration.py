"""Calibrate bench.py's cpu_baseline (the numpy oracle, "port") against the UNMODIFIED
reference: both run the config-2 workload (N=2000, D=62, d=3, C=2, P=100k, sigma_n=0.1) on
the same 8 threads of this container, a few frames each after one warm-up frame; the ratio
lets the port's number on the GPU box be read as the reference's.

Run here only (the reference never travels; imported through tests/golden/make_golden.py's
stand-ins).  Output recorded in profiles/r03/cpu_calibration.txt.
"""
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
from threadpoolctl import threadpool_limits

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tests" / "golden"))
sys.path.insert(0, str(ROOT))
import make_golden as mg  # noqa: E402
from gpmdm_amd import synthetic  # noqa: E402
from oracle import gpmdm_oracle as O  # noqa: E402

THREADS = 8
P = int(os.environ.get("CAL_P", "100000"))
FRAMES = int(os.environ.get("CAL_FRAMES", "2"))
torch.set_num_threads(THREADS)
c = synthetic.CONFIGS[2]
m, data = mg.build_reference_model(c["C"], c["S"], c["L"], c["D"], c["d"], 0.1)
z = data.observation_stream(FRAMES + 1, seed=1)
T = torch.tensor(synthetic.markov_matrix(2))

torch.manual_seed(11)
pf = mg.GPMDM_PF(m, markov_switching_model=T, num_particles=P)
pf.update(z[0])
t0 = time.perf_counter()
for f in range(FRAMES):
    pf.update(z[1 + f])
    pf.get_most_likely_class()
    pf.class_probabilities()
    pf.current_state_mean()
t_ref = (time.perf_counter() - t0) / FRAMES
print(f"reference gpmdm_pf (torch CPU, {torch.get_num_threads()} threads): P={P}, {t_ref:.2f} s/frame, "
      f"{P / t_ref:.4g} particle-steps/s", flush=True)

arr = mg.model_arrays(m)
om = O.OracleModel(X=arr["X"], Y=arr["Y"], seq_lengths=arr["seq_lengths"].tolist(),
                   y_log_lengthscales=arr["y_log_lengthscales"], y_log_lambdas=arr["y_log_lambdas"],
                   y_log_sigma_n=float(arr["y_log_sigma_n"]), x_log_lengthscales=arr["x_log_lengthscales"],
                   x_log_lambdas=arr["x_log_lambdas"], x_log_sigma_n=float(arr["x_log_sigma_n"]),
                   x_log_lin_coeff=arr["x_log_lin_coeff"], sigma_n_num_X=0.0, sigma_n_num_Y=0.0).precompute()
rng = np.random.RandomState(0)
parts = [rng.randint(0, om.X_for_class(k).shape[0], P // 2) for k in range(2)]
s, cl = O.init_particles(om, P, parts)
Tn = synthetic.markov_matrix(2)
with threadpool_limits(THREADS):
    def step(zf):
        r = O.step(om, Tn, s, cl, zf, rng.exponential(size=(P, 2)), rng.randn(P, 3), rng.rand(P))
        return r.states, r.classes
    s, cl = step(z[0])
    t0 = time.perf_counter()
    for f in range(FRAMES):
        s, cl = step(z[1 + f])
    t_port = (time.perf_counter() - t0) / FRAMES
print(f"port (numpy oracle, BLAS {THREADS} threads): P={P}, {t_port:.2f} s/frame, {P / t_port:.4g} particle-steps/s",
      flush=True)
print(f"ratio port/reference throughput: {t_ref / t_port:.3f} (reference = port x {t_port / t_ref:.3f})", flush=True)
