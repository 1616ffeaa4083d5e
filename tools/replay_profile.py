"""Host-side phase timing of one rng='torch' (replay) frame at the headline size
(config 2, P = 100k): where the frame's time goes between the GPU's work."""
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from gpmdm_amd import GPMDM_PF, _lib, synthetic  # noqa: E402

bench.WORKLOAD = bench.workload(2)
dev = torch.device("cuda", 0)
model, data = bench.build_model(dev)
T = torch.from_numpy(synthetic.markov_matrix(2))
P = 100_000
zs = data.observation_stream(80, seed=1)
torch.manual_seed(11)
pf = GPMDM_PF(model, T, P)
lib, h = _lib.load(), pf._h
phases = {k: [] for k in ("begin", "switch", "normals", "propagate", "uniforms", "resample+preswitch", "read")}
for k in range(40):
    z = np.ascontiguousarray(zs[k], dtype=np.float64)
    s = pf._stream()
    t0 = time.perf_counter()
    if pf._draws is None:
        pf.update(z)
        pf.class_probabilities()
        continue
    # GPMDM_PF.update's replay branch, phase by phase (pre-switch and staged normals included)
    dr, counts = pf._draws, pf._counts
    pE, pC, pN, pU = pf._draw_ptr
    dr.switch()
    if pf._pre_sw and not dr.last_hit:
        _lib.check(lib.gpmdm_pf_preswitch(h, pE, s))
    pf._pre_sw = False
    t1 = time.perf_counter()
    _lib.check(lib.gpmdm_pf_switch(h, pE, pC, s))
    t2 = time.perf_counter()
    dr.dynamics(counts)
    if pf._n_staged:
        _lib.check(lib.gpmdm_pf_stage_normals(h, pN, dr.ahead_valid if dr.last_hit else 0, P * pf.latent_dim, s))
        pf._n_staged = False
    t3 = time.perf_counter()
    pf._propagate(z, dr.N, s, pN)
    t4 = time.perf_counter()
    dr.resample()
    t5 = time.perf_counter()
    _lib.check(lib.gpmdm_pf_resample(h, pU, s))
    pf._readout = None
    if pf._replay_preswitch() and dr.ahead_ready():
        _lib.check(lib.gpmdm_pf_preswitch(h, pE, s))
        _lib.check(lib.gpmdm_pf_stage_normals(h, pN, 0, P * pf.latent_dim, s))
        pf._pre_sw = pf._n_staged = True
    t6 = time.perf_counter()
    pf.class_probabilities()
    t7 = time.perf_counter()
    if k >= 5:
        for name, a, b in zip(phases, (t0, t1, t2, t3, t4, t5, t6), (t1, t2, t3, t4, t5, t6, t7)):
            phases[name].append((b - a) * 1e3)
tot = 0.0
for name, v in phases.items():
    print(f"{name:10s} {np.median(v):7.3f} ms (median), {np.mean(v):7.3f} mean")
    tot += np.median(v)
print(f"frame      {tot:7.3f} ms (sum of medians); threads {pf._draws.threads}, hits {pf._draws.prefetch_hits}, "
      f"counts {pf._counts.tolist()}")
