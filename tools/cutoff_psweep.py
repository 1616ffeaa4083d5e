"""Cutoff (or dense, --dense) step time against the particle count around the headline P: if the cutoff kernel's
grid runs in whole rounds of equal workgroups (512 slots), the time steps at multiples of
512 x 32 particles instead of growing with P.

    python tools/cutoff_psweep.py [--config 2] [--steps 30]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--dense", action="store_true", help="the dense observation kernel instead")
    ap.add_argument("--split", default=None, choices=("tail", "none", "all"), help="the cutoff's tile split policy")
    ap.add_argument("--ps", default="81920,90112,98304,100000,106496,114688,122880,131072")
    a = ap.parse_args()
    import bench
    from gpmdm_amd import GPMDM_PF, synthetic
    bench.WORKLOAD = bench.workload(a.config)
    model, data = bench.build_model(torch.device("cuda", 0))
    T = torch.from_numpy(synthetic.markov_matrix(bench.WORKLOAD["C"]))
    zs = data.observation_stream(a.steps + a.warmup + 2, seed=1)
    out = []
    for P in [int(x) for x in a.ps.split(",")]:
        pf = GPMDM_PF(model, T, P, rng="philox", seed=11, obs_cutoff=not a.dense)
        if a.split and not a.dense:
            pf.set_obs_cutoff(True, split=a.split)
        for k in range(a.warmup):
            pf.update(zs[k])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.steps):
            pf.update(zs[a.warmup + k])
        torch.cuda.synchronize()
        med = 1e3 * (time.perf_counter() - t0) / a.steps
        row = {"split": a.split, "P": P, "tiles": -(-P // 32), "rounds_at_512": -(-P // 32) / 512, "ms_per_step": med,
               "us_per_1k_particles": 1e3 * med / (P / 1e3)}
        print(json.dumps(row), flush=True)
        out.append(row)
        del pf
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
