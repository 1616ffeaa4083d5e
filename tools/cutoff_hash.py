"""Bit-level fingerprint of a cutoff filter's trajectory (sha256 of the exported states, ll,
log-weights and ancestors over a few frames of the bench's stream), to show two builds give
the same bits.

    python tools/cutoff_hash.py [--config 2] [--P 100000] [--frames 5]
"""
from __future__ import annotations

import argparse
import hashlib
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--P", type=int, default=100_000)
    ap.add_argument("--frames", type=int, default=5)
    a = ap.parse_args()
    import bench
    from gpmdm_amd import GPMDM_PF, synthetic
    bench.WORKLOAD = bench.workload(a.config)
    model, data = bench.build_model(torch.device("cuda", 0))
    T = torch.from_numpy(synthetic.markov_matrix(bench.WORKLOAD["C"]))
    zs = data.observation_stream(a.frames + 1, seed=1)
    torch.manual_seed(4)
    pf = GPMDM_PF(model, T, a.P, rng="philox", seed=11, obs_cutoff=True)
    h = hashlib.sha256()
    for k in range(a.frames):
        pf.update(zs[k])
        ex = pf.export_state()
        for key in ("states", "classes", "ll", "log_w", "resample_idx"):
            h.update(np.ascontiguousarray(ex[key]).tobytes())
    print(f"config {a.config} P {a.P} frames {a.frames} sha256 {h.hexdigest()}")


if __name__ == "__main__":
    main()
