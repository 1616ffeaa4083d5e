"""The cutoff kernel's launch time under each tile split policy (set_obs_cutoff(split=...)),
from the filter's own stage events on the observation launch, on one box and one stream.

    python tools/cutoff_split_ab.py [--config 2] [--frames 12] [--rounds 2]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--frames", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--P", default=None, help="comma-separated particle counts (default: the config's)")
    a = ap.parse_args()
    import bench
    from gpmdm_amd import GPMDM_PF, synthetic
    bench.WORKLOAD = bench.workload(a.config)
    model, data = bench.build_model(torch.device("cuda", 0))
    model.enable_obs_cutoff(True)
    T = torch.from_numpy(synthetic.markov_matrix(bench.WORKLOAD["C"]))
    Ps = [int(x) for x in a.P.split(",")] if a.P else [bench.WORKLOAD["P_per_gpu"]]
    zs = data.observation_stream(a.warmup + a.frames + 2, seed=1)
    for r, P, split in [(r, P, s) for r in range(a.rounds) for P in Ps for s in ("none", "tail", "all", "auto")]:
        if True:
            torch.manual_seed(11)
            pf = GPMDM_PF(model, T, P, rng="philox", seed=11, obs_cutoff=True)
            pf.set_obs_cutoff(True, split=split)
            for k in range(a.warmup):
                pf.update(zs[k])
            torch.cuda.synchronize()
            pf.stage_times()
            pf.enable_timing(True, stages=("obs_gemm", "obs_finish"))
            for k in range(a.frames):
                pf.update(zs[a.warmup + k])
            torch.cuda.synchronize()
            st = pf.stage_times()
            pf.enable_timing(False)
            row = {"config": a.config, "P": P, "round": r, "split": split,
                   "obs_launch_ms": st["obs_gemm"][0] / max(st["obs_gemm"][1], 1),
                   "obs_finish_ms": st["obs_finish"][0] / max(st["obs_finish"][1], 1)}
            print(json.dumps(row), flush=True)
            del pf


if __name__ == "__main__":
    main()
