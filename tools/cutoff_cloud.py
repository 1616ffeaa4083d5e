"""Why the cutoff kernel runs the MFMA groups it runs: the bench's cloud (Philox, the mocap
stream, obs_cutoff=True) after a few frames -- its extent in the observation GP's scaled
latent space, the radius of its particle tiles in index order, and the fraction of training
K-steps (spatial order, host_image.h) within the cutoff distance of the cloud's bounding
sphere and of each tile's -- beside the kernel's own count of MFMA groups run.

    python tools/cutoff_cloud.py [--config 2] [--frames 7]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def kd_order(X, idx, leaf=16):
    if len(idx) <= leaf:
        return [idx]
    sub = X[idx]
    j = int(np.argmax(sub.max(0) - sub.min(0)))
    o = idx[np.lexsort((idx, sub[:, j]))]
    leaves = (len(o) + leaf - 1) // leaf
    left = ((leaves + 1) // 2) * leaf
    return kd_order(X, o[:left], leaf) + kd_order(X, o[left:], leaf)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--frames", type=int, default=7)
    a = ap.parse_args()
    import bench
    from gpmdm_amd import GPMDM_PF, synthetic
    bench.WORKLOAD = bench.workload(a.config)
    model, data = bench.build_model(torch.device("cuda", 0))
    T = torch.from_numpy(synthetic.markov_matrix(bench.WORKLOAD["C"]))
    P = bench.WORKLOAD["P_per_gpu"]
    zs = data.observation_stream(a.frames + 2, seed=1)
    pf = GPMDM_PF(model, T, P, rng="philox", seed=11, obs_cutoff=True)
    pf.set_obs_cutoff(True, stats=True)
    for k in range(a.frames):
        pf.obs_cutoff_stats(reset=True)
        pf.update(zs[k])
    st = pf.obs_cutoff_stats()
    tau = model.obs_cutoff_tau
    cut = np.sqrt(-np.log(tau))
    ls = np.exp(model.y_log_lengthscales.detach().cpu().numpy())
    X = model.X.detach().cpu().numpy() / ls
    ex = pf.export_state()
    S = ex["states"] / ls
    w = ex["w"]
    c = S.mean(0)
    r_cloud = float(np.sqrt(((S - c) ** 2).sum(1)).max())
    leaves = kd_order(X, np.arange(X.shape[0]))
    cen = np.array([X[l].mean(0) for l in leaves])
    rad = np.array([np.sqrt(((X[l] - X[l].mean(0)) ** 2).sum(1)).max() for l in leaves])
    gap = np.sqrt(((cen - c) ** 2).sum(1)) - r_cloud - rad
    f_cloud = float(np.mean(~((gap > 0) & (gap > cut))))
    PT = 32 if model.d <= 8 else 64
    tr = [float(np.sqrt(((S[i:i + PT] - S[i:i + PT].mean(0)) ** 2).sum(1)).max()) for i in range(0, P, PT)]
    anc = len(np.unique(ex["resample_idx"]))
    out = {"config": a.config, "frames": a.frames, "tau": tau, "cutoff_distance": float(cut),
           "cloud_radius_scaled": r_cloud, "latent_extent_scaled": float(np.sqrt(((X - X.mean(0)) ** 2).sum(1)).max()),
           "ess": float(1.0 / np.sum(w * w)), "distinct_ancestors": anc,
           "ksteps_within_cutoff_of_cloud_sphere": f_cloud,
           "tile_radius_index_order": {"median": float(np.median(tr)), "max": float(np.max(tr))},
           "kernel_mfma_groups_run_fraction_last_frame": st["fraction_run"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
