"""How much of the cutoff kernel's time is grid imbalance: per particle tile (class order,
the kernel's bounding sphere) the active K-steps n_act and the K-loop positions its chunks
run, then the launch simulated as greedy dispatch (workgroup i to XCD i mod 8, each XCD's
slots taking the next workgroup as one frees) in index order and in longest-first order,
beside the ideal sum / slots.

    python tools/cutoff_sched.py [--config 2] [--frames 7]
"""
from __future__ import annotations

import argparse
import heapq
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from tools.cutoff_cloud import kd_order  # noqa: E402


def makespan(work, slots_per_xcd, n_xcd=8):
    """Greedy in-order dispatch per XCD (round-robin assignment of workgroups to XCDs)."""
    end = 0.0
    for x in range(n_xcd):
        w = work[x::n_xcd]
        h = [0.0] * slots_per_xcd
        for t in w:
            s = heapq.heappop(h)
            heapq.heappush(h, s + t)
        end = max(end, max(h))
    return end


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--frames", type=int, default=7)
    ap.add_argument("--overhead", type=float, default=6.0, help="per-workgroup fixed cost, in K positions")
    a = ap.parse_args()
    import bench
    from gpmdm_amd import GPMDM_PF, synthetic
    bench.WORKLOAD = bench.workload(a.config)
    model, data = bench.build_model(torch.device("cuda", 0))
    T = torch.from_numpy(synthetic.markov_matrix(bench.WORKLOAD["C"]))
    P = bench.WORKLOAD["P_per_gpu"]
    zs = data.observation_stream(a.frames + 2, seed=1)
    pf = GPMDM_PF(model, T, P, rng="philox", seed=11, obs_cutoff=True)
    for k in range(a.frames):
        pf.update(zs[k])
    tau = model.obs_cutoff_tau
    cut = np.sqrt(-np.log(tau))
    ls = np.exp(model.y_log_lengthscales.detach().cpu().numpy())
    X = model.X.detach().cpu().numpy() / ls
    ex = pf.export_state()
    S = ex["states"] / ls
    order = np.argsort(ex["classes"], kind="stable")
    S = S[order]
    leaves = kd_order(X, np.arange(X.shape[0]))
    cen = np.array([X[l].mean(0) for l in leaves])
    rad = np.array([np.sqrt(((X[l] - X[l].mean(0)) ** 2).sum(1)).max() for l in leaves])
    PT = 32 if model.d <= 8 else 64
    TPC = 32
    T_M = (model.D + 15) // 16
    nact, work = [], []
    for i in range(0, P, PT):
        t = S[i:i + PT]
        c = t.mean(0)
        r = float(np.sqrt(((t - c) ** 2).sum(1)).max())
        gap = np.sqrt(((cen - c) ** 2).sum(1)) - r - rad
        na = int(np.sum(~((gap > 0) & (gap * gap > cut * cut))))
        nt = na + T_M
        pos = 0
        for c0 in range(0, nt, TPC):
            last = min(c0 + TPC, nt) - 1
            pos += na if last >= na else last + 1
        nact.append(na)
        work.append(pos + a.overhead)
    work = np.array(work, float)
    out = {"config": a.config, "frames": a.frames, "tiles": len(work),
           "n_act": {"min": int(np.min(nact)), "median": float(np.median(nact)), "max": int(np.max(nact)),
                     "K_steps": len(leaves)},
           "work_positions": {"min": float(work.min()), "median": float(np.median(work)),
                              "mean": float(work.mean()), "max": float(work.max())}}
    lpt = np.sort(work)[::-1]
    for spc in (1, 2, 3, 4):
        slots = 8 * 32 * spc
        ideal = work.sum() / slots
        out[f"{spc}_per_cu"] = {"ideal": ideal, "in_order": makespan(list(work), 32 * spc) / ideal,
                               "longest_first": makespan(list(lpt), 32 * spc) / ideal}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
