"""Per-rank step time of the weak-scaling bench at N ranks, simulated on one GPU.

Rank 0 of N is built with ``shard=(N, 0)`` (100k particles of its own, P_total = 100k N
replicated) and an exchange that tiles its own packed rows over the receive buffer in place
of the RCCL all-gather.  Everything the rank computes is real -- the replicated O(P_total)
switch / grouping / normalise / resample / read-out kernels grow with N -- and only the
collective itself is missing, so the result is the compute floor of each rank's step.

    python tools/scale_sim.py [steps] [N,N,...]
    python tools/scale_sim.py --ranks [--no-order] [--per-rank=P] [steps] [N,N,...]

--ranks runs all N ranks on the one GPU, one after another, with the real exchange done
in-process (the data every rank sees is exactly what an N-GPU run sees), and reports each
rank's GPU time per step from its stage events (kernels only, no host gaps) and its
dynamics-GP rows; the slowest rank bounds the N-GPU step.

The RCCL all-gathers are modelled, not measured (one GPU here): every rank receives the
(N-1)/N share of P_total rows.  Two bounds per N: a ring on one xGMI link per GPU
(153 GB/s) and the ring's chunks spread over min(N-1, 7) links (RCCL's channels use
distinct links on the fully connected 8-GPU node).  GPMDM_PF exchanges {class, state}
(d+1 doubles per row) while the observation GP runs and {ll} (1 double) after it, so the
modelled step is the slowest rank's compute + the ll gather + whatever of the state
gather the observation GP does not cover; the fully serial figure (one (d+2)-wide gather
after the step's compute) is printed beside it.
"""

XGMI_LINK_GBPS = 153.0


def allgather_ms(P_total, width, n):
    """(one-link ring, multi-link) all-gather time in ms for P_total rows of `width` doubles."""
    if n == 1:
        return 0.0, 0.0
    recv = (n - 1) / n * P_total * width * 8.0
    return recv / (XGMI_LINK_GBPS * 1e9) * 1e3, recv / (XGMI_LINK_GBPS * 1e9 * min(n - 1, 7)) * 1e3
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    bench.WORKLOAD = bench.workload(2)
    bench.WORKLOAD["y_lambda"] = 1.0           # the headline (mocap) stream's model
    from gpmdm_amd import GPMDM_PF, synthetic
    dev = torch.device("cuda", 0)
    model, data = bench.build_model(dev)
    T = torch.from_numpy(synthetic.markov_matrix(2))
    zs = data.observation_stream(steps + 5, seed=1)
    ns = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4, 8]
    for n in ns:
        P = 100_000 * n

        def tile(recv, send, n=n):
            recv.view(n, -1, recv.shape[1]).copy_(send.unsqueeze(0).expand(n, -1, -1))

        pf = GPMDM_PF(model, T, P, rng="philox", seed=11, shard=(n, 0) if n > 1 else None,
                      exchange=tile if n > 1 else None)
        for k in range(5):
            pf.update(zs[k])
            pf.class_probabilities()
        torch.cuda.synchronize()
        pf.stage_times()
        pf.enable_timing(True)
        t0 = time.perf_counter()
        for k in range(steps):
            pf.update(zs[5 + k])
            pf.get_most_likely_class()
            pf.class_probabilities()
            pf.current_state_mean()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        pf.enable_timing(False)
        st = {k: round(v[0] / max(v[1], 1), 4) for k, v in pf.stage_times().items()}
        print(f"N={n}: P_total={P}, per-rank step {ms:.3f} ms (no collective), "
              f"weak-scaling floor {100_000 * n * 1e3 / ms:.3e} particle-steps/s; "
              f"dyn rows {pf.dynamics_rows()}; stages ms {st}", flush=True)
        del pf


def ranks_mode():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    order = "--no-order" not in sys.argv
    per_rank = next((int(a.split("=")[1]) for a in sys.argv if a.startswith("--per-rank=")), 100_000)
    steps = int(args[0]) if args else 20
    bench.WORKLOAD = bench.workload(2)
    bench.WORKLOAD["y_lambda"] = 1.0           # the headline (mocap) stream's model
    from gpmdm_amd import GPMDM_PF, synthetic
    dev = torch.device("cuda", 0)
    model, data = bench.build_model(dev)
    T = torch.from_numpy(synthetic.markov_matrix(2))
    zs = data.observation_stream(steps + 5, seed=1)
    ns = [int(x) for x in args[1].split(",")] if len(args) > 1 else [1, 2, 4, 8]
    for n in ns:
        P = per_rank * n
        pfs = []
        for r in range(n):                  # same initial particles on every rank (torch draws)
            torch.manual_seed(11)
            pfs.append(GPMDM_PF(model, T, P, rng="philox", seed=11, shard=(n, r) if n > 1 else None,
                                shard_order=order))

        def step(k):
            if n == 1:
                pfs[0].update(zs[k])
            else:
                full = torch.cat([pf._stage_propagate(zs[k]) for pf in pfs], 0)
                for pf in pfs:
                    pf._recv.copy_(full)
                    pf._stage_resample()
            for pf in pfs:
                pf.class_probabilities()

        for k in range(5):
            step(k)
        torch.cuda.synchronize()
        for pf in pfs:
            pf.stage_times()
            pf.enable_timing(True)
        rows = [0] * n
        for k in range(steps):
            step(5 + k)
            for r, pf in enumerate(pfs):
                rows[r] += pf.dynamics_rows()
        torch.cuda.synchronize()
        per = []
        for pf in pfs:
            pf.enable_timing(False)
            st = pf.stage_times()
            per.append({k: v[0] / max(v[1], 1) for k, v in st.items()})
        tot = [sum(p.values()) for p in per]
        worst = max(range(n), key=lambda r: tot[r])
        ser1, serm = allgather_ms(P, model.d + 2, n)
        st1, stm = allgather_ms(P, model.d + 1, n)
        ll1, llm = allgather_ms(P, 1, n)
        obs = per[worst]["obs_gemm"] + per[worst]["obs_finish"]
        ag1, agm = ll1 + max(0.0, st1 - obs), llm + max(0.0, stm - obs)
        print(f"[shard_order={order}] N={n}: serial exchange (one gather after compute) "
              f"{ser1:.3f} / {serm:.3f} ms -> step {max(tot) + ser1:.3f} / {max(tot) + serm:.3f} ms", flush=True)
        print(f"[shard_order={order}] N={n}: P_total={P}, GPU ms per step per rank: max {max(tot):.3f} min {min(tot):.3f} "
              f"(rank {worst}: dyn_gemm {per[worst]['dyn_gemm']:.3f} obs_gemm {per[worst]['obs_gemm']:.3f} "
              f"switch {per[worst]['switch']:.3f} resample {per[worst]['resample']:.3f}); "
              f"dyn rows per rank (mean over steps): {[r // steps for r in rows]}; "
              f"modelled exposed exchange (states overlapped with the observation GP, then ll) {ag1:.3f} ms (1 link) / {agm:.3f} ms ({min(max(n - 1, 1), 7)} links) -> "
              f"step {max(tot) + ag1:.3f} / {max(tot) + agm:.3f} ms, "
              f"{P * 1e3 / (max(tot) + ag1):.3e} / {P * 1e3 / (max(tot) + agm):.3e} particle-steps/s", flush=True)
        del pfs


if __name__ == "__main__":
    ranks_mode() if "--ranks" in sys.argv else main()
