"""Per-rank step time of the weak-scaling bench at N ranks, simulated on one GPU.

Rank 0 of N is built with ``shard=(N, 0)`` (100k particles of its own, P_total = 100k N
replicated) and an exchange that tiles its own packed rows over the receive buffer in place
of the RCCL all-gather.  Everything the rank computes is real -- the replicated O(P_total)
switch / grouping / normalise / resample / read-out kernels grow with N -- and only the
collective itself is missing, so the result is the compute floor of each rank's step.

    python tools/scale_sim.py [steps] [N,N,...]
"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    bench.WORKLOAD = bench.workload(2)
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
        t0 = time.perf_counter()
        for k in range(steps):
            pf.update(zs[5 + k])
            pf.get_most_likely_class()
            pf.class_probabilities()
            pf.current_state_mean()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        print(f"N={n}: P_total={P}, per-rank step {ms:.3f} ms (no collective), "
              f"weak-scaling floor {100_000 * n * 1e3 / ms:.3e} particle-steps/s", flush=True)
        del pf


if __name__ == "__main__":
    main()
