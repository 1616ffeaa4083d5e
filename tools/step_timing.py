"""Per-step host wall times of the bench loop (config 2): distribution and host-side split
(update call vs read-out wait).  Diagnostic for the gap between the kernel timeline and
bench.py's ms_per_step.

    python tools/step_timing.py [steps]
"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    bench.WORKLOAD = bench.workload(2)
    from gpmdm_amd import GPMDM_PF, synthetic
    dev = torch.device("cuda", 0)
    model, data = bench.build_model(dev)
    pf = GPMDM_PF(model, torch.from_numpy(synthetic.markov_matrix(2)), 100_000, rng="philox", seed=11)
    zs = data.observation_stream(steps + 10, seed=1)
    for k in range(10):
        pf.update(zs[k])
        pf.class_probabilities()
    torch.cuda.synchronize()
    tu, tr, tt = [], [], []
    for k in range(steps):
        t0 = time.perf_counter()
        pf.update(zs[10 + k])
        t1 = time.perf_counter()
        pf.get_most_likely_class()
        pf.class_probabilities()
        pf.current_state_mean()
        t2 = time.perf_counter()
        tu.append(t1 - t0)
        tr.append(t2 - t1)
        tt.append(t2 - t0)
    for name, a in (("update call", tu), ("read wait", tr), ("step", tt)):
        a = np.array(a) * 1e3
        print(f"{name:12s} mean {a.mean():.3f} ms  p50 {np.median(a):.3f}  min {a.min():.3f}  max {a.max():.3f}")


if __name__ == "__main__":
    main()
