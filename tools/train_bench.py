"""Seconds per Adam step of GPMDM.train_adam on the GPU (gpmdm_amd/training.py).

    python tools/train_bench.py [steps] [configs, e.g. 1,2,3]

Synthetic models of the BASELINE.json shapes (SURVEY.md §8(d) generator); one warm-up
step, then ``steps`` timed steps.  Prints one JSON line per config.
"""
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    cfgs = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 3]
    from gpmdm_amd import training
    for cfg in cfgs:
        bench.WORKLOAD = bench.workload(cfg)
        model, _ = bench.build_model(torch.device("cuda", 0))
        tr = training.Trainer(model)
        params = [tr.p[n] for n in training.PARAM_NAMES]
        opt = torch.optim.Adam(params, lr=0.01)

        def step():
            opt.zero_grad()
            loss = tr.loss()
            loss.backward()
            opt.step()
            return loss.item()

        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        s = (time.perf_counter() - t0) / steps
        w = bench.WORKLOAD
        print(json.dumps({"config": cfg, "N": model.X.shape[0], "D": w["D"], "d": w["d"], "C": w["C"],
                          "seconds_per_adam_step": s, "steps": steps}), flush=True)
        del tr, opt, model
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
