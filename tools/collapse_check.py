"""Dynamics rows per frame of a single P=200k Philox filter and of 2 logical ranks (in-process
exchange) on the bench model, over the frame sequence bench.py runs at --steps 5 --warmup 2."""
import sys, torch, numpy as np
sys.path.insert(0, "/root/repo")
import bench
bench.WORKLOAD = bench.workload(2)
from gpmdm_amd import GPMDM_PF, synthetic
dev = torch.device("cuda", 0)
model, data = bench.build_model(dev)
T = torch.from_numpy(synthetic.markov_matrix(2))
zs0 = data.observation_stream(7, seed=1)
zs = [zs0[i] for i in list(range(7)) + list(range(2, 7))]   # bench.py at --gpus 2 --steps 5 --warmup 2: timed frames, then the breakdown pass
P = 200_000
torch.manual_seed(11)
ref = GPMDM_PF(model, T, P, rng="philox", seed=11)
ranks = []
for r in range(2):
    torch.manual_seed(11)
    ranks.append(GPMDM_PF(model, T, P, rng="philox", seed=11, shard=(2, r)))
for k in range(len(zs)):
    ref.update(zs[k])
    full = torch.cat([pf._stage_propagate(zs[k]) for pf in ranks], 0)
    for pf in ranks:
        pf._recv.copy_(full)
        pf._stage_resample()
    a, b = ref.export_state(), ranks[0].export_state()
    same = all(np.array_equal(a[key], b[key]) for key in ("states", "classes", "ll"))
    print(k, "ref rows", ref.dynamics_rows(), "rank rows", [pf.dynamics_rows() for pf in ranks], "same", same,
          ref.class_probabilities().numpy(), flush=True)
