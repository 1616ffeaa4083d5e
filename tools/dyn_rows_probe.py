import sys, torch
sys.path.insert(0, '.')
import bench
from gpmdm_amd import GPMDM_PF, synthetic
bench.WORKLOAD = bench.workload(2)
model, data = bench.build_model(torch.device("cuda", 0))
T = torch.from_numpy(synthetic.markov_matrix(2))
zs = data.observation_stream(50, seed=1)
for cut in (False, True):
    pf = GPMDM_PF(model, T, 100000, rng="philox", seed=11, obs_cutoff=cut)
    rows = []
    for k in range(48):
        pf.update(zs[k]); rows.append(pf.dynamics_rows())
    print("cutoff" if cut else "dense", rows[8:48:4])
