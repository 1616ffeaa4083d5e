"""Host-side profile of the notebook loop (bench.py --config 1 workload): cProfile over
200 frames of update + get_most_likely_class + class_probabilities + current_state_mean,
after warm-up.  Run on the GPU box: python tools/notebook_profile.py > out.txt"""
import cProfile
import io
import pstats
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
from gpmdm_amd import GPMDM_PF, synthetic  # noqa: E402

bench.WORKLOAD = bench.workload(1)
bench.WORKLOAD["y_lambda"] = 1.0
dev = torch.device("cuda", 0)
model, data = bench.build_model(dev)
T = torch.from_numpy(synthetic.markov_matrix(bench.WORKLOAD["C"]))
torch.manual_seed(11)
pf = GPMDM_PF(model, T, bench.WORKLOAD["P_per_gpu"], rng="torch")
zs = data.observation_stream(260, seed=1)


def one(k):
    pf.update(zs[k])
    pf.get_most_likely_class()
    pf.class_probabilities()
    pf.current_state_mean()


for k in range(20):
    one(k)
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(20, 220):
    one(k)
torch.cuda.synchronize()
print(f"plain: {(time.perf_counter() - t0) / 200 * 1e3:.4f} ms/frame")
pr = cProfile.Profile()
pr.enable()
for k in range(20, 220):
    one(k)
torch.cuda.synchronize()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
print(s.getvalue())
