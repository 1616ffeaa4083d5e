"""Host-side costs of the replay draws (no GPU): torch's CPU samplers serial and in threads,
the thread pool's dispatch, and ParallelFrameDraws.dynamics at the headline's class counts
for several chunk sizes -- where the replay frame's normals phase goes."""
import sys
import threading
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gpmdm_amd import replay  # noqa: E402


def tm(f, n=30):
    f()
    t = time.perf_counter()
    for _ in range(n):
        f()
    return (time.perf_counter() - t) / n * 1e6


nthr = replay.host_threads()
print(f"host threads {nthr}, torch intra-op threads {torch.get_num_threads()}")
for name, op in (("normal_", lambda x, g: x.normal_(0, 1, generator=g)),
                 ("uniform_", lambda x, g: x.uniform_(0, 1, generator=g)),
                 ("exponential_", lambda x, g: x.exponential_(1, generator=g))):
    xs = [torch.empty(8192, dtype=torch.float64) for _ in range(16)]
    gs = [torch.Generator() for _ in range(16)]
    one = tm(lambda: op(xs[0], gs[0]))
    line = f"{name:13s} 8192 values: {one:7.1f} us serial ({one / 8192 * 1e3:5.1f} ns/value);"
    for k in (4, 8, 16):
        def work(i, n=20):
            for _ in range(n):
                op(xs[i], gs[i])
        th = [threading.Thread(target=work, args=(i,)) for i in range(k)]
        t = time.perf_counter()
        [h.start() for h in th]
        [h.join() for h in th]
        dt = (time.perf_counter() - t) / 20 * 1e6
        line += f" {k} threads x 8192: {dt:7.1f} us ({k * one / dt:4.1f}x)"
    print(line)
from concurrent.futures import ThreadPoolExecutor  # noqa: E402
pool = ThreadPoolExecutor(nthr)
print(f"pool submit+result of {nthr} no-ops: {tm(lambda: [f.result() for f in [pool.submit(lambda: None) for _ in range(nthr)]]):.1f} us")
w = replay._Walk()
s = torch.get_rng_state().numpy().copy()
w.reset(s, 10 ** 6)
print(f"walk.state: {tm(lambda: w.state(500_000, s)):.1f} us; Generator+set_state: "
      f"{tm(lambda: replay.ParallelFrameDraws._gen(w.state(100))):.1f} us")
P, C, d = 100_000, 2, 3
counts = np.array([89917, 10083])
for native, chunk in ((False, 8192), (True, 4096), (True, 2048), (True, 1024), (True, 512)):
    dr = replay.ParallelFrameDraws(P, C, d, P, chunk=chunk, native=native)
    torch.manual_seed(1)
    ts = {"begin": [], "dynamics": [], "resample": [], "ahead": []}
    for k in range(25):
        t0 = time.perf_counter()
        dr.switch()
        t1 = time.perf_counter()
        dr.dynamics(counts)
        t2 = time.perf_counter()
        dr.resample()
        t3 = time.perf_counter()
        dr.ahead_ready()
        t4 = time.perf_counter()
        for key, v in zip(ts, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            ts[key].append(v)
        time.sleep(0.007)
    dr.close()
    print(f"{'native' if native else 'python pool'} chunk {chunk}: " +
          ", ".join(f"{key} {np.median(v[5:]) * 1e6:.1f} us" for key, v in ts.items()) +
          f" (median; counts {counts.tolist()})")

# the pieces of one dynamics() call: walk states, the native call, its per-chunk floor
nat = replay._Native.load()
if nat is not None:
    import ctypes  # noqa: E402
    flat = torch.empty(400_000, dtype=torch.float64)
    offs = np.arange(17, dtype=np.int64) * 1904 + 200_000
    print(f"walk.states x17: {tm(lambda: w.states(offs, s)):.1f} us")
    st17 = w.states(offs, s)
    for n_ch, per in ((1, 1904), (16, 1904), (16, 64), (1, 64)):
        bounds = np.array([(k * per, (k + 1) * per) for k in range(n_ch)], dtype=np.int64)
        print(f"native normal_ {n_ch} chunks x {per}: "
              f"{tm(lambda: nat.gpmdm_replay_draw_chunks(1, flat.data_ptr(), bounds.ctypes.data, st17.ctypes.data, n_ch, nthr)):.1f} us")
