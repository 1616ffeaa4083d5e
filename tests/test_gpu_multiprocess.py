"""GPU: the real process-group path -- GPMDM_PF(process_group=...) in separate processes.

Two ranks are spawned on this box's GPU with the gloo backend (RCCL refuses two ranks on
one device; gloo moves the all-gather through host memory, the library and every kernel
are the same as with nccl).  Each rank seeds torch *differently*: the filter must still be
one replicated filter, because the Philox seed and the initial particles are broadcast
from rank 0 (gpmdm_amd/pf.py).  After 3 frames every rank's states, classes, ll,
resample indices and read-outs must be bitwise equal to a single-rank filter built in
the parent with rank 0's torch seed.  Replay mode (rng='torch') with identical torch
seeds is bitwise as well; with different seeds it must refuse (ValueError) instead of
silently diverging.
"""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import product_model

pytestmark = pytest.mark.gpu

P = 10_001
FRAMES = 3


def _store_file():
    """A fresh rendezvous file for a FileStore (no TCP port to race for: a port found free
    and released can be taken again, or sit in TIME_WAIT, before the store listens)."""
    import tempfile
    fd, path = tempfile.mkstemp(prefix="gpmdm_store_")
    os.close(fd)
    os.unlink(path)
    return path


def _obs(m):
    Y = m.get_Y()
    return [np.asarray(Y[200 + 5 * k], dtype=np.float64) for k in range(FRAMES)]


def _worker(rank, world, store_path, rng, seeds, out_q):
    import faulthandler
    import sys
    import torch.distributed as dist
    # a rank that hangs dumps its stacks and exits (the parent's queue wait then fails with
    # the dump in the captured stderr) instead of holding the run until an outer watchdog
    faulthandler.dump_traceback_later(100, exit=True, file=sys.stderr)
    from conftest import load_fixture
    from gpmdm_amd import GPMDM_PF
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", store=dist.FileStore(store_path, world), rank=rank, world_size=world)
    try:
        m = product_model(load_fixture("config2_n2000_p1000"))
        T = torch.tensor([[0.9, 0.1], [0.1, 0.9]])
        torch.manual_seed(seeds[rank])
        try:
            pf = GPMDM_PF(m, T, P, rng=rng, process_group=dist.group.WORLD)
        except ValueError as e:
            out_q.put((rank, "ValueError", str(e)))
            return
        for z in _obs(m):
            pf.update(z)
        st = pf.export_state()
        out_q.put((rank, "ok", dict(states=st["states"], classes=st["classes"], ll=st["ll"],
                                     resample_idx=st["resample_idx"],
                                     post=pf.class_probabilities().numpy(),
                                     mean=pf.current_state_mean().numpy(), lik=pf.log_likelihood(),
                                     seed=pf._seed)))
    finally:
        dist.destroy_process_group()


def _run(rng, seeds):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = _store_file()
    procs = [ctx.Process(target=_worker, args=(r, world, store, rng, seeds, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict((r, (kind, payload)) for r, kind, payload in (q.get(timeout=130) for _ in range(world)))
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return res


def _single(m, rng, seed_torch):
    from gpmdm_amd import GPMDM_PF
    T = torch.tensor([[0.9, 0.1], [0.1, 0.9]])
    torch.manual_seed(seed_torch)
    pf = GPMDM_PF(m, T, P, rng=rng)
    for z in _obs(m):
        pf.update(z)
    return pf


@pytest.mark.timeout(400)
@pytest.mark.parametrize("rng,seeds", [("philox", (100, 101)), ("torch", (7, 7))])
def test_process_group_filter_matches_single_rank(fx_config2, rng, seeds):
    res = _run(rng, seeds)
    m = product_model(fx_config2)
    ref = _single(m, rng, seeds[0])
    a = ref.export_state()
    for r in range(2):
        kind, got = res[r]
        assert kind == "ok", got
        if rng == "philox":
            assert got["seed"] == ref._seed
        for key in ("states", "classes", "ll", "resample_idx"):
            assert np.array_equal(a[key], got[key]), (r, key)
        assert np.array_equal(ref.class_probabilities().numpy(), got["post"])
        assert np.array_equal(ref.current_state_mean().numpy(), got["mean"])
        assert ref.log_likelihood() == got["lik"]


@pytest.mark.timeout(400)
def test_process_group_replay_refuses_different_torch_states():
    res = _run("torch", (7, 8))
    for r in range(2):
        kind, msg = res[r]
        assert kind == "ValueError" and "identical torch RNG" in msg


def _nccl_worker(store_path, out_q):
    """World-size-1 RCCL group: the asynchronous all-gather GPMDM_PF overlaps with the
    observation GP (distributed.allgather_rows_start, nccl branch), with kernels queued on
    the current stream between start and wait.  Both branches run: the even
    all_gather_into_tensor and -- forced with pad_rows, since one rank's shard is never
    uneven -- the padded gather with its copy-back in wait()."""
    import torch.distributed as dist
    from gpmdm_amd.distributed import allgather_rows_start
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", store=dist.FileStore(store_path, 1), rank=0, world_size=1, device_id=dev)
    try:
        ok = True
        for P, W, pad in ((100_000, 4, None), (7, 1, None), (100_000, 4, 100_001), (7, 1, 9)):
            send = torch.arange(P * W, dtype=torch.float64, device=dev).reshape(P, W)
            recv = torch.full((P, W), -1.0, dtype=torch.float64, device=dev)
            wait = allgather_rows_start(recv, send, pad_rows=pad)
            busy = torch.randn(2048, 2048, dtype=torch.float64, device=dev)
            for _ in range(4):                     # work on the current stream meanwhile
                busy = busy @ busy * 1e-3
            wait()
            ok = ok and bool(torch.equal(recv, send))
        torch.cuda.synchronize()
        out_q.put(("ok", ok))
    except Exception as e:                         # noqa: BLE001 -- reported to the parent
        out_q.put(("error", repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_async_allgather_world1():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_store_file(), q))
    p.start()
    try:
        kind, payload = q.get(timeout=130)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert kind == "ok", payload
    assert payload
    assert p.exitcode == 0
