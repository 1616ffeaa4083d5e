"""World-size-2 gloo tests of the multi-rank host path (CPU only)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, P, W, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gpmdm_amd.distributed import allgather_rows, shard_range
        from gpmdm_amd import replay
        lo, hi = shard_range(P, world, rank)
        send = torch.arange(lo * W, hi * W, dtype=torch.float64).reshape(hi - lo, W)
        recv = torch.full((P, W), -1.0, dtype=torch.float64)
        allgather_rows(recv, send)
        ok_rows = bool(torch.equal(recv, torch.arange(P * W, dtype=torch.float64).reshape(P, W)))
        # the split exchange's start/wait form (GPMDM_PF._propagate): {class, state} columns
        # started first, {ll} gathered and waited, then the first completed
        from gpmdm_amd.distributed import allgather_rows_start
        rs, rl = torch.full((P, W - 1), -1.0, dtype=torch.float64), torch.full((P, 1), -1.0, dtype=torch.float64)
        wait_s = allgather_rows_start(rs, send[:, 1:].contiguous())
        allgather_rows_start(rl, send[:, :1].contiguous())()
        wait_s()
        ok_rows = ok_rows and bool(torch.equal(torch.cat([rl, rs], 1), recv))
        # replicated draws: every rank seeds torch identically and draws the same streams
        torch.manual_seed(123)
        E = replay.switch_draws(P, 3)
        g = [torch.empty_like(torch.tensor(E)) for _ in range(world)]
        dist.all_gather(g, torch.tensor(E))
        ok_draws = all(torch.equal(g[0], x) for x in g)
        out_q.put((rank, ok_rows, ok_draws))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P", [8, 7])   # even and uneven shards
def test_allgather_rows_two_ranks(P):
    world, W = 2, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, W, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_rows, ok_draws in res:
        assert ok_rows, f"rank {rank}: gathered rows wrong"
        assert ok_draws, f"rank {rank}: replicated draws differ"


def test_shard_ranges_cover():
    from gpmdm_amd.distributed import shard_range
    for P in (1, 7, 100, 100_001):
        for world in (1, 2, 3, 8):
            r = [shard_range(P, world, k) for k in range(world)]
            assert r[0][0] == 0 and r[-1][1] == P
            assert all(r[k][1] == r[k + 1][0] for k in range(world - 1))


def _bcast_worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gpmdm_amd.distributed import broadcast_array, identical_on_all_ranks
        a = np.arange(12, dtype=np.float64).reshape(3, 4) * (rank + 1)
        b = broadcast_array(a)
        seed = broadcast_array(np.array([1000 + rank], dtype=np.int64))
        same = identical_on_all_ranks(b"abc")
        differ = identical_on_all_ranks(bytes([rank]))
        out_q.put((rank, b, int(seed[0]), same, differ))
    finally:
        dist.destroy_process_group()


def test_broadcast_and_consistency_check_two_ranks():
    """The helpers GPMDM_PF(process_group=...) uses so every rank holds one replicated
    filter: rank 0's seed / particles broadcast, and the replay-mode RNG-state check."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, b, seed, same, differ in res:
        assert np.array_equal(b, np.arange(12, dtype=np.float64).reshape(3, 4)), rank
        assert seed == 1000 and same and not differ


def test_gather_plan():
    """The branch choice of the all-gather (even shards -> one all_gather_into_tensor;
    uneven, or padding forced -> padded gather + copy-back) as a pure function."""
    from gpmdm_amd.distributed import gather_plan
    assert gather_plan(8, 2) == ([4, 4], 4, False)
    assert gather_plan(7, 2) == ([3, 4], 4, True)
    assert gather_plan(7, 1) == ([7], 7, False)
    assert gather_plan(7, 1, pad_rows=9) == ([7], 9, True)
    assert gather_plan(10, 3)[0] == [3, 3, 4]
    with pytest.raises(ValueError):
        gather_plan(7, 2, pad_rows=3)


def test_device_shard_plan():
    """GPMDM_PF(devices=[...]): rank r on devices[r] owns the library's shard of particles."""
    from gpmdm_amd.pf import device_shard_plan
    from gpmdm_amd.distributed import shard_range
    for P in (1, 7, 100_000, 1_000_001):
        for devs in ([0], [0, 1], [3, 1, 2], list(range(8))):
            plan = device_shard_plan(P, devs)
            assert [p[0] for p in plan] == devs and [p[1] for p in plan] == list(range(len(devs)))
            assert plan[0][2] == 0 and plan[-1][3] == P
            assert all(plan[k][3] == plan[k + 1][2] for k in range(len(devs) - 1))
            assert all((p[2], p[3]) == shard_range(P, len(devs), p[1]) for p in plan)
    for bad in ([], [0, 0], [1, -1]):
        with pytest.raises(ValueError):
            device_shard_plan(10, bad)
