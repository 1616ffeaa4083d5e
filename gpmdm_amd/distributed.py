"""Particle sharding over ranks (one process per GPU).

Rank r owns particles [r*P/R, (r+1)*P/R) of the dynamics and observation GPs; the
filter state is replicated.  Once per frame every rank's rows {ll, class, state[d]} are
all-gathered into the full P-row array that every rank unpacks before the identical,
replicated normalise/resample.  GPMDM_PF splits the rows in two: {class, state[d]} is known
after the dynamics GP and is all-gathered while the observation GP runs (allgather_rows_start:
with the nccl backend -- RCCL over xGMI -- the collective runs on RCCL's own stream, ordered
after the packing kernel and joined back to torch's current stream, the stream the library
launches on); only {ll} (8 bytes per particle) is exchanged after it.
"""
from __future__ import annotations

import hashlib

import numpy as np
import torch


def _comm_device(group, device):
    """Tensors of a collective live on the GPU for nccl (RCCL), on the host for gloo."""
    import torch.distributed as dist
    return device if dist.get_backend(group) == "nccl" else torch.device("cpu")


def broadcast_array(a: np.ndarray, group=None, device=None) -> np.ndarray:
    """Rank 0's copy of ``a`` (same shape and dtype on every rank) on every rank."""
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(a).copy()).to(_comm_device(group, device))
    dist.broadcast(t, src=dist.get_global_rank(group or dist.group.WORLD, 0), group=group)
    return t.cpu().numpy()


def identical_on_all_ranks(blob: bytes, group=None, device=None) -> bool:
    """True when every rank passed the same bytes (64-bit digest, min == max over ranks)."""
    import torch.distributed as dist
    h = int.from_bytes(hashlib.blake2b(blob, digest_size=8).digest(), "little", signed=True)
    dev = _comm_device(group, device)
    lo = torch.tensor([h], dtype=torch.int64, device=dev)
    hi = lo.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    return int(lo.item()) == int(hi.item())


def shard_range(P: int, world: int, rank: int):
    """[lo, hi) of rank `rank` (the library's own rule, gpmdm_pf_create)."""
    return P * rank // world, P * (rank + 1) // world


def allgather_rows(recv: torch.Tensor, send: torch.Tensor, group=None) -> None:
    """recv (P x W) <- concatenation over ranks of each rank's send (P_r x W).

    Shards may differ in length by one row when P % world != 0, so the collective runs on
    rows padded to the largest shard and the padding is dropped on the way out."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    P, W = recv.shape
    sizes = [shard_range(P, world, r)[1] - shard_range(P, world, r)[0] for r in range(world)]
    mx = max(sizes)
    if all(s == mx for s in sizes) and dist.get_backend(group) != "gloo":
        dist.all_gather_into_tensor(recv, send, group=group)
        return
    padded = torch.zeros((mx, W), dtype=send.dtype, device=send.device)
    padded[: send.shape[0]] = send
    parts = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(parts, padded, group=group)
    off = 0
    for r, s in enumerate(sizes):
        recv[off: off + s] = parts[r][:s]
        off += s


def allgather_rows_start(recv: torch.Tensor, send: torch.Tensor, group=None):
    """Start allgather_rows(recv, send); returns ``wait()``, after which recv is valid on the
    current stream.  nccl: asynchronous (the collective overlaps the kernels the caller
    launches before wait(); wait() orders the current stream after it, without blocking the
    host).  gloo: done before returning (wait() is a no-op)."""
    import torch.distributed as dist
    if dist.get_backend(group) == "gloo":
        allgather_rows(recv, send, group)
        return lambda: None
    world = dist.get_world_size(group)
    P, W = recv.shape
    sizes = [shard_range(P, world, r)[1] - shard_range(P, world, r)[0] for r in range(world)]
    mx = max(sizes)
    if all(s == mx for s in sizes):
        work = dist.all_gather_into_tensor(recv, send, group=group, async_op=True)
        return work.wait
    padded = torch.zeros((mx, W), dtype=send.dtype, device=send.device)
    padded[: send.shape[0]] = send
    parts = [torch.empty_like(padded) for _ in range(world)]
    work = dist.all_gather(parts, padded, group=group, async_op=True)

    def wait():
        work.wait()
        off = 0
        for r, s in enumerate(sizes):
            recv[off: off + s] = parts[r][:s]
            off += s
    return wait
