"""Particle sharding over ranks (one process per GPU).

Rank r owns particles [r*P/R, (r+1)*P/R) of the dynamics and observation GPs; the
filter state is replicated.  Once per frame every rank packs its rows {ll, class,
state[d]} (gpmdm_pf_pack) and one all-gather builds the full P x (d+2) array that every
rank unpacks (gpmdm_pf_unpack) before the identical, replicated normalise/resample.  With
the nccl backend (RCCL over xGMI) the tensors live on the GPU and the collective runs on
torch's current stream, the same stream the library launches on.
"""
from __future__ import annotations

import torch


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
