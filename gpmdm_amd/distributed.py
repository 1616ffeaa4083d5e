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


def gather_plan(P: int, world: int, pad_rows=None):
    """(shard sizes, rows per rank in the collective, padded?) for an all-gather of P rows
    over ``world`` ranks.  Shards differ by at most one row; the collective carries the
    largest shard's rows per rank, or ``pad_rows`` (>= the largest shard; a larger value
    forces the padded path even for even shards -- tests)."""
    sizes = [shard_range(P, world, r)[1] - shard_range(P, world, r)[0] for r in range(world)]
    mx = max(sizes)
    rows = mx if pad_rows is None else int(pad_rows)
    if rows < mx:
        raise ValueError(f"pad_rows {rows} is smaller than the largest shard {mx}")
    return sizes, rows, rows != mx or any(s != mx for s in sizes)


def allgather_rows(recv: torch.Tensor, send: torch.Tensor, group=None) -> None:
    """recv (P x W) <- concatenation over ranks of each rank's send (P_r x W).

    Shards may differ in length by one row when P % world != 0, so the collective runs on
    rows padded to the largest shard and the padding is dropped on the way out."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    P, W = recv.shape
    sizes, mx, uneven = gather_plan(P, world)
    if not uneven and dist.get_backend(group) != "gloo":
        dist.all_gather_into_tensor(recv, send, group=group)
        return
    pbuf = torch.zeros((mx, W), dtype=send.dtype, device=send.device)
    pbuf[: send.shape[0]] = send
    parts = [torch.empty_like(pbuf) for _ in range(world)]
    dist.all_gather(parts, pbuf, group=group)
    off = 0
    for r, s in enumerate(sizes):
        recv[off: off + s] = parts[r][:s]
        off += s


def allgather_rows_start(recv: torch.Tensor, send: torch.Tensor, group=None, pad_rows=None):
    """Start allgather_rows(recv, send); returns ``wait()``, after which recv is valid on the
    current stream.  nccl: asynchronous (the collective overlaps the kernels the caller
    launches before wait(); wait() orders the current stream after it, without blocking the
    host).  gloo: done before returning (wait() is a no-op).  ``pad_rows``: see
    gather_plan (a world-1 test forces the padded gather and copy-back with it)."""
    import torch.distributed as dist
    if dist.get_backend(group) == "gloo":
        allgather_rows(recv, send, group)
        return lambda: None
    world = dist.get_world_size(group)
    P, W = recv.shape
    sizes, mx, uneven = gather_plan(P, world, pad_rows)
    if not uneven:
        work = dist.all_gather_into_tensor(recv, send, group=group, async_op=True)
        return work.wait
    pbuf = torch.zeros((mx, W), dtype=send.dtype, device=send.device)
    pbuf[: send.shape[0]] = send
    parts = [torch.empty_like(pbuf) for _ in range(world)]
    work = dist.all_gather(parts, pbuf, group=group, async_op=True)

    def wait():
        work.wait()
        off = 0
        for r, s in enumerate(sizes):
            recv[off: off + s] = parts[r][:s]
            off += s
    return wait


class RcclComm:
    """An RCCL communicator made by the library (gpmdm_comm_unique_id / gpmdm_comm_init),
    for ``GPMDM_PF.set_comm``.  ``RcclComm.single(device)`` is a one-rank communicator;
    for several ranks, rank 0's ``unique_id()`` bytes reach every rank out of band
    (e.g. a torch.distributed broadcast) and each calls ``RcclComm(world, rank, uid,
    device)`` (collective).  ``destroy()`` after the filters using it."""

    def __init__(self, world: int, rank: int, uid: bytes, device: int):
        import ctypes
        from . import _lib
        if len(uid) != _lib.GPMDM_COMM_ID_BYTES:
            raise ValueError("unique id must be GPMDM_COMM_ID_BYTES bytes")
        buf = ctypes.create_string_buffer(bytes(uid), len(uid))
        h = ctypes.c_void_p()
        _lib.check(_lib.load().gpmdm_comm_init(int(world), int(rank), buf, int(device), ctypes.byref(h)),
                   "gpmdm_comm_init")
        self.ptr = h.value
        self.world, self.rank, self.device = int(world), int(rank), int(device)

    @staticmethod
    def unique_id() -> bytes:
        import ctypes
        from . import _lib
        buf = ctypes.create_string_buffer(_lib.GPMDM_COMM_ID_BYTES)
        _lib.check(_lib.load().gpmdm_comm_unique_id(buf), "gpmdm_comm_unique_id")
        return buf.raw

    @classmethod
    def single(cls, device: int = 0) -> "RcclComm":
        return cls(1, 0, cls.unique_id(), device)

    def destroy(self) -> None:
        from . import _lib
        if self.ptr:
            _lib.check(_lib.load().gpmdm_comm_destroy(self.ptr), "gpmdm_comm_destroy")
            self.ptr = None


class LoopbackComms:
    """TEST ONLY: the library's in-process loopback communicators (gpmdm_comm_init_loopback),
    ``comms[r]`` = rank r of ``len(devices)`` on ``devices[r]`` (a device may repeat).  They
    take the place of RCCL communicators in ``GPMDM_PF.set_comm``: R filters of
    ``shard=(R, r)``, each stepped on a thread of its own, run the library's exchange among
    themselves in this process.  ``destroy()`` after the filters using them."""

    def __init__(self, devices):
        import ctypes
        from . import _lib
        devs = [int(x) for x in devices]
        n = len(devs)
        out = (ctypes.c_void_p * n)()
        _lib.check(_lib.load().gpmdm_comm_init_loopback(n, (ctypes.c_int * n)(*devs), out),
                   "gpmdm_comm_init_loopback")
        self.ptrs = [int(p) for p in out]
        self.devices = devs

    def __getitem__(self, r: int) -> int:
        return self.ptrs[r]

    def __len__(self) -> int:
        return len(self.ptrs)

    def destroy(self) -> None:
        from . import _lib
        for p in self.ptrs:
            if p:
                _lib.check(_lib.load().gpmdm_comm_destroy(p), "gpmdm_comm_destroy")
        self.ptrs = []
