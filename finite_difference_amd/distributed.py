"""Scenario sharding across GPUs (one process per GPU, torch.distributed).

Scenarios are independent, so the partition is a contiguous block of rows per
rank and there is no exchange inside the time march.  The only collectives
are at the edges of a batch job: the scenario table is read by every rank
from the same file (or broadcast with ``broadcast_rows``), and the result
rows are gathered to rank 0 (``gather_rows``).  On MI355X the backend is
"nccl" (RCCL over xGMI); the CPU tests use "gloo".  The result payload is a
few hundred bytes per scenario, so these calls are latency-bound.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple, TypeVar

T = TypeVar("T")


def _dist():
    try:
        import torch.distributed as dist
    except Exception:  # pragma: no cover - torch is always present here
        return None
    return dist if dist.is_available() and dist.is_initialized() else None


def is_initialized() -> bool:
    return _dist() is not None


def rank_world() -> Tuple[int, int]:
    d = _dist()
    if d is None:
        return 0, 1
    return d.get_rank(), d.get_world_size()


def local_rank() -> int:
    """This process's GPU ordinal on its node: LOCAL_RANK as torch.distributed.run
    exports it (0 when unset)."""
    return int(os.environ.get("LOCAL_RANK", "0"))


def bind_device() -> Optional[int]:
    """One process per GPU: make GPU `local_rank()` current for libfdcn (the
    host-array entry points run on the calling thread's HIP device) and for
    torch (RCCL collectives need it).  Returns the ordinal, or None on a host
    with no gfx950 device (CPU tests over gloo).  Raises if the rank has no
    GPU of its own -- every rank marching on GPU 0 is the failure this guards."""
    from . import capi
    try:
        n = capi.device_count()
    except capi.FdcnError:
        return None
    if n == 0:
        return None
    lr = local_rank()
    if lr >= n:
        raise capi.FdcnError(f"LOCAL_RANK={lr} but only {n} gfx950 device(s) are visible")
    capi.select_device(lr)
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.set_device(lr)
    except ImportError:  # pragma: no cover - torch is always present here
        pass
    return lr


def shard_range(n: int, rank: Optional[int] = None, world: Optional[int] = None) -> range:
    """Contiguous, balanced block [lo, hi) of n items for `rank`."""
    if rank is None or world is None:
        rank, world = rank_world()
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return range(lo, hi)


def shard(items: Sequence[T]) -> List[T]:
    r = shard_range(len(items))
    return list(items[r.start:r.stop])


def gather_rows(rows: List[dict]) -> Optional[List[dict]]:
    """Concatenate every rank's rows on rank 0 (in rank order); None elsewhere."""
    d = _dist()
    if d is None:
        return rows
    rank, world = d.get_rank(), d.get_world_size()
    out = [None] * world if rank == 0 else None
    d.gather_object(rows, out, dst=0)
    if rank != 0:
        return None
    merged: List[dict] = []
    for part in out:
        merged.extend(part)
    return merged


def broadcast_rows(rows: Optional[List[dict]]) -> List[dict]:
    """Rank 0's scenario table to every rank."""
    d = _dist()
    if d is None:
        return rows or []
    box = [rows if d.get_rank() == 0 else None]
    d.broadcast_object_list(box, src=0)
    return box[0]
