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


def _single_device_for_every_rank() -> bool:
    """A rank other than local rank 0 that sees exactly one device may bind
    it when the launcher evidently gave each rank its own GPU (a per-rank
    HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES, or one
    rank per node), or when ranks are told to share it on purpose
    (FDCN_SHARE_DEVICE=1: several ranks rehearsing the sharded path on one
    GPU, tests/test_gpu_multirank.py)."""
    if os.environ.get("FDCN_SHARE_DEVICE") == "1":
        return True
    if any(os.environ.get(v) for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                       "CUDA_VISIBLE_DEVICES")):
        return True
    return int(os.environ.get("LOCAL_WORLD_SIZE", "1")) <= 1


def _choose_device(ords) -> int:
    """The HIP ordinal local rank LOCAL_RANK binds among the visible gfx950
    ordinals (bind_device), or FdcnError."""
    from . import capi
    lr = local_rank()
    if lr < len(ords) and (len(ords) > 1 or lr == 0):
        return ords[lr]
    if len(ords) == 1 and _single_device_for_every_rank():
        return ords[0]
    raise capi.FdcnError(
        f"LOCAL_RANK={lr} (LOCAL_WORLD_SIZE={os.environ.get('LOCAL_WORLD_SIZE', '?')}) but "
        f"only {len(ords)} gfx950 device(s) are visible; give each rank its own device "
        f"(HIP_VISIBLE_DEVICES) or set FDCN_SHARE_DEVICE=1 to share one on purpose")


def bind_device(raise_local: bool = True) -> Optional[int]:
    """One process per GPU: make this rank's GPU current for libfdcn (the
    host-array entry points run on the calling thread's HIP device) and for
    torch (RCCL collectives need it).  Local rank k binds the k-th visible
    gfx950 device (its HIP ordinal may differ on a host with other GPUs).
    When exactly one device is visible every rank binds it only if the
    launcher gave each rank its own (see _single_device_for_every_rank);
    otherwise local ranks > 0 fail, as they do when several devices are
    visible but fewer than the local rank needs: every rank silently marching
    on GPU 0 is the failure this guards.  Returns the HIP ordinal, or None on
    a host with no gfx950 device (CPU tests over gloo).

    Once the process group exists, every rank enters the binding check
    (check_device_binding) whatever happened locally -- a rank with no
    device or a failed binding reports it there -- so every rank raises
    together and none is left waiting in the collective.  Before
    the group exists a failure raises at once; a caller that forms the group
    afterwards (bench.py) passes raise_local=False, keeps the error from
    bind_error() and hands it to check_device_binding after forming it."""
    from . import capi
    global _bind_error
    _bind_error = None
    dev = None
    try:
        ords = capi.device_ordinals()
    except capi.FdcnError:
        ords = []
    try:
        if ords:
            dev = _choose_device(ords)
            capi.select_device(dev)
            try:
                import torch
                if torch.cuda.is_available():
                    torch.cuda.set_device(dev)
            except ImportError:  # pragma: no cover - torch is always present here
                pass
    except capi.FdcnError as e:
        _bind_error, dev = str(e), None
    if is_initialized():  # bound after the group formed (the scenario runners)
        check_device_binding(dev, _bind_error)
    elif _bind_error and raise_local:
        raise capi.FdcnError(_bind_error)
    return dev


_bind_error: Optional[str] = None


def bind_error() -> Optional[str]:
    """The local failure of the last bind_device(raise_local=False), if any."""
    return _bind_error


_VISIBLE_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def check_device_binding(dev: Optional[int], local_error: Optional[str] = None) -> None:
    """Collective check, once the group exists, that every rank bound a
    device and that no two ranks of a host march on the same GPU unless they
    were told to share it.  bind_device accepts a non-empty *_VISIBLE_DEVICES
    with one visible device as a per-rank assignment, which a job-wide
    HIP_VISIBLE_DEVICES=0 with several local ranks also looks like (ADVICE
    r4).  Every rank reports (host name, its visible-device variables, the
    HIP ordinal it bound) and its local binding error, if any: a rank-local
    failure becomes every rank's error, and two equal reports name the same
    physical device.  The decision is taken on the gathered list, so every
    rank raises together (none is left waiting in a later collective)."""
    import socket
    from . import capi
    d = _dist()
    if d is None:
        if local_error:
            raise capi.FdcnError(local_error)
        return
    share = os.environ.get("FDCN_SHARE_DEVICE") == "1"
    me = None if dev is None else (socket.gethostname(),
                                   tuple(os.environ.get(v, "") for v in _VISIBLE_VARS), int(dev))
    reports = [None] * d.get_world_size()
    d.all_gather_object(reports, (me, share, local_error))
    failed = [(r, rep[2]) for r, rep in enumerate(reports) if len(rep) > 2 and rep[2]]
    if failed:
        raise capi.FdcnError("device binding failed on rank(s) " +
                             "; ".join(f"{r}: {msg}" for r, msg in failed))
    seen = {}
    for r, rep in enumerate(reports):
        key, sh = rep[0], rep[1]
        if key is None:
            continue
        if key in seen and not (sh and reports[seen[key]][1]):
            raise capi.FdcnError(
                f"ranks {seen[key]} and {r} both bound HIP device {key[2]} on {key[0]} "
                f"(visible-device variables {dict(zip(_VISIBLE_VARS, key[1]))}); give each "
                f"rank its own device or set FDCN_SHARE_DEVICE=1 to share one on purpose")
        seen.setdefault(key, r)


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


def gather_columns(cols: dict) -> Optional[dict]:
    """Concatenate every rank's result columns (name -> list or array) on rank
    0, in rank order; None elsewhere.  One gather_object of the column dict:
    arrays travel as arrays, not as per-row dicts."""
    d = _dist()
    if d is None:
        return cols
    import numpy as np
    rank, world = d.get_rank(), d.get_world_size()
    # the column schemas first, on every rank, so a mismatch fails every rank
    # together instead of rank 0 alone after the gather; a rank
    # with no rows sends an empty dict and is skipped
    schemas = [None] * world
    d.all_gather_object(schemas, list(cols))
    named = [(r, k) for r, k in enumerate(schemas) if k]
    for r, k in named[1:]:
        if k != named[0][1]:
            raise ValueError(f"gather_columns: rank {r} has columns {k}, rank {named[0][0]} "
                             f"{named[0][1]}")
    parts = [None] * world if rank == 0 else None
    d.gather_object(cols, parts, dst=0)
    if rank != 0:
        return None
    parts = [p for p in parts if p]
    if not parts:
        return {}
    keys = list(parts[0])
    out = {}
    for k in keys:
        vals = [p[k] for p in parts]
        if all(isinstance(v, np.ndarray) for v in vals):
            out[k] = np.concatenate(vals)
        else:
            out[k] = [x for v in vals for x in (v.tolist() if isinstance(v, np.ndarray) else v)]
    return out


def broadcast_rows(rows: Optional[List[dict]]) -> List[dict]:
    """Rank 0's scenario table to every rank."""
    d = _dist()
    if d is None:
        return rows or []
    box = [rows if d.get_rank() == 0 else None]
    d.broadcast_object_list(box, src=0)
    return box[0]
