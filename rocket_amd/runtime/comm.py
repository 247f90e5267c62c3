"""Process-group bootstrap and collectives.

Replaces what the reference reaches through ``accelerate.PartialState`` and
``accelerate.utils.broadcast_object_list`` (``rocket/core/launcher.py:150,161,291``;
SURVEY §2.5 N2/N12/N13, §3.5).

Design (MI355X-first):

* one process per GPU; rank/world/local-rank come from the ``torchrun``
  environment; the device is ``cuda:LOCAL_RANK`` (a HIP device);
* the tensor process group is ``nccl`` — RCCL on ROCm — when GPUs are present,
  ``gloo`` on CPU.  The group is created *eagerly* with ``device_id`` so the RCCL
  communicator exists before the first step (no lazy init inside a timed loop
  or a graph capture);
* host-side object traffic (project-dir broadcast, barriers, metric objects)
  runs on a separate **gloo** group over the TCP store so it never touches the
  GPU or RCCL streams;
* the process group is initialised *before* anything else collective happens —
  fixing the reference's ordering hazard Q9, where the project-dir broadcast
  created a state before the accelerator and CPU multi-process runs silently
  went un-distributed.
"""

from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Any, List

import torch
import torch.distributed as dist


@dataclass
class ProcessContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    num_nodes: int = 1
    device: torch.device = torch.device("cpu")
    backend: str | None = None
    host_group: Any = None  # gloo group for object collectives
    owns_group: bool = False

    @property
    def distributed(self) -> bool:
        return self.world_size > 1

    @property
    def is_main_process(self) -> bool:
        return self.rank == 0

    @property
    def is_local_main_process(self) -> bool:
        return self.local_rank == 0


_CTX: ProcessContext | None = None


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def use_gpu(cpu: bool | None = None) -> bool:
    if cpu is None:
        cpu = os.environ.get("ROCKET_CPU", os.environ.get("ACCELERATE_USE_CPU", "0")).lower() in ("1", "true", "yes")
    return (not cpu) and torch.cuda.is_available()


def init(cpu: bool | None = None, timeout_s: float | None = None) -> ProcessContext:
    """Initialise (once) and return the process context."""
    global _CTX
    if _CTX is not None and (not _CTX.distributed or dist.is_initialized()):
        return _CTX

    world = _env_int("WORLD_SIZE", 1)
    rank = _env_int("RANK", 0)
    local_rank = _env_int("LOCAL_RANK", rank)
    local_world = _env_int("LOCAL_WORLD_SIZE", world)
    gpu = use_gpu(cpu)

    if gpu:
        ndev = torch.cuda.device_count()
        device = torch.device("cuda", local_rank % max(ndev, 1))
        torch.cuda.set_device(device)
    else:
        device = torch.device("cpu")

    backend = None
    host_group = None
    owns = False
    if world > 1:
        timeout = datetime.timedelta(seconds=timeout_s or float(os.environ.get("ROCKET_PG_TIMEOUT", "1800")))
        if not dist.is_initialized():
            # ROCKET_DIST_BACKEND=gloo: rehearse multi-rank GPU paths with several ranks on one device
            backend = os.environ.get("ROCKET_DIST_BACKEND") or ("nccl" if gpu else "gloo")
            kwargs = dict(backend=backend, timeout=timeout)
            if gpu and backend == "nccl":
                kwargs["device_id"] = device
            dist.init_process_group(**kwargs)
            owns = True
        backend = dist.get_backend()
        rank, world = dist.get_rank(), dist.get_world_size()
        host_group = dist.new_group(backend="gloo", timeout=timeout) if backend != "gloo" else dist.group.WORLD

    _CTX = ProcessContext(
        rank=rank,
        world_size=world,
        local_rank=local_rank,
        local_world_size=local_world,
        num_nodes=max(1, world // max(local_world, 1)),
        device=device,
        backend=backend,
        host_group=host_group,
        owns_group=owns,
    )
    return _CTX


def context() -> ProcessContext:
    return _CTX if _CTX is not None else init()


def shutdown() -> None:
    """Destroy the process group (reference ``Launcher.destroy_process_group``)."""
    global _CTX
    if dist.is_available() and dist.is_initialized():
        try:
            dist.barrier(group=_CTX.host_group if _CTX else None)
        except Exception:
            pass
        dist.destroy_process_group()
    _CTX = None


# ---------------------------------------------------------------- host objects
def broadcast_object(obj: Any, src: int = 0) -> Any:
    ctx = context()
    if not ctx.distributed:
        return obj
    box = [obj]
    dist.broadcast_object_list(box, src=src, group=ctx.host_group)
    return box[0]


def all_gather_object(obj: Any) -> List[Any]:
    ctx = context()
    if not ctx.distributed:
        return [obj]
    out: List[Any] = [None] * ctx.world_size
    dist.all_gather_object(out, obj, group=ctx.host_group)
    return out


def all_ranks_agree(ok: bool) -> bool:
    """True only when ``ok`` holds on EVERY rank (host gloo group; no device involvement).

    Used wherever a rank-local outcome (a communicator init, a graph capture) picks between two
    code paths that issue different collectives: all ranks must take the same branch or they
    desynchronise and hang."""
    ctx = context()
    if not ctx.distributed:
        return bool(ok)
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=ctx.host_group)
    return bool(t.item())


def barrier() -> None:
    ctx = context()
    if ctx.distributed:
        dist.barrier(group=ctx.host_group)


# --------------------------------------------------------------- tensor collectives
def all_gather_tensor(t: torch.Tensor) -> torch.Tensor:
    """Concatenate ``t`` from every rank along dim 0 (0-d tensors become ``[W]``)."""
    ctx = context()
    if t.dim() == 0:
        t = t.reshape(1)
    if not ctx.distributed:
        return t
    t = t.contiguous()
    if dist.get_backend() == "gloo":
        parts = [torch.empty_like(t) for _ in range(ctx.world_size)]
        dist.all_gather(parts, t)
        return torch.cat(parts, 0)
    out = torch.empty((ctx.world_size * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t)
    return out


def all_reduce_(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    ctx = context()
    if not ctx.distributed:
        return t
    if op == "mean":
        if dist.get_backend() == "nccl" and t.is_floating_point():
            dist.all_reduce(t, op=dist.ReduceOp.AVG)
        else:
            dist.all_reduce(t)
            t.div_(ctx.world_size)
        return t
    rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
    dist.all_reduce(t, op=rop)
    return t


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if context().distributed:
        dist.broadcast(t, src=src)
    return t
