"""Data-parallel replica wrapper with a bucketed, backward-overlapped gradient reducer.

Replaces ``torch.nn.parallel.DistributedDataParallel`` that the reference gets
from ``accelerator.prepare(model)`` (``rocket/core/module.py:106``; SURVEY §2.5
N1/N3/N4, §2.6 C3-C5).

Design for MI355X + RCCL over xGMI (SURVEY §5 "communication design"):

* **flat buckets, gradients as bucket views** – every parameter's ``.grad`` is a
  view into a contiguous bucket, so a bucket is all-reduced in place with one
  RCCL call and no pack/unpack copies; ``zero_grad`` is one fill per bucket;
* **bucket sizing for point-to-point xGMI** – RCCL splits a bucket into W
  shards that travel over the 7 links concurrently; per-link messages below
  ~1 MB are latency-bound, so the default cap is 32 MB (≈4 MB per peer at W=8)
  with a small first bucket (1 MB) so communication starts as soon as the last
  layers' gradients are ready;
* **overlap** – buckets are filled in reverse parameter order (≈ backward
  order); when every parameter of a bucket has reported its gradient, the
  bucket's all-reduce is issued asynchronously (RCCL runs it on its own HIP
  stream, ordered after the producing kernels) while autograd keeps computing
  earlier layers.  The optimizer's stream waits on the work handles — no host
  synchronisation;
* **accumulation aware** – inside ``no_sync()`` nothing is communicated and
  gradients keep accumulating in the bucket views;
* params that received no gradient in the whole accumulation window have their
  slot zeroed before the final bucket is reduced (no stale data is ever averaged
  in); a param unused only in the sync micro-step keeps its accumulated gradient;
* rank-0 parameters and buffers are broadcast once at construction as one flat
  buffer per dtype (N3); module buffers (BatchNorm statistics) are broadcast
  from rank 0 before each synchronised forward (N4, ``broadcast_buffers``) as
  ONE persistent byte buffer: one multi-tensor copy + one collective.

A native RCCL communicator (``rocket_amd.parallel.rccl``) can be plugged in
through ``comm=``; the default uses the ``torch.distributed`` RCCL group, except that when all
buckets together are small (≤ 16 MB fp32, one node) they are reduced by the one-shot xGMI kernel
of :mod:`rocket_amd.parallel.p2p` — stream-ordered and graph-capturable (``capturable``).
"""

from __future__ import annotations

import os

import contextlib
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
from torch import nn

DEFAULT_BUCKET_MB = 32.0
DEFAULT_FIRST_BUCKET_MB = 1.0
SIDE_SLOTS = 16


def _padded(n: int) -> int:
    """Elements a parameter occupies in a flat buffer: rounded up to 4 (16 B of fp32); the pad
    stays zero, so reducing the whole flat buffer is unaffected."""
    return (n + 3) // 4 * 4


class _Bucket:
    __slots__ = ("index", "params", "offsets", "flat", "pending", "work", "ready", "touched", "numel_params")

    def __init__(self, index: int, params: List[nn.Parameter], dtype, device, extra: int = 0):
        self.index = index
        self.params = params
        self.offsets = []
        n = 0
        for p in params:
            self.offsets.append(n)
            n += _padded(p.numel())  # every grad view 16-byte aligned (native kernels store 16 B)
        self.numel_params = n
        self.flat = torch.zeros(n + extra, dtype=dtype, device=device)
        self.pending = len(params)
        self.work = None
        self.ready: set = set()    # params that reported a gradient in this (sync) backward
        self.touched: set = set()  # params that got a gradient anywhere in the accumulation window

    def view(self, i: int) -> torch.Tensor:
        from rocket_amd.parallel.flat_grads import _param_view

        return _param_view(self.flat, self.offsets[i], self.params[i])


class _TorchDistComm:
    """All-reduce through the default ``torch.distributed`` group (RCCL/gloo)."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.avg_native = dist.get_backend(group) == "nccl"

    def all_reduce_avg(self, flat: torch.Tensor):
        if self.avg_native:
            return dist.all_reduce(flat, op=dist.ReduceOp.AVG, group=self.group, async_op=True)
        work = dist.all_reduce(flat, group=self.group, async_op=True)
        return _ScaleAfter(work, flat, 1.0 / self.world)

    def broadcast(self, t: torch.Tensor, src: int = 0):
        dist.broadcast(t, src=src, group=self.group)


class _ScaleAfter:
    def __init__(self, work, flat, scale):
        self.work, self.flat, self.scale = work, flat, scale

    def wait(self):
        self.work.wait()
        self.flat.mul_(self.scale)


class _StreamOrdered:
    """Work handle of a reduction already ordered on the compute stream (P2P kernel / native
    reducer joined before the optimizer): nothing to wait for on the host."""

    def wait(self):
        pass


_ISSUED = _StreamOrdered()


class DataParallel(nn.Module):
    """Replicate ``module`` on every rank and average gradients across ranks."""

    def __init__(
        self,
        module: nn.Module,
        comm=None,
        bucket_cap_mb: float = DEFAULT_BUCKET_MB,
        first_bucket_mb: float = DEFAULT_FIRST_BUCKET_MB,
        broadcast_buffers: bool = True,
    ):
        super().__init__()
        self.module = module
        self.comm = comm or _TorchDistComm()
        self.broadcast_buffers = broadcast_buffers
        self.require_backward_grad_sync = True
        self._rank = getattr(self.comm, "rank", None)
        if self._rank is None:
            self._rank = dist.get_rank(getattr(self.comm, "group", None)) if dist.is_initialized() else 0
        self._sync_module_states()
        self._flat_buffers = self._pack_buffers() if broadcast_buffers else None
        self._build_buckets(bucket_cap_mb, first_bucket_mb)
        self._armed = False
        self._deferred = False
        self._reduces = 0
        self._debug = os.environ.get("ROCKET_DEBUG_SYNC", "0") == "1"
        self._launched: List[int] = []
        self.fused_updates = 0  # captured sync steps whose P2P reduce applied the optimizer update
        self._loss_fold = None  # (bucket, element, ring, slot) of the next inline P2P reduce (fold_loss_ring)
        self.loss_folds = 0  # captured steps whose P2P reduce did the loss-ring bookkeeping
        # small models: one-shot xGMI all-reduce kernel (graph-capturable) instead of RCCL
        self._p2p = self._make_p2p()
        # native transport: per-bucket all-reduce on a side stream, one join before the optimizer
        self._native = None
        # set (on every rank together) when an overlapped capture failed: captured sync steps then
        # use two graphs with the host-issued reduction between them (runtime/graphs.py)
        self.force_split = False
        if self._p2p is None and hasattr(self.comm, "make_reducer"):
            self._native = self.comm.make_reducer([b.flat for b in self.buckets])

    # ----------------------------------------------------------------- setup
    def _flat_broadcast(self, tensors: List[torch.Tensor]) -> None:
        by_dtype: Dict[torch.dtype, List[torch.Tensor]] = {}
        for t in tensors:
            by_dtype.setdefault(t.dtype, []).append(t)
        for ts in by_dtype.values():
            flat = torch.cat([t.detach().reshape(-1) for t in ts])
            self.comm.broadcast(flat, 0)
            off = 0
            with torch.no_grad():
                for t in ts:
                    t.copy_(flat[off : off + t.numel()].view_as(t))
                    off += t.numel()

    def _sync_module_states(self) -> None:
        tensors = [p.data for p in self.module.parameters()] + list(self.module.buffers())
        if tensors:
            self._flat_broadcast(tensors)

    def _pack_buffers(self) -> Optional[torch.Tensor]:
        """Persistent byte buffer for the per-forward rank-0 broadcast of the module buffers
        (BatchNorm running statistics, counters; N4): one collective on it per sync forward,
        with one multi-tensor copy in (rank 0) or out (other ranks) -- not a cat, a broadcast
        and a copy per buffer.  Each buffer keeps its own storage: views of one base would
        share a version counter, and autograd checks the running statistics' versions."""
        bufs, seen = [], set()
        for b in self.module.buffers():
            if b.numel() > 0 and id(b) not in seen:
                seen.add(id(b))
                bufs.append(b)
        if not bufs or len({b.device for b in bufs}) != 1:
            return None
        offs, n = [], 0
        for b in bufs:
            offs.append(n)
            n += (b.numel() * b.element_size() + 15) // 16 * 16  # every view 16-byte aligned
        flat = torch.empty(n, dtype=torch.uint8, device=bufs[0].device)
        self._bufs = bufs
        self._buf_views = [flat[o : o + b.numel() * b.element_size()].view(b.dtype).view(b.shape)
                           for o, b in zip(offs, bufs)]
        return flat

    def _build_buckets(self, cap_mb: float, first_mb: float) -> None:
        params = [p for p in self.module.parameters() if p.requires_grad]
        params = params[::-1]  # backward produces the last layers' grads first
        self.buckets: List[_Bucket] = []
        self._slot: Dict[int, tuple] = {}
        cur: List[nn.Parameter] = []
        cur_bytes = 0
        limit = first_mb * 2**20

        def close():
            nonlocal cur, cur_bytes, limit
            if not cur:
                return
            groups: Dict[tuple, List[nn.Parameter]] = {}
            for p in cur:
                groups.setdefault((p.dtype, p.device), []).append(p)
            for (dtype, device), ps in groups.items():
                b = _Bucket(len(self.buckets), ps, dtype, device)
                self.buckets.append(b)
            cur, cur_bytes, limit = [], 0, cap_mb * 2**20

        for p in params:
            cur.append(p)
            cur_bytes += p.numel() * p.element_size()
            if cur_bytes >= limit:
                close()
        close()
        # side channel: a few fp32 slots behind the last fp32 bucket's gradients, averaged by the
        # same collective (captured steps reduce their loss scalar with the gradients, no extra call)
        self._side = None
        self._side_used = 0
        for bi in range(len(self.buckets) - 1, -1, -1):
            b = self.buckets[bi]
            if b.flat.dtype == torch.float32:
                nb = _Bucket(b.index, b.params, b.flat.dtype, b.flat.device, extra=SIDE_SLOTS)
                self.buckets[bi] = nb
                self._side = nb.flat[nb.numel_params :]
                break
        for b in self.buckets:
            for i, p in enumerate(b.params):
                self._slot[id(p)] = (b, i)
                with torch.no_grad():
                    if p.grad is not None:
                        b.view(i).copy_(p.grad)
                p.grad = b.view(i)
                p._rocket_direct_grad = True  # fused kernels may accumulate into the view directly
                p._rocket_grad_hook = self._on_grad
                p.register_post_accumulate_grad_hook(self._on_grad)
        self.params = [p for b in self.buckets for p in b.params]
        self._ids = {id(p) for p in self.params}

    def _make_p2p(self):
        from rocket_amd.parallel import p2p
        from rocket_amd.runtime import comm as rcomm

        ctx = rcomm.context()
        if ctx.world_size < 2 or not dist.is_initialized():
            return None
        rccl = getattr(self.comm, "native", False) or (isinstance(self.comm, _TorchDistComm) and self.comm.avg_native)
        if (not p2p.enabled() or not (rccl or (isinstance(self.comm, _TorchDistComm) and p2p.forced()))
                or ctx.local_world_size != ctx.world_size or ctx.world_size > 8 or not self.buckets
                or any(b.flat.dtype != torch.float32 or b.flat.device.type != "cuda" for b in self.buckets)
                or sum(b.flat.numel() for b in self.buckets) > p2p.MAX_ELEMS):
            return None
        return p2p.P2PAllReduce.create(max(b.flat.numel() for b in self.buckets), group=ctx.host_group,
                                       device=self.buckets[0].flat.device)

    def check_comm(self) -> None:
        """Surface an asynchronous transport failure (P2P peer timeout) as an exception."""
        if self._p2p is not None:
            self._p2p.check()

    @property
    def capture_mode(self) -> str:
        """How a captured gradient-sync step reduces (``runtime/graphs.py``):

        * ``"overlap"`` — native RCCL reducer: each bucket's all-reduce is launched from the
          gradient hooks *during capture*, forked onto the reducer's side stream and joined before
          the optimizer, so the step is ONE graph whose all-reduce nodes run in parallel branches
          with the rest of backward;
        * ``"inline"`` — P2P one-shot kernel: one reduction between backward and optimizer, in
          the same graph (small models: the whole gradient is one latency-bound bucket);
        * ``"split"`` — torch.distributed group (ProcessGroupNCCL's own streams cannot be
          captured): two graphs with the host-issued bucket all-reduce between them."""
        if self._p2p is not None:
            return "inline"
        if self._native is not None and not self.force_split:
            return "overlap"
        return "split"

    @property
    def capturable(self) -> bool:
        """True when a synchronising step can be captured as ONE graph (P2P or native reducer)."""
        return self.capture_mode != "split"

    # --------------------------------------------------------------- runtime
    @contextlib.contextmanager
    def no_sync(self):
        old = self.require_backward_grad_sync
        self.require_backward_grad_sync = False
        try:
            yield
        finally:
            self.require_backward_grad_sync = old

    def forward(self, *args, **kwargs):
        if torch.is_grad_enabled() and not self._deferred:
            self._arm()
        if self.broadcast_buffers and self.require_backward_grad_sync and not self._deferred:
            self.sync_buffers()
        return self.module(*args, **kwargs)

    def sync_buffers(self) -> None:
        """Broadcast rank-0 module buffers (BatchNorm statistics) to every rank: one collective on
        the persistent flat buffer the buffers are views of."""
        if self._flat_buffers is not None:
            with torch.no_grad():
                if self._rank == 0:
                    torch._foreach_copy_(self._buf_views, self._bufs)
                self.comm.broadcast(self._flat_buffers, 0)
                if self._rank != 0:
                    torch._foreach_copy_(self._bufs, self._buf_views)
            return
        bufs = list(self.module.buffers())
        if bufs:
            self._flat_broadcast(bufs)

    # ----------------------------------------------------- captured (graph) steps
    @contextlib.contextmanager
    def deferred(self):
        """Record gradients into the buckets without communicating (HIP-graph capture).

        The captured region contains no collective; the step executor calls
        :meth:`reduce_now` on the host between the backward graph and the
        optimizer graph, so RCCL never runs inside a graph.
        """
        old = self._deferred
        self._deferred = True
        self._armed = False
        try:
            yield
        finally:
            self._deferred = old

    def fold_loss_ring(self, acc: torch.Tensor, ring: torch.Tensor, slot: torch.Tensor) -> bool:
        """Inline P2P steps: the next :meth:`reduce_now` moves the reduced loss accumulator ``acc`` (a
        side-slot view of a bucket) into ``ring[slot]``, advances ``slot`` and clears ``acc`` inside
        the all-reduce launch (``rk_p2p_set_loss_ring``).  True when taken: the caller then skips its
        own bookkeeping launch."""
        if self._p2p is None or self.capture_mode != "inline" or acc.numel() != 1:
            return False
        p = acc.data_ptr()
        for i, b in enumerate(self.buckets):
            f = b.flat
            lo = f.data_ptr()
            if lo <= p < lo + f.numel() * f.element_size():
                self._loss_fold = (i, (p - lo) // f.element_size(), ring, slot)
                return True
        return False

    def _fold_for(self, i: int) -> None:
        if self._loss_fold is not None and self._loss_fold[0] == i:
            _, idx, ring, slot = self._loss_fold
            self._p2p.set_loss_ring(ring, slot, idx)
            self.loss_folds += 1

    def reduce_now(self) -> None:
        """Average every bucket (incl. the side channel) across ranks; stream-ordered, no host wait."""
        self._launched = []
        try:
            if self._p2p is not None and self._reduce_with_update():
                return
            works = []
            for i, b in enumerate(self.buckets):
                if self._p2p is not None:
                    self._fold_for(i)
                works.append(self._launch(b))
        finally:
            self._loss_fold = None
        if self._native is not None:
            self._native.join()
        for w in works:
            if w is not None:
                w.wait()

    def _reduce_with_update(self) -> bool:
        """P2P transport, captured sync step: when ONE fused Adam-family optimizer owns exactly the
        bucketed parameters and has armed its reduce epilogue (``Optimizer.graph_prepare``: sync
        step, W > 1, no AMP scaler), each bucket's all-reduce applies the update in its write-back
        and the optimizer's own launch is skipped (``epilogue_done``): the data-parallel LeNet step
        is then backward -> reduce+update, one launch fewer than reduce -> update."""
        fused = self.prepare_reduce()
        if fused is None:
            return False
        opt, plans = fused
        last = len(self.buckets) - 1
        for i, (b, plan) in enumerate(zip(self.buckets, plans)):
            if self._debug:
                self._debug_check_launch(b)
            self._fold_for(i)
            self._p2p.all_reduce_adam_(b.flat, 1.0 / self.comm.world, plan, advance=i == last)
        # (the arming stays: one prepare can precede several captures — the loader ring's slots are
        # captured together — and every one of them takes this path; graph_host disarms)
        opt.epilogue_done = True
        self.fused_updates += 1
        return True

    def prepare_reduce(self):
        """``(optimizer, per-bucket plans)`` of the reduce-with-update path, or None.  The plans
        (device segment tables) are built on first use and cached by the optimizer: the graph
        executor calls this before capturing a step, so no table is uploaded inside a capture."""
        opt = None
        for b in self.buckets:
            for p in b.params:
                o = getattr(p, "_rocket_optimizer", None)
                if o is None or not getattr(o, "reduce_epilogue_armed", False) or (opt is not None and o is not opt):
                    return None
                opt = o
        if opt is None or {id(p) for _, p in opt._active()} != {id(p) for b in self.buckets for p in b.params}:
            return None
        plans = [opt.reduce_plan(b.flat, b.params) for b in self.buckets]
        return None if any(pl is None for pl in plans) else (opt, plans)

    def side_slot(self, n: int = 1) -> torch.Tensor:
        """``n`` fp32 slots that are averaged together with the gradients on every sync step."""
        if self._side is None or self._side_used + n > self._side.numel():
            return None
        v = self._side[self._side_used : self._side_used + n]
        self._side_used += n
        return v

    def _arm(self) -> None:
        for b in self.buckets:
            b.pending = len(b.params)
            b.ready.clear()
            b.work = None
        self._armed = True
        self._finalize_queued = False
        self._launched = []
        if self._debug and torch.cuda.is_available() and self.buckets and self.buckets[0].flat.is_cuda:
            self._stream0 = torch.cuda.current_stream(self.buckets[0].flat.device)

    def _debug_check_launch(self, b: _Bucket) -> None:
        """ROCKET_DEBUG_SYNC=1 stream-ordering / bucket assertions: a bucket is
        reduced once per sync step, only after every gradient in it was written into its flat
        view, on the stream the backward ran on (the side-stream reducer forks from it)."""
        if b.index in self._launched:
            raise RuntimeError(f"DDP debug: bucket {b.index} reduced twice in one step")
        for i, p in enumerate(b.params):
            if p.grad is not None and p.grad.data_ptr() != b.view(i).data_ptr():
                raise RuntimeError(f"DDP debug: bucket {b.index} param {i} gradient is not its flat view")
        if self._armed and b.pending != 0:
            raise RuntimeError(f"DDP debug: bucket {b.index} launched with {b.pending} gradients outstanding")
        s0 = getattr(self, "_stream0", None)
        if s0 is not None and torch.cuda.current_stream(b.flat.device) != s0:
            raise RuntimeError(f"DDP debug: bucket {b.index} launched on a different stream than backward")
        self._launched.append(b.index)

    def _on_grad(self, p: nn.Parameter) -> None:
        b, i = self._slot[id(p)]
        view = b.view(i)
        if p.grad is not view and p.grad.data_ptr() != view.data_ptr():
            with torch.no_grad():
                view.copy_(p.grad)
            p.grad = view
        b.touched.add(i)
        if self._deferred or not self._armed or i in b.ready:
            return
        if not self._finalize_queued:
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
            self._finalize_queued = True
        b.ready.add(i)
        b.pending -= 1
        if b.pending == 0 and self.require_backward_grad_sync:
            b.work = self._launch(b)

    def _finalize(self) -> None:
        """Runs at the end of backward: reduce buckets with params that got no grad."""
        if not self._armed:
            return
        self._armed = False
        if not self.require_backward_grad_sync:
            return
        for b in self.buckets:
            if b.work is None:
                with torch.no_grad():
                    for i in range(len(b.params)):
                        # never-touched slots are zeroed (no stale data is averaged in); a param
                        # unused in THIS micro-step but with gradient accumulated in earlier no_sync
                        # micro-steps keeps it, as torch DDP all-reduces the defined local grad
                        if i not in b.ready and i not in b.touched:
                            b.view(i).zero_()
                            b.params[i].grad = b.view(i)
                b.work = self._launch(b)
        if self._debug and sorted(self._launched) != list(range(len(self.buckets))):
            raise RuntimeError(f"DDP debug: buckets reduced this step {self._launched} != all {len(self.buckets)}")
        for b in self.buckets:
            b.touched.clear()  # the accumulation window ends with this reduction
        if self._native is not None:
            self._native.join()
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                b.work = None

    def _launch(self, b: _Bucket):
        if self._debug:
            self._debug_check_launch(b)
        if self._p2p is not None:
            self._p2p.all_reduce_(b.flat, 1.0 / self.comm.world)
            return _ISSUED
        if self._native is not None:
            self._native.launch(b.index)
            return _ISSUED
        return self.comm.all_reduce_avg(b.flat)

    def owns(self, p) -> bool:
        return id(p) in self._ids

    def zero_(self) -> None:
        for b in self.buckets:
            b.flat.zero_()
            b.touched.clear()
            for i, p in enumerate(b.params):
                if p.grad is None or p.grad.data_ptr() != b.view(i).data_ptr():
                    p.grad = b.view(i)

    def zero_grad(self, set_to_none: bool = False) -> None:
        self.zero_()

    # ---------------------------------------------------------------- access
    def state_dict(self, *args, **kwargs):
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, *args, **kwargs):
        return self.module.load_state_dict(*args, **kwargs)

    @property
    def bucket_sizes(self) -> List[int]:
        return [b.flat.numel() for b in self.buckets]


def unwrap(model: nn.Module) -> nn.Module:
    while isinstance(model, DataParallel):
        model = model.module
    return model
