"""HIP-graph capture of the training micro-step (MI355X: graphs instead of a tracing compiler).

A LeNet-sized step is launch-bound: ~10 kernels of a few µs each, separated by
host launch latency (~5-10 µs per eager launch).  :class:`StepGraphs` captures
the complete device side of a ``Module`` capsule's micro-step —

    forward → objective → backward (incl. the fused kernels' direct gradient
    accumulation) → [gradient all-reduce] → optimizer update + gradient clear

— into HIP graphs per variant (gradient-sync step vs. accumulation step, keyed
by input signature) and replays them every iteration, while every host-side
duty of the capsules still runs each iteration: loss/lr reporting to the
tracker and progress bar, scheduler stepping, GA bookkeeping.

Data parallel (W>1), by the replica's ``capture_mode`` (``parallel/ddp.py``):

* ``overlap`` (default on GPUs: the native RCCL communicator) — the whole sync
  step is ONE graph.  During capture every bucket's ``ncclAllReduce`` is
  launched from the gradient hooks the moment the bucket is complete, forked
  onto the reducer's high-priority side stream with an event and joined back
  before the optimizer; the instantiated graph therefore holds each bucket's
  all-reduce as a parallel branch that runs while the rest of backward
  continues (replayed with hipGraphLaunch, which keeps the branches parallel).
  The rank-0 BatchNorm buffer broadcast is captured in the forward as well;
* ``inline`` (small models: the one-shot P2P xGMI kernel) — one graph with the
  reduction kernel between backward and optimizer;
* ``split`` (torch.distributed fallback) — two graphs, ``A`` (forward/backward,
  gradients land in the reducer's flat buckets) and ``B`` (optimizer), with the
  bucket all-reduce issued from the host between them.

The loss scalar rides in the reducer's side channel, so it is averaged by the
same collective as the gradients.

Protocol for children of a captured ``Module`` (built-ins implement it):

* ``graph_prepare(attrs)``  – host work before each replay (e.g. the fused
  optimizer uploads changed hyper-parameters);
* ``graph_device(attrs)``   – device work of phase A (captured);
* ``graph_device_synced(attrs)`` – optional device work of phase B, after the
  gradient reduction (captured);
* ``graph_host(attrs)``     – host bookkeeping after every replay;
* ``graph_supported()``     – optional veto; ``graph_token()`` – optional value
  whose change invalidates captured graphs (e.g. re-allocated optimizer tables).

A child without ``graph_device`` makes the module fall back to eager
execution, as do unseen input signatures until warmed up, and CPU tensors.
The first ``warmup`` iterations of each (sync, signature) variant run eagerly,
which also primes lazily created state (optimizer moments, workspaces).

Replay: each captured graph is walked once into a native *launch list*
(``native/runtime/launchlist.cpp``) and re-issued as plain stream launches —
hipGraphLaunch costs a fixed ~5-8 µs of GPU idle time per launch on MI355X,
back-to-back dispatches ~1-2 µs; the graph object stays alive because the list
points into its node argument arrays.  A graph with a node type the list does
not support (or ``ROCKET_LAUNCH_LIST=0``) is replayed with ``graph.replay()``.

Inputs: tensors flagged ``_rocket_persistent`` (the device loader's ring
buffers) are captured in place and get one graph per buffer set — no copy per
step; the variants of every slot of a loader ring are captured together, on
the first capture, so no capture lands in a later (timed) iteration.  Any
other input is copied into a static buffer before replay.
"""

from __future__ import annotations

import collections
import operator
import os
from typing import Any, Dict, List, Optional, Tuple

import torch

from rocket_amd.core.attributes import Attributes
from rocket_amd.ops import _lib
from rocket_amd.utils.logging import get_logger

logger = get_logger(__name__)

MAX_VARIANTS = 32


def _use_launch_lists() -> bool:
    return os.environ.get("ROCKET_LAUNCH_LIST", "1") != "0"


_VERSION = operator.attrgetter("_version")


class _Part:
    """One captured graph and, when every node is supported, its launch list (preferred replay)."""

    __slots__ = ("graph", "ll")

    def __init__(self, graph):
        self.graph = graph
        self.ll = None

    def finish(self) -> Optional[str]:
        if not _use_launch_lists():
            return "disabled (ROCKET_LAUNCH_LIST=0)"
        from rocket_amd.runtime.native import LaunchList

        try:
            self.ll, why = LaunchList.build(self.graph)
        except Exception as e:  # runtime library missing: graph replay still works
            self.ll, why = None, f"{type(e).__name__}: {e}"
        return why

    def run(self, stream: int) -> None:
        if self.ll is not None:
            self.ll.launch(stream)
        else:
            self.graph.replay()


def _signature(batch) -> Tuple:
    if isinstance(batch, torch.Tensor):
        return (tuple(batch.shape), batch.dtype, batch.device.type)
    if isinstance(batch, (list, tuple)):
        return (type(batch).__name__,) + tuple(_signature(b) for b in batch)
    if isinstance(batch, dict):
        return ("dict",) + tuple((k, _signature(v)) for k, v in sorted(batch.items(), key=lambda kv: str(kv[0])))
    return (type(batch).__name__, batch if isinstance(batch, (int, float, str, bool, type(None))) else id(batch))


def _tensors(batch) -> List[torch.Tensor]:
    if isinstance(batch, torch.Tensor):
        return [batch]
    if isinstance(batch, (list, tuple)):
        return [t for b in batch for t in _tensors(b)]
    if isinstance(batch, dict):
        return [t for k in sorted(batch, key=str) for t in _tensors(batch[k])]
    return []


def _rebuild(batch, it):
    if isinstance(batch, torch.Tensor):
        return next(it)
    if isinstance(batch, tuple) and hasattr(batch, "_fields"):
        return type(batch)(*[_rebuild(b, it) for b in batch])
    if isinstance(batch, (list, tuple)):
        return type(batch)(_rebuild(b, it) for b in batch)
    if isinstance(batch, dict):
        keys = sorted(batch, key=str)
        vals = {k: _rebuild(batch[k], it) for k in keys}
        return type(batch)((k, vals[k]) for k in batch)
    return batch


class _Captured:
    __slots__ = ("graphs", "static_in", "persistent", "out", "sync", "host_sync_buffers", "rows_in_graph")

    def __init__(self):
        self.graphs: list = []   # [_Part A] or [A, B] (B after the host-side gradient reduction)
        self.static_in = None
        self.persistent = None   # per input tensor: captured in place (no copy at replay)
        self.out = None
        self.sync = False
        self.host_sync_buffers = False
        self.rows_in_graph = False  # the step gathers its deferred loader batch itself (PendingRows)


class StepGraphs:
    def __init__(self, module_capsule, warmup: int = 3):
        self.mod = module_capsule
        self.warmup = max(1, int(warmup))
        self.variants: Dict[Any, _Captured] = {}
        self.parts = 0  # most graphs one captured step was split into (1 = whole step in one graph)
        self.seen = collections.Counter()
        self.pool = None
        self.disabled_reason = None
        self.replays = 0
        self.captures = 0
        self.sync_captures = 0  # captures of gradient-sync steps
        self._token = None
        self._checked = False
        self._rep = False  # resolved lazily (the module is wrapped during setup)
        self._preps = None  # bound graph_prepare / graph_host / graph_token methods of the children
        self._hosts = None
        self._toks = None
        self._params = None  # parameter list for the version token (fixed once graphs exist)
        self._dev = None
        self._bcache: dict = {}  # id(batch) -> (batch, tensors, signature, persistent key) of ring slots
        self._bcache_ring = None  # id of the ring (mark_ring sets) those entries belong to
        self.launch_lists = 0  # captured parts replayed as native launch lists
        self.launch_list_reason = None  # why a part kept hipGraphLaunch replay (first such part)

    def release(self) -> None:
        self.variants.clear()
        self._bcache.clear()
        self.pool = None
        self.disabled_reason = self.disabled_reason or "released"

    # ------------------------------------------------------------------ checks
    def _replica(self):
        if self._rep is False:
            from rocket_amd.parallel.ddp import DataParallel

            rep = self.mod._module
            self._rep = rep if isinstance(rep, DataParallel) else None
        return self._rep

    def _children_ok(self) -> bool:
        for c in self.mod._capsules:
            if not hasattr(c, "graph_device"):
                self.disabled_reason = f"child {type(c).__name__} has no graph protocol"
                return False
            ok = getattr(c, "graph_supported", None)
            if ok is not None and not ok():
                self.disabled_reason = f"child {type(c).__name__} is not graph-safe"
                return False
        for p in self.mod._module.parameters():
            if p.requires_grad and not getattr(p, "_rocket_direct_grad", False):
                self.disabled_reason = "parameters lack persistent gradient buffers"
                return False
        if self.mod._accelerator.num_processes > 1 and self._replica() is None:
            self.disabled_reason = "multi-process run without the rocket data-parallel reducer"
            return False
        return True

    def side_slot(self, n: int = 1) -> torch.Tensor:
        """``n`` static fp32 device slots; under data parallelism they are averaged across ranks
        by the same collective as the gradients on every sync step."""
        rep = self._replica()
        v = rep.side_slot(n) if rep is not None else None
        if v is None:
            if rep is not None:
                raise RuntimeError("data-parallel side channel exhausted")
            v = torch.zeros(n, device=self.mod._accelerator.device)
        return v

    def _tokens(self):
        # parameter versions: weights rewritten outside the captured step (checkpoint load, manual
        # edits) invalidate the graphs — captured kernels may depend on derived state of them
        # (e.g. the fused LeNet's optimizer-maintained bf16 fragment table)
        if self._params is None:
            self._params = list(self.mod._module.parameters())
        # (map + attrgetter: ~1 us less per step than a generator over the parameters)
        return tuple([t() for t in self._toks]) + (sum(map(_VERSION, self._params)),)

    def _predict_sync(self) -> bool:
        engine = self.mod._accelerator
        if engine.gradient_state.end_of_dataloader:
            return True
        return (engine.step + 1) % engine.gradient_accumulation_steps == 0

    # ------------------------------------------------------------------ launch
    def launch(self, attrs: Attributes) -> bool:
        """Run the micro-step through a graph; False -> the caller runs it eagerly."""
        if self.disabled_reason is not None:
            return False
        batch = attrs.get("batch")
        ent = self._bcache.get(id(batch))
        if ent is not None and ent[0] is batch:
            # a loader ring slot seen before (the same tuple of persistent buffers: fixed shapes)
            _, tens, bsig, pkey = ent
        else:
            tens = _tensors(batch)
            if not tens or any(t.device.type != "cuda" for t in tens):
                return False
            bsig = _signature(batch)
            pkey = tuple(t.data_ptr() if getattr(t, "_rocket_persistent", False) else 0 for t in tens)
            if type(batch) is tuple and all(pkey):
                # entries pin their ring's buffers: a batch from another ring (a recreated loader, a
                # resumed with_skip loader, another batch size) drops the old ring's entries
                ring = getattr(tens[0], "_rocket_ring", None)
                rid = id(ring[0]) if ring is not None else None
                if rid != self._bcache_ring or len(self._bcache) >= 64:
                    self._bcache.clear()
                    self._bcache_ring = rid
                self._bcache[id(batch)] = (batch, tens, bsig, pkey)
        sync = self._predict_sync()
        sig = (sync, bsig)
        key = (sig, pkey)
        v = self.variants.get(key)
        if v is None:
            self.seen[sig] += 1
            if self.seen[sig] <= self.warmup:
                return False  # eager warm-up (primes optimizer state / workspaces)
            if not self._checked:
                self._checked = True
                if not self._children_ok():
                    logger.info(f"graph capture disabled: {self.disabled_reason}")
                    return False
                for c in self.mod._capsules:
                    bind = getattr(c, "graph_bind", None)
                    if bind is not None:
                        bind(self)
                caps = self.mod._capsules
                self._preps = [c.graph_prepare for c in caps if hasattr(c, "graph_prepare")]
                self._hosts = [c.graph_host for c in caps]
                self._toks = [c.graph_token for c in caps if hasattr(c, "graph_token")]
            if len(self.variants) >= MAX_VARIANTS:
                return False
            self.mod._accelerator._do_sync()
            self._prepare(attrs)
            self._check_tokens()
            self._capture_all(sig, key, attrs, tens)
            return True
        self.mod._accelerator._do_sync()
        self._prepare(attrs)
        if self._check_tokens():  # tables re-allocated: every graph is stale, capture again
            self._capture_all(sig, key, attrs, tens)
            return True
        self._replay(v, attrs, tens)
        return True

    @staticmethod
    def _ring_peers(tens: List[torch.Tensor]) -> List[List[torch.Tensor]]:
        """Input lists of the OTHER slots of the loader ring the persistent inputs come from.

        A captured graph reads persistent loader buffers in place, so every ring slot is its own
        variant.  Capturing them all when the first one is captured keeps every capture inside
        the warm-up (one slot per iteration would put RING-1 captures into the first timed
        iterations).  Empty when the inputs are not (all) from one ring slot."""
        ring = slot = None
        for t in tens:
            tag = getattr(t, "_rocket_ring", None)
            if tag is None:
                if getattr(t, "_rocket_persistent", False):
                    return []
                continue
            sets, k, j = tag
            if ring is None:
                ring, slot = sets, k
            elif sets is not ring or k != slot or sets[k][j] is not t:
                return []
        if ring is None:
            return []
        out = []
        for k in range(len(ring)):
            if k == slot:
                continue
            alt = []
            for t in tens:
                tag = getattr(t, "_rocket_ring", None)
                alt.append(ring[k][tag[2]] if tag is not None else t)
            out.append(alt)
        return out

    def _capture_all(self, sig, key, attrs: Attributes, tens: List[torch.Tensor]) -> None:
        for alt in self._ring_peers(tens):
            akey = (sig, tuple(t.data_ptr() if getattr(t, "_rocket_persistent", False) else 0 for t in alt))
            if akey not in self.variants and len(self.variants) < MAX_VARIANTS - 1:
                self.variants[akey] = self._capture(attrs, alt, run=False)
        self.variants[key] = self._capture(attrs, tens)

    def _prepare(self, attrs: Attributes) -> None:
        for prep in self._preps:
            prep(attrs)

    def _check_tokens(self) -> bool:
        tok = self._tokens()
        if self._token is None:
            self._token = tok
            return False
        if tok != self._token:
            self._token = tok
            self.variants.clear()
            return True
        return False

    # ----------------------------------------------------------------- capture
    def _phase_a(self, attrs: Attributes, overlap: bool = False) -> None:
        mod = self.mod
        engine = mod._accelerator
        rep = self._replica()
        with engine.autocast():
            with engine.no_sync(mod._module) if not engine.sync_gradients else _null():
                # overlap: the gradient hooks launch every bucket's all-reduce during capture
                with rep.deferred() if (rep is not None and not overlap) else _null():
                    attrs.batch = mod._module(attrs.batch)
                    for c in mod._capsules:
                        c.graph_device(attrs)

    def _phase_b(self, attrs: Attributes) -> None:
        for c in self.mod._capsules:
            fn = getattr(c, "graph_device_synced", None)
            if fn is not None:
                fn(attrs)

    @staticmethod
    def _bind_pending(attrs: Attributes, tens: List[torch.Tensor], run: bool):
        """The deferred-batch record the captured step sees: this iteration's own (``run``), or the
        same pending batch rebound to the ring slot of a variant captured ahead (``tens`` = that
        slot's buffers), temporarily attached to them.  Returns (record, [(buffer, old attr)])."""
        from rocket_amd.runtime.data import pending_rows

        p = pending_rows(attrs.batch)
        if p is None or run:
            return p, []
        tag = next((getattr(t, "_rocket_ring", None) for t in tens if getattr(t, "_rocket_ring", None)), None)
        if tag is None:
            return None, []
        bufs = tag[0][tag[1]]
        q = p.rebind(bufs)
        restore = [(b, getattr(b, "_rocket_pending", None)) for b in bufs]
        for b in bufs:
            b._rocket_pending = q
        return q, restore

    def _capture(self, attrs: Attributes, tens: List[torch.Tensor], run: bool = True) -> _Captured:
        """Capture the micro-step for inputs ``tens``; ``run``: also replay it for this iteration."""
        pend, restore = self._bind_pending(attrs, tens, run)
        rep = self._replica()
        engine = self.mod._accelerator
        # an overlapped step captures RCCL calls: a capture error may be rank-local, so the ranks
        # agree on the outcome BEFORE anything runs, and all drop to split mode together
        agree = (rep is not None and engine.sync_gradients and rep.capture_mode == "overlap"
                 and engine.num_processes > 1)
        side = self._side_effects(pend) if agree else None
        try:
            err = None
            try:
                v = self._capture_inner(attrs, tens, pend)
            except Exception as e:
                if not agree:
                    raise
                err, v = e, None
            if agree:
                from rocket_amd.runtime import comm as _comm

                if not _comm.all_ranks_agree(err is None):
                    logger.warning(f"overlapped capture failed on some rank ({err or 'peer failed'}); "
                                   "every rank captures sync steps in split mode")
                    rep.force_split = True
                    torch.cuda.synchronize()
                    # the discarded capture already claimed the pending batch and set the fused
                    # optimizers' per-step flags: undo that, or the retried graph would skip the
                    # batch gather and the cursor advance on every replay
                    self._restore_side_effects(pend, side)
                    err2 = None
                    try:
                        v = self._capture_inner(attrs, tens, pend)
                    except Exception as e:
                        err2, v = e, None
                    if not _comm.all_ranks_agree(err2 is None):
                        raise RuntimeError(f"split-mode graph capture failed on some rank ({err2 or 'peer failed'})") \
                            from err2
        finally:
            for b, old in restore:
                b._rocket_pending = old
        if run:
            # the captured work has not run yet: replay it for this iteration
            self._run(v, rep if len(v.graphs) > 1 else None)
            attrs.batch = v.out
            self._host(attrs)
        return v

    _OPT_FLAGS = ("amp_checked", "epilogue_done")

    def _side_effects(self, pend):
        """Host-side state a capture mutates (pending batch, fused-optimizer step flags, counters)."""
        opts = [getattr(o, "optimizer", o) for o in getattr(self.mod._accelerator, "_optimizers", [])]
        flags = [(o, {f: getattr(o, f) for f in self._OPT_FLAGS if hasattr(o, f)}) for o in opts]
        return ((pend.done, pend.advanced) if pend is not None else None, flags, self.captures, self.parts,
                self.launch_lists, self.sync_captures)

    def _restore_side_effects(self, pend, side) -> None:
        pstate, flags, self.captures, self.parts, self.launch_lists, self.sync_captures = side
        if pend is not None:
            pend.done, pend.advanced = pstate
        for o, vals in flags:
            for f, val in vals.items():
                setattr(o, f, val)

    def _capture_inner(self, attrs: Attributes, tens: List[torch.Tensor], pend) -> _Captured:
        engine = self.mod._accelerator
        v = _Captured()
        v.sync = engine.sync_gradients
        v.persistent = [bool(getattr(t, "_rocket_persistent", False)) for t in tens]
        v.static_in = [t if keep else t.detach().clone() for t, keep in zip(tens, v.persistent)]
        rep = self._replica()
        mode = rep.capture_mode if (v.sync and rep is not None) else None
        inline = mode == "inline"    # P2P kernel between backward and optimizer, same graph
        overlap = mode == "overlap"  # bucket all-reduces forked off backward, same graph
        split = mode == "split"      # host-issued all-reduce between two graphs
        v.host_sync_buffers = v.sync and rep is not None and rep.broadcast_buffers and not overlap
        if v.host_sync_buffers:
            rep.sync_buffers()
        if rep is not None and getattr(rep, "_loss_fold", None) is not None:
            rep._loss_fold = None  # a fold registered by an abandoned capture
        if inline:
            rep.prepare_reduce()  # device tables of a reduce-with-update step: uploaded before capture
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        cap = Attributes(attrs)
        cap.batch = _rebuild(attrs.batch, iter(v.static_in))
        cap.capturing = True
        cap.graph_split = v.sync and rep is not None  # a cross-rank reduce separates device / device_synced
        # inline P2P step: the loss capsule may hand its ring bookkeeping to the reduce launch
        cap.fold_loss = rep.fold_loss_ring if (inline and hasattr(rep, "fold_loss_ring")) else None
        torch.cuda.synchronize()
        ga = torch.cuda.CUDAGraph(keep_graph=True)
        # thread_local: the RCCL watchdog thread keeps polling its events while we capture
        with torch.cuda.graph(ga, pool=self.pool, capture_error_mode="thread_local"):
            self._phase_a(cap, overlap)
            if inline:
                rep.reduce_now()
            if not split:
                self._phase_b(cap)
        v.graphs.append(_Part(ga))
        if split:
            gb = torch.cuda.CUDAGraph(keep_graph=True)
            with torch.cuda.graph(gb, pool=self.pool, capture_error_mode="thread_local"):
                self._phase_b(cap)
            v.graphs.append(_Part(gb))
        for part in v.graphs:
            # a graph with parallel branches (the overlapped all-reduce) keeps hipGraphLaunch:
            # a launch list would serialise the branches onto one stream
            why = part.finish() if not overlap else "parallel branches (overlapped all-reduce)"
            if part.ll is not None:
                self.launch_lists += 1
            elif self.launch_list_reason is None:
                self.launch_list_reason = why
                logger.info(f"graph replay (no launch list): {why}")
        if self._dev is None:
            self._dev = engine.device
        v.out = cap.batch
        # the captured step gathered its deferred batch (claimed by the model's kernels or gathered
        # by a captured cursor-mode launch): every replay gathers the batch of its iteration
        v.rows_in_graph = pend is not None and pend.done
        self.captures += 1
        self.sync_captures += int(v.sync)
        self.parts = max(self.parts, len(v.graphs))
        logger.info(f"captured HIP graph(s) for sync={v.sync} ({len(v.graphs)} part(s), mode={mode})")
        return v

    # ------------------------------------------------------------------ replay
    def _run(self, v: _Captured, rep) -> None:
        stream = _lib.stream_ptr(self._dev)
        v.graphs[0].run(stream)
        if len(v.graphs) > 1:
            rep.reduce_now()  # host-issued RCCL between the two graphs
            v.graphs[1].run(stream)
        self.replays += 1

    def _host(self, attrs: Attributes) -> None:
        for host in self._hosts:
            host(attrs)

    def _replay(self, v: _Captured, attrs: Attributes, tens: List[torch.Tensor]) -> None:
        from rocket_amd.runtime.data import pending_rows

        pend = pending_rows(attrs.get("batch"))
        if pend is not None:
            if v.rows_in_graph:
                pend.done = pend.advanced = True  # the replay below gathers it and advances the cursor
            else:
                pend.materialize()
        for dst, src, keep in zip(v.static_in, tens, v.persistent):
            if not keep:
                dst.copy_(src, non_blocking=True)
        rep = self._replica() if v.sync else None
        if rep is not None and v.host_sync_buffers:
            rep.sync_buffers()  # (an overlapped step broadcasts inside its graph)
        if rep is not None:
            rep.check_comm()  # P2P peer timeouts surface at the next step (one host load)
        self._run(v, rep if len(v.graphs) > 1 else None)
        attrs["batch"] = v.out
        self._host(attrs)


class _null:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False
