"""One-shot peer-to-peer all-reduce over xGMI (``native/kernels/p2p.hip``).

For gradient buckets that are latency-bound on RCCL — LeNet's whole gradient is 247 KB — every
rank maps every peer's staging buffer once (HIP IPC handles exchanged over the host gloo group)
and a single kernel reads all W contributions directly over the point-to-point xGMI links,
sums them in rank order (bit-identical on every rank) and writes the average in place.  The
kernel synchronises with its peers through per-block epoch flags in device memory, so it is
stream-ordered and **graph-capturable**: a data-parallel training step becomes one HIP graph
(forward, backward, all-reduce, optimizer) with no host hop between backward and optimizer.

This replaces, for small buckets, the RCCL all-reduce DDP issues at the reference's
``loss.py:119`` backward (SURVEY §2.6 C5, §5 "Tiny models such as LeNet ... one-shot P2P").
Large buckets stay on RCCL, whose ring/direct algorithms are bandwidth-optimal.
"""

from __future__ import annotations

import ctypes
import logging
import os
from typing import Optional

import torch
import torch.distributed as dist

from rocket_amd.ops import _lib

logger = logging.getLogger(__name__)

#: largest total bucket size (fp32 elements) routed through the P2P kernel (16 MB)
MAX_ELEMS = int(os.environ.get("ROCKET_P2P_MAX_ELEMS", str(4 << 20)))


def enabled() -> bool:
    """``ROCKET_P2P``: "1" (default: used with the RCCL backend), "0" (never), "force" (also with a
    gloo tensor group — tests that put several ranks on one GPU, where RCCL cannot run)."""
    return os.environ.get("ROCKET_P2P", "1").lower() not in ("0", "false", "no")


def forced() -> bool:
    return os.environ.get("ROCKET_P2P", "").lower() == "force"


class P2PAllReduce:
    """Per-process context: this rank's IPC-exported stage/flags plus every peer's mapping."""

    def __init__(self, ctx: int, rank: int, world: int, cap: int, device: torch.device):
        self._ctx = ctx
        self.rank, self.world, self.cap, self.device = rank, world, cap, device
        self.launches = 0
        # the kernel's error word lives in host-mapped memory: read it with a plain load, no call
        self._err = ctypes.c_uint.from_address(_lib.kernels().rk_p2p_error_ptr(ctx))
        # fault guard: an identity loss-scaling block (optim_common.h AmpSlot: scale 1, growth and
        # backoff 1) handed to the fused optimizers of the replicated model.  A timed-out launch
        # raises its found flag, so the update that would consume un-reduced gradients is skipped.
        self.fault = torch.tensor([1.0, 1.0, 0.0, 0.0, 1.0, 1.0, float("inf"), 0.0] + [0.0] * 4, device=device)  # kAmpSlots
        self._scaler_state = None
        self._set_skip()

    def _set_skip(self) -> None:
        sc = self._scaler_state
        _lib.check(_lib.kernels().rk_p2p_set_skip(self._ctx, self.fault.data_ptr(),
                                                  sc.data_ptr() if sc is not None else None), "rk_p2p_set_skip")

    def guard_scaler(self, state: Optional[torch.Tensor]) -> None:
        """Also raise the found flag of an fp16 scaler's device state on a timeout (the fused
        optimizer reads that block instead of the fault guard on scaled steps)."""
        self._scaler_state = state
        self._set_skip()

    @classmethod
    def create(cls, cap: int, group=None, device: Optional[torch.device] = None) -> Optional["P2PAllReduce"]:
        """Collective over ``group`` (a host/gloo group): every rank gets a context, or every
        rank gets None (any failure anywhere -> the caller keeps RCCL)."""
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        device = device or torch.device("cuda", torch.cuda.current_device())
        lib = _lib.kernels()
        ctx = ctypes.c_void_p()
        hb = int(lib.rk_p2p_handle_bytes())
        buf = (ctypes.c_char * hb)()
        with torch.cuda.device(device):
            rc = lib.rk_p2p_create(rank, world, int(cap), ctypes.byref(ctx), buf)
        mine = bytes(buf) if rc == 0 else None
        if rc != 0:
            logger.warning(f"p2p all-reduce unavailable on rank {rank}: rk_p2p_create -> hipError {rc}")
        every = [None] * world
        dist.all_gather_object(every, mine, group=group)
        if any(h is None for h in every):
            if rc == 0:
                lib.rk_p2p_destroy(ctx)
            return None
        with torch.cuda.device(device):
            rc = lib.rk_p2p_open(ctx, b"".join(every))
        if rc != 0:
            logger.warning(f"p2p all-reduce unavailable on rank {rank}: rk_p2p_open -> hipError {rc}")
        oks = [None] * world
        dist.all_gather_object(oks, rc == 0, group=group)
        if not all(oks):
            lib.rk_p2p_destroy(ctx)
            return None
        dist.barrier(group=group)  # every mapping exists before any rank launches
        out = cls(ctx.value, rank, world, int(cap), device)
        ok = out._self_test()
        oks = [None] * world
        dist.all_gather_object(oks, ok, group=group)
        if not all(oks):
            if rank == 0:
                logger.warning(f"p2p all-reduce failed its self-test on rank(s) "
                               f"{[r for r, o in enumerate(oks) if not o]}; gradients stay on RCCL")
            # the test launches have completed (or timed out) everywhere: safe to unmap
            dist.barrier(group=group)
            out.close()
            return None
        return out

    def _self_test(self) -> bool:
        """Reduce a rank-dependent pattern once (short peer timeout) and compare with its exact
        sum.  Checks the cross-device IPC mappings and the flag protocol over the real links before
        any gradient depends on them; a failure anywhere makes every rank fall back to RCCL."""
        lib = _lib.kernels()
        n = min(self.cap, 3 * 2048 + 17)  # several blocks and a partial tail block
        lib.rk_p2p_set_skip(self._ctx, None, None)  # a timed-out self-test only reports
        try:
            lib.rk_p2p_set_timeout(self._ctx, 5.0)
            with torch.cuda.device(self.device):
                i = torch.arange(n, device=self.device, dtype=torch.float32)
                x = (i % 97) * (self.rank + 1)  # small integers: the fp32 sum is exact in any order
                self.all_reduce_(x, 1.0)
                torch.cuda.synchronize(self.device)
                want = (i % 97) * (self.world * (self.world + 1) / 2)
                ok = bool(torch.equal(x, want)) and not self._err.value
        except Exception as e:  # pragma: no cover - depends on the platform
            logger.warning(f"p2p self-test raised on rank {self.rank}: {e}")
            ok = False
        finally:
            lib.rk_p2p_set_timeout(self._ctx, 30.0)
            self._set_skip()
        return ok

    def all_reduce_(self, flat: torch.Tensor, scale: float = 1.0) -> None:
        """``flat <- scale * sum_ranks(flat)`` in place on the current stream (graph-capturable)."""
        if flat.dtype != torch.float32 or not flat.is_contiguous() or flat.numel() > self.cap:
            raise ValueError("p2p all-reduce takes a contiguous fp32 buffer within the capacity")
        _lib.check(_lib.kernels().rk_p2p_allreduce(self._ctx, flat.data_ptr(), flat.numel(), float(scale),
                                                   _lib.stream_ptr(flat.device)), "rk_p2p_allreduce")
        self.launches += 1
        self.check()  # a plain load of a host-mapped word: reports a timeout of any earlier launch

    def set_loss_ring(self, ring: torch.Tensor, slot: torch.Tensor, idx: int) -> None:
        """The NEXT launch also does the Loss capsule's ring bookkeeping for element ``idx`` of its
        buffer (the loss side channel): ``ring[slot] = reduced value; slot = (slot + 1) % len(ring);
        element = 0`` (``rk_p2p_set_loss_ring``) — one launch per data-parallel step fewer."""
        _lib.check(_lib.kernels().rk_p2p_set_loss_ring(self._ctx, ring.data_ptr(), slot.data_ptr(), ring.numel(),
                                                       int(idx)), "rk_p2p_set_loss_ring")

    def all_reduce_adam_(self, flat: torch.Tensor, scale: float, plan: tuple, advance: bool = True,
                         zero_grads: bool = True) -> None:
        """``all_reduce_`` whose write-back applies the Adam/AdamW update of the parameters whose
        gradients live in ``flat`` (``plan`` = :meth:`rocket_amd.ops.optim._FusedBase.reduce_plan`);
        ``advance``: this launch advances the optimizer's step counter (its last bucket)."""
        if flat.dtype != torch.float32 or not flat.is_contiguous() or flat.numel() > self.cap:
            raise ValueError("p2p all-reduce takes a contiguous fp32 buffer within the capacity")
        segs, ngroups, hyper, step, counter, amp = plan
        _lib.check(_lib.kernels().rk_p2p_allreduce_adam(
            self._ctx, flat.data_ptr(), flat.numel(), float(scale), segs.data_ptr(), segs.shape[0], hyper, ngroups,
            step, counter, amp, int(zero_grads), int(advance), _lib.stream_ptr(flat.device)), "rk_p2p_allreduce_adam")
        self.launches += 1
        self.check()

    def check(self) -> None:
        """Raise if a launch ever timed out waiting for a peer.  Its timed-out blocks left their
        gradients un-reduced, and raised the fault guard's found flag, so the optimizer launch of
        that same step (same stream / graph) skipped its update; this surfaces the failure on the
        host.  Costs one host load: called on every launch and every replay."""
        if self._ctx and self._err.value:
            raise RuntimeError("p2p all-reduce: a peer did not signal within the timeout (dead or desynchronised rank)")

    def close(self) -> None:
        """Unmap the peers and free the buffers (collective: every rank, when no launch is pending
        anywhere).  Not done implicitly: at interpreter exit the mappings are simply left."""
        if self._ctx:
            self._err = ctypes.c_uint(0)  # the mapped word is freed with the context
            _lib.kernels().rk_p2p_destroy(self._ctx)
            self._ctx = 0


class P2PComm:
    """A complete data-parallel transport on the P2P kernel (no RCCL): every gradient bucket is
    reduced by :meth:`P2PAllReduce.all_reduce_` on a side stream forked off backward when the
    bucket completes, joined before the optimizer — the same stream/event structure as the native
    RCCL reducer (``DataParallel.capture_mode == "overlap"``), fully graph-capturable.

    RCCL needs one device per rank; this transport does not, so it is how the overlapped,
    captured DP step (per-bucket all-reduce branches, in-graph rank-0 buffer broadcast, side-channel
    loss) is rehearsed with several ranks on ONE GPU (``ROCKET_DP_COMM=p2p``,
    ``tests/gpu/test_ddp_graph.py``).  Single node only; bandwidth is not its purpose (each rank
    reads every peer's whole bucket)."""

    native = False  # not RCCL: DataParallel must not route small models to its own P2P path

    def __init__(self, ar: P2PAllReduce):
        self.ar = ar
        self.rank, self.world = ar.rank, ar.world
        self.avg_native = True

    @classmethod
    def create(cls, cap: int, group=None, device: Optional[torch.device] = None) -> "P2PComm":
        ar = P2PAllReduce.create(cap, group=group, device=device)
        if ar is None:
            raise RuntimeError("P2PComm: the P2P all-reduce could not be set up on every rank")
        return cls(ar)

    def all_reduce_avg(self, flat: torch.Tensor):
        self._reduce(flat, 1.0 / self.world)
        return _Issued()

    def _reduce(self, t: torch.Tensor, scale: float) -> None:
        """``t <- scale * sum_ranks(t)`` for any dtype / size: fp32 staging in cap-sized chunks
        (integers and bytes below 2^24 are exact in fp32)."""
        if not t.is_contiguous():
            # reshape would return a copy: reduce a contiguous copy and write it back
            tmp = t.contiguous()
            self._reduce(tmp, scale)
            t.copy_(tmp)
            return
        flat = t.reshape(-1)
        f32 = flat if (flat.dtype == torch.float32 and flat.is_contiguous()) else flat.to(torch.float32)
        for off in range(0, f32.numel(), self.ar.cap):
            self.ar.all_reduce_(f32[off : off + self.ar.cap], scale)
        if f32 is not flat:
            flat.copy_(f32.round() if not flat.dtype.is_floating_point else f32)

    def broadcast(self, t: torch.Tensor, src: int = 0) -> None:
        """Rank ``src``'s values everywhere: the other ranks contribute zeros to a sum (stream-
        ordered, capturable)."""
        with torch.no_grad():
            if self.rank != src:
                t.zero_()
            self._reduce(t, 1.0)

    def make_reducer(self, flats):
        return _P2PReducer(self, flats)


class _Issued:
    def wait(self):
        return None


class _P2PReducer:
    """Per-bucket reduction on a side stream, event fork/join with the compute stream (the
    Python twin of ``native/runtime/comm.cpp``'s reducer)."""

    def __init__(self, comm: P2PComm, flats):
        self.comm = comm
        self.flats = list(flats)
        dev = self.flats[0].device
        self.stream = torch.cuda.Stream(device=dev, priority=-1)
        self.done = [torch.cuda.Event() for _ in self.flats]
        self.pending = set()

    def launch(self, i: int) -> None:
        cur = torch.cuda.current_stream(self.flats[i].device)
        ready = torch.cuda.Event()
        ready.record(cur)
        self.stream.wait_event(ready)
        with torch.cuda.stream(self.stream):
            self.comm.ar.all_reduce_(self.flats[i], 1.0 / self.comm.world)
            self.done[i].record(self.stream)
        self.pending.add(i)

    def join(self) -> None:
        if not self.pending:
            return
        cur = torch.cuda.current_stream(self.flats[0].device)
        for i in sorted(self.pending):
            cur.wait_event(self.done[i])
        self.pending.clear()
