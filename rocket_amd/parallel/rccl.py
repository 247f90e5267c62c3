"""Native RCCL communicator for the data-parallel reducer (``native/runtime/comm.cpp``).

``RcclComm`` bootstraps an RCCL communicator directly (ncclUniqueId from rank 0 over the host
gloo/TCP group, then ``ncclCommInitRank``) and exposes stream-ordered collectives on the
caller's current HIP stream — graph-capturable, no ProcessGroupNCCL bookkeeping per call.
``DataParallel(comm=RcclComm(...))`` additionally uses the native bucket reducer: every
complete bucket is all-reduced on a dedicated high-priority HIP stream fenced by events, and
the compute stream waits for all buckets once at the end of backward.

This is the engine's default data-parallel transport on GPUs (``Engine(comm="torch")`` or
``ROCKET_NATIVE_COMM=0`` selects torch.distributed's RCCL process group instead).  Creation is
agreed over the host group: if any rank fails, every rank falls back to the torch group together
(``runtime/engine.py`` ``_dp_comm``); a failed overlapped capture likewise drops every rank to the
two-graph ``split`` mode (``runtime/graphs.py``).
"""

from __future__ import annotations

import ctypes

import torch

from rocket_amd.runtime import comm as _comm
from rocket_amd.runtime.native import check, runtime

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int64: 3, torch.int32: 4, torch.uint8: 5}
SUM, AVG, MAX, MIN = 0, 1, 2, 3


class _Done:
    def wait(self):
        return None


class RcclComm:
    graph_safe = True
    native = True

    def __init__(self, device: torch.device | None = None):
        self.rt = runtime()
        ctx = _comm.context()
        self.world, self.rank = ctx.world_size, ctx.rank
        self.device = device or ctx.device
        uid = None
        if self.rank == 0:
            try:
                buf = ctypes.create_string_buffer(self.rt.rkr_unique_id_bytes())
                check(self.rt.rkr_unique_id(buf), "ncclGetUniqueId")
                uid = buf.raw
            except Exception:
                uid = None  # still broadcast: the peers must not wait for an id that never comes
        uid = _comm.broadcast_object(uid, src=0)
        # every rank enters ncclCommInitRank (a blocking collective bootstrap) or none does
        if not _comm.all_ranks_agree(uid is not None):
            raise RuntimeError("ncclGetUniqueId failed on rank 0")
        h = ctypes.c_void_p()
        idbuf = ctypes.create_string_buffer(uid, len(uid))
        check(self.rt.rkr_comm_init(ctypes.byref(h), self.world, self.rank, idbuf, self.device.index or 0),
              "ncclCommInitRank")
        self.h = h
        self.avg_native = True

    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def all_reduce(self, t: torch.Tensor, op: int = SUM) -> torch.Tensor:
        check(self.rt.rkr_all_reduce(self.h, t.data_ptr(), t.numel(), _DT[t.dtype], op, self._stream()),
              "rkr_all_reduce")
        return t

    def all_reduce_avg(self, flat: torch.Tensor):
        self.all_reduce(flat, AVG)
        return _Done()

    def broadcast(self, t: torch.Tensor, src: int = 0) -> None:
        check(self.rt.rkr_broadcast(self.h, t.data_ptr(), t.numel(), _DT[t.dtype], src, self._stream()),
              "rkr_broadcast")

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        check(self.rt.rkr_all_gather(self.h, inp.data_ptr(), out.data_ptr(), inp.numel(), _DT[inp.dtype],
                                     self._stream()), "rkr_all_gather")
        return out

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: int = SUM) -> torch.Tensor:
        check(self.rt.rkr_reduce_scatter(self.h, inp.data_ptr(), out.data_ptr(), out.numel(), _DT[inp.dtype], op,
                                         self._stream()), "rkr_reduce_scatter")
        return out

    def make_reducer(self, flats):
        return NativeReducer(self, flats)

    def close(self) -> None:
        if getattr(self, "h", None) is not None:
            self.rt.rkr_comm_destroy(self.h)
            self.h = None


class NativeReducer:
    """Bucket all-reduce on a side stream (event fork/join with the compute stream)."""

    def __init__(self, comm: RcclComm, flats):
        self.comm = comm
        self.rt = comm.rt
        h = ctypes.c_void_p()
        check(self.rt.rkr_reducer_create(ctypes.byref(h), comm.h, len(flats)), "rkr_reducer_create")
        self.h = h
        for i, f in enumerate(flats):
            check(self.rt.rkr_reducer_set_bucket(self.h, i, f.data_ptr(), f.numel(), _DT[f.dtype]),
                  "rkr_reducer_set_bucket")

    def launch(self, i: int) -> None:
        check(self.rt.rkr_reducer_launch(self.h, i, self.comm._stream()), "rkr_reducer_launch")

    def join(self) -> None:
        check(self.rt.rkr_reducer_join(self.h, self.comm._stream()), "rkr_reducer_join")

    def close(self) -> None:
        if getattr(self, "h", None) is not None:
            self.rt.rkr_reducer_destroy(self.h)
            self.h = None
