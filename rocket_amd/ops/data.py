"""Data-path ops: batch row gather and on-device loss bookkeeping (``native/kernels/data.hip``)."""

from __future__ import annotations

import ctypes
from typing import Sequence

import torch

from rocket_amd.ops import _lib

_MAX_GATHER = 4


def gather_rows(srcs: Sequence[torch.Tensor], idx: torch.Tensor, outs: Sequence[torch.Tensor]) -> None:
    """``outs[t][r] = srcs[t][idx[r]]`` for every tensor in one launch (HIP) or per tensor (CPU)."""
    n = idx.numel()
    dev = idx.device
    if dev.type != "cuda" or len(srcs) > _MAX_GATHER:
        for s, o in zip(srcs, outs):
            torch.index_select(s, 0, idx, out=o)
        return
    for s, o in zip(srcs, outs):
        if not (s.is_contiguous() and o.is_contiguous() and s.device == dev and o.shape[0] >= n
                and s.dtype == o.dtype and s.shape[1:] == o.shape[1:]):
            raise ValueError("gather_rows: contiguous same-dtype tensors on the index device expected")
    if idx.dtype != torch.int64:
        idx = idx.long()
    k = len(srcs)
    P = ctypes.c_void_p * k
    I = ctypes.c_int64 * k
    src_p = P(*[s.data_ptr() for s in srcs])
    dst_p = P(*[o.data_ptr() for o in outs])
    rb = I(*[s[0].numel() * s.element_size() if s.shape[0] else 0 for s in srcs])
    rows = I(*[s.shape[0] for s in srcs])
    lib = _lib.kernels()
    _lib.check(lib.rk_gather_rows(k, src_p, dst_p, rb, rows, idx.data_ptr(), n, _lib.stream_ptr(dev)),
               "rk_gather_rows")


class RowGather:
    """Pre-bound :func:`gather_rows` for fixed source/destination tensors (a loader ring slot):
    the argument arrays are built once, each call is one native launch."""

    def __init__(self, srcs: Sequence[torch.Tensor], outs: Sequence[torch.Tensor]):
        self.srcs, self.outs = list(srcs), list(outs)
        self.native = outs[0].device.type == "cuda" and len(srcs) <= _MAX_GATHER
        if self.native:
            for s, o in zip(srcs, outs):
                if not (s.is_contiguous() and o.is_contiguous() and s.dtype == o.dtype and s.shape[1:] == o.shape[1:]
                        and s.device == o.device):
                    raise ValueError("RowGather: contiguous same-dtype tensors on one device expected")
            k = len(srcs)
            self._args = ((ctypes.c_void_p * k)(*[s.data_ptr() for s in srcs]),
                          (ctypes.c_void_p * k)(*[o.data_ptr() for o in outs]),
                          (ctypes.c_int64 * k)(*[s[0].numel() * s.element_size() if s.shape[0] else 0 for s in srcs]),
                          (ctypes.c_int64 * k)(*[s.shape[0] for s in srcs]))
            self._k = k
            self._fn = _lib.kernels().rk_gather_rows
            self._any = _lib.kernels().rk_gather_rows_any_order
            self._dev = outs[0].device

    def __call__(self, idx: torch.Tensor, any_order: bool = False):
        """``any_order``: launch without waiting for the stream's previous packet (see
        ``rk_gather_rows_any_order``) — only when nothing in flight reads the destination or writes
        ``idx``."""
        if not self.native:
            for s, o in zip(self.srcs, self.outs):
                torch.index_select(s, 0, idx, out=o)
            return self.outs
        if any_order:
            self._any()
        code = self._fn(self._k, *self._args, idx.data_ptr(), idx.numel(), _lib.stream_ptr(self._dev))
        if code:
            _lib.check(code, "rk_gather_rows")
        return self.outs


def loss_accum(loss: torch.Tensor, acc: torch.Tensor, ring: torch.Tensor, slot: torch.Tensor, scale: float,
               sync: bool) -> None:
    """``acc += loss*scale``; if ``sync``: ``ring[slot] = acc; slot = (slot+1) % len(ring); acc = 0``.

    All operands are device tensors with static addresses (graph-capturable).
    """
    if loss.device.type == "cuda" and loss.dtype == torch.float32 and loss.numel() == 1:
        lib = _lib.kernels()
        _lib.check(lib.rk_loss_accum(loss.data_ptr(), acc.data_ptr(), ring.data_ptr(), slot.data_ptr(),
                                     ring.numel(), float(scale), int(sync), _lib.stream_ptr(loss.device)),
                   "rk_loss_accum")
        return
    acc.add_(loss.detach().float().reshape(acc.shape) * scale)
    if sync:
        ring.index_copy_(0, slot, acc.reshape(1))
        slot.add_(1).remainder_(ring.numel())
        acc.zero_()
