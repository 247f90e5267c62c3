"""Persistent flat gradient storage.

Every parameter's ``.grad`` becomes a view into one contiguous fp32 buffer per
(device, dtype).  What this buys on MI355X:

* gradients have **static addresses**, so a training step that produces and
  consumes them can be captured once into a HIP graph and replayed;
* ``zero_grad`` is one ``memset`` of the buffer instead of one kernel per tensor
  (or an allocation per tensor per step with ``set_to_none``);
* the fused kernels (:mod:`rocket_amd.ops`) accumulate weight gradients
  straight into ``param.grad`` (``param._rocket_direct_grad``), skipping
  autograd's AccumulateGrad copies;
* the data-parallel reducer can all-reduce the buffer (or contiguous slices of
  it) in place.

``DataParallel`` builds its bucket views with the same conventions, so a model
gets exactly one of the two.
"""

from __future__ import annotations

from typing import Dict, List, Tuple

import torch
from torch import nn


def _padded(n: int) -> int:
    """Elements a parameter occupies in a flat gradient buffer: rounded up to 4 (16 B of fp32),
    so every view starts 16-byte aligned for the native kernels' vector stores."""
    return (n + 3) // 4 * 4


def _param_view(flat: torch.Tensor, off: int, p: torch.Tensor) -> torch.Tensor:
    """A slice of ``flat`` shaped AND strided like ``p`` (channels-last weights get channels-last
    grads, so autograd accumulates in place instead of copying through a layout change)."""
    n = p.numel()
    if p.is_contiguous() or not _dense(p):
        return flat[off : off + n].view_as(p)
    return flat.as_strided(p.shape, p.stride(), flat.storage_offset() + off)


def _dense(p: torch.Tensor) -> bool:
    # non-overlapping and dense: the strides are a permutation of a contiguous layout
    dims = sorted(range(p.dim()), key=lambda d: p.stride(d))
    expect = 1
    for d in dims:
        if p.shape[d] != 1 and p.stride(d) != expect:
            return False
        expect *= p.shape[d]
    return True


class FlatGrads:
    def __init__(self, params: List[nn.Parameter]):
        groups: Dict[Tuple[torch.device, torch.dtype], List[nn.Parameter]] = {}
        for p in params:
            if p.requires_grad:
                groups.setdefault((p.device, p.dtype), []).append(p)
        self.buffers: List[torch.Tensor] = []
        self.params: List[nn.Parameter] = []
        self.views: List[torch.Tensor] = []
        for (dev, dtype), ps in groups.items():
            n = sum(_padded(p.numel()) for p in ps)
            flat = torch.zeros(n, dtype=dtype, device=dev)
            off = 0
            for p in ps:
                view = _param_view(flat, off, p)
                if p.grad is not None:
                    with torch.no_grad():
                        view.copy_(p.grad)
                p.grad = view
                p._rocket_direct_grad = True
                off += _padded(p.numel())  # 16-byte aligned views (zero pad between them)
                self.params.append(p)
                self.views.append(view)
            self.buffers.append(flat)
        self._ids = {id(p) for p in self.params}

    def owns(self, p: torch.Tensor) -> bool:
        return id(p) in self._ids

    def restore_views(self) -> None:
        """Re-point ``.grad`` at the buffer views (e.g. after ``zero_grad(set_to_none=True)``)."""
        for p, v in zip(self.params, self.views):
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                if p.grad is not None:
                    with torch.no_grad():
                        v.copy_(p.grad)
                else:
                    v.zero_()
                p.grad = v

    def zero_(self) -> None:
        for flat in self.buffers:
            flat.zero_()

    @property
    def numel(self) -> int:
        return sum(b.numel() for b in self.buffers)
