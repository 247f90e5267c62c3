"""Fused softmax cross-entropy (HIP kernel ``native/kernels/cross_entropy.hip``).

``cross_entropy(logits[N, C], target[N])`` matches ``torch.nn.functional.cross_entropy``
(class-index targets, ``ignore_index``, ``label_smoothing``, ``reduction`` in
{"mean", "sum"}).  Forward = one launch (loss reduced in-launch); backward =
one launch that recomputes the softmax and applies the incoming gradient read
from device memory.  Used by the reference example's loss
(``examples/mnist.py:81-84``) and the ViT/ResNet heads.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

from rocket_amd.ops import _lib


class _FusedCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index: int, smoothing: float, mean: bool):
        lib = _lib.kernels()
        logits = logits.contiguous()
        target = target.contiguous().to(torch.int64)
        N, C = logits.shape
        dev = logits.device
        stats = torch.empty(2, dtype=torch.float32, device=dev)
        partials = torch.empty(lib.rk_ce_partials_needed(N, C), dtype=torch.float32, device=dev)
        counter = _lib.Workspace.get(dev).counter("ce_fwd")
        _lib.check(
            lib.rk_ce_fwd(logits.data_ptr(), _lib.dtype_code(logits), target.data_ptr(), N, C, int(ignore_index),
                          float(smoothing), partials.data_ptr(), counter, stats.data_ptr(), int(mean),
                          _lib.stream_ptr(dev)),
            "rk_ce_fwd",
        )
        ctx.save_for_backward(logits, target, stats)
        ctx.cfg = (int(ignore_index), float(smoothing), bool(mean))
        return stats[0]

    @staticmethod
    def backward(ctx, g):
        lib = _lib.kernels()
        logits, target, stats = ctx.saved_tensors
        ignore_index, smoothing, mean = ctx.cfg
        N, C = logits.shape
        g = g.detach().float().contiguous()
        dlogits = torch.empty_like(logits)
        _lib.check(
            lib.rk_ce_bwd(logits.data_ptr(), _lib.dtype_code(logits), target.data_ptr(), dlogits.data_ptr(), N, C,
                          ignore_index, smoothing, g.data_ptr(), stats.data_ptr(), int(mean),
                          _lib.stream_ptr(logits.device)),
            "rk_ce_bwd",
        )
        return dlogits, None, None, None, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int = -100,
                  label_smoothing: float = 0.0, reduction: str = "mean") -> torch.Tensor:
    if (
        logits.device.type != "cuda"
        or logits.dim() != 2
        or target.dim() != 1
        or target.dtype.is_floating_point
        or reduction not in ("mean", "sum")
        or logits.dtype not in (torch.float32, torch.bfloat16, torch.float16)
    ):
        return F.cross_entropy(logits.float(), target, ignore_index=ignore_index,
                               label_smoothing=label_smoothing, reduction=reduction)
    return _FusedCE.apply(logits, target, ignore_index, label_smoothing, reduction == "mean")


def ce_train(logits: torch.Tensor, target: torch.Tensor, grad_scale: float, accum=None, ignore_index: int = -100,
             label_smoothing: float = 0.0, reduction: str = "mean"):
    """Loss AND d(logits) of a training step in one launch (see ``ce_train_kernel``).

    ``grad_scale`` is the upstream gradient of the loss (e.g. 1/GA); ``accum`` optionally
    ``(acc, ring, slot, acc_scale, sync)`` — the Loss capsule's device bookkeeping, updated by the
    same launch.  Returns ``(loss[0-d], dlogits)`` or ``None`` when the case is not covered.
    """
    if (logits.device.type != "cuda" or logits.dim() != 2 or target.dim() != 1 or target.dtype.is_floating_point
            or reduction not in ("mean", "sum") or logits.dtype not in (torch.float32, torch.bfloat16, torch.float16)
            or logits.shape[0] > 65536):
        return None
    lib = _lib.kernels()
    logits = logits.detach().contiguous()
    target = target.contiguous().to(torch.int64)
    N, C = logits.shape
    dev = logits.device
    stats = torch.empty(2, dtype=torch.float32, device=dev)
    partials = torch.empty(lib.rk_ce_partials_needed(N, C), dtype=torch.float32, device=dev)
    dlogits = torch.empty_like(logits)
    counter = _lib.Workspace.get(dev).counter("ce_train")
    acc = ring = slot = None
    acc_scale, sync = 0.0, 0
    if accum is not None:
        acc, ring, slot, acc_scale, sync = accum
    _lib.check(lib.rk_ce_train(logits.data_ptr(), _lib.dtype_code(logits), target.data_ptr(), dlogits.data_ptr(), N, C,
                               int(ignore_index), float(label_smoothing), float(grad_scale), partials.data_ptr(),
                               counter, stats.data_ptr(), int(reduction == "mean"), _lib.ptr(acc), _lib.ptr(ring),
                               _lib.ptr(slot), ring.numel() if ring is not None else 0, float(acc_scale), int(sync),
                               _lib.stream_ptr(dev)), "rk_ce_train")
    return stats[0], dlogits
