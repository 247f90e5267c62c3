"""GELU and row softmax on HIP (``native/kernels/act.hip``) + the attention composite.

* :func:`gelu` — exact (erf) GELU; backward recomputes the derivative from the saved input.
* :func:`softmax` — ``softmax(x * scale)`` over the last dim in one read/one write, with the
  fused backward ``scale * y * (dy - <dy, y>)`` (rows up to 1024 long).
* :func:`attention` — ``softmax(q k^T * scale) v`` for short sequences (ViT: 197 tokens):
  the two batched GEMMs run on the library (hipBLASLt) path, the scaled softmax on the
  kernel above, so the score matrix is read and written once per direction.
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

import rocket_amd.ops as _ops
from rocket_amd.ops import _lib


class _Gelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        y = torch.empty_like(x)
        _lib.check(_lib.kernels().rk_gelu_fwd(_lib.dtype_code(x), _lib.dtype_code(y), x.data_ptr(), y.data_ptr(),
                                              x.numel(), _lib.stream_ptr(x.device)), "rk_gelu_fwd")
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        _lib.check(_lib.kernels().rk_gelu_bwd(_lib.dtype_code(x), _lib.dtype_code(dy), dy.data_ptr(), x.data_ptr(),
                                              dx.data_ptr(), x.numel(), _lib.stream_ptr(x.device)), "rk_gelu_bwd")
        return dx


def gelu(x: torch.Tensor) -> torch.Tensor:
    if _ops.fused_enabled() and x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and x.numel() % 4 == 0:
        return _Gelu.apply(x)
    return F.gelu(x)


class _Softmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scale):
        x = x.contiguous()
        L = x.shape[-1]
        rows = x.numel() // L
        y = torch.empty_like(x)
        _lib.check(_lib.kernels().rk_softmax_fwd(_lib.dtype_code(x), _lib.dtype_code(y), x.data_ptr(), y.data_ptr(),
                                                 rows, L, float(scale), _lib.stream_ptr(x.device)), "rk_softmax_fwd")
        ctx.scale = scale
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = dy.contiguous()
        L = y.shape[-1]
        rows = y.numel() // L
        dx = torch.empty_like(dy)
        _lib.check(_lib.kernels().rk_softmax_bwd(_lib.dtype_code(y), _lib.dtype_code(dy), dy.data_ptr(), y.data_ptr(),
                                                 dx.data_ptr(), rows, L, float(ctx.scale), _lib.stream_ptr(y.device)),
                   "rk_softmax_bwd")
        return dx, None


def softmax(x: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    if _ops.fused_enabled() and x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and x.shape[-1] <= 1024:
        return _Softmax.apply(x, scale)
    return torch.softmax(x.float() * scale, dim=-1).to(x.dtype)


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float | None = None) -> torch.Tensor:
    """q, k, v: [B, H, L, D] -> [B, H, L, D]."""
    scale = 1.0 / math.sqrt(q.shape[-1]) if scale is None else scale
    s = torch.matmul(q, k.transpose(-2, -1))
    p = softmax(s, scale)
    return torch.matmul(p, v)
