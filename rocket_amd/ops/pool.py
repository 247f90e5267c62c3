"""Global average pooling of channels-last activations (the ResNet head, ``norm.hip rk_gap_fwd /
rk_gap_bwd``): the pooled [N, C] comes out in the activation's dtype with fp32 sums, and the
backward writes the broadcast ``dy / HW`` straight into a channels-last gradient — one launch each,
where ``F.adaptive_avg_pool2d`` + ``flatten`` cost a reduction plus an expand / divide pass.

Reference parity: ``torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)`` (torchvision ResNet head)."""

from __future__ import annotations

import torch
import torch.nn.functional as F

from rocket_amd.ops import _lib

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


class _GapFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        out = torch.empty(N, C, dtype=x.dtype, device=x.device)
        _lib.check(_lib.kernels().rk_gap_fwd(_DT[x.dtype], _DT[out.dtype], x.data_ptr(), out.data_ptr(), N, H * W, C,
                                             _lib.stream_ptr(x.device)), "rk_gap_fwd")
        ctx.shape = (N, C, H, W)
        ctx.dtype = x.dtype
        return out

    @staticmethod
    def backward(ctx, dy):
        N, C, H, W = ctx.shape
        dy = dy.contiguous()
        if dy.dtype not in _DT:
            dy = dy.float()
        dx = torch.empty((N, C, H, W), dtype=ctx.dtype, device=dy.device, memory_format=torch.channels_last)
        _lib.check(_lib.kernels().rk_gap_bwd(_DT[ctx.dtype], _DT[dy.dtype], dy.data_ptr(), dx.data_ptr(), N, H * W, C,
                                             _lib.stream_ptr(dy.device)), "rk_gap_bwd")
        return dx


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """``[N, C, H, W] -> [N, C]`` mean over H, W.  Native for a channels-last CUDA tensor with C % 8 == 0
    (16-bit dtypes must match between the pooled output and its gradient), else PyTorch's."""
    if (x.is_cuda and x.dim() == 4 and x.dtype in _DT and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last)):
        return _GapFn.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
