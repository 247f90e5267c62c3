"""Fused conv2d + bias + ReLU + 2x2 max-pool (``native/kernels/conv_pool.hip``).

``conv_bias_relu_pool(x, weight, bias, padding)`` ==
``max_pool2d(relu(conv2d(x, weight, bias, padding=padding)), 2)`` for stride-1
square kernels and small channel counts (the LeNet / MNIST layers).  The
forward writes only the pooled activation (bf16 under AMP) and a 1-byte
argmax/ReLU code per pooled element; the backward routes gradients through
that code (no dense pre-pool tensors, no separate pool/ReLU backward kernels).
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

from rocket_amd.ops import _lib
from rocket_amd.ops.linear import _autocast_on, _direct, grad_ready


class _ConvReluPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, padding: int, out_dtype):
        lib = _lib.kernels()
        x = x.contiguous()
        if x.dtype not in (torch.float32, torch.bfloat16):
            x = x.float()
        N, Ci, H, W = x.shape
        Co, Ci2, K, K2 = weight.shape
        assert Ci == Ci2 and K == K2, "square kernel / matching channels required"
        Hp, Wp = (H + 2 * padding - K + 1) // 2, (W + 2 * padding - K + 1) // 2
        w = weight.detach().float().contiguous()
        b = bias.detach().float().contiguous() if bias is not None else None
        y = torch.empty(N, Co, Hp, Wp, dtype=out_dtype, device=x.device)
        code = torch.empty(N, Co, Hp, Wp, dtype=torch.uint8, device=x.device)
        _lib.check(
            lib.rk_conv_pool_fwd(x.data_ptr(), _lib.dtype_code(x), w.data_ptr(), _lib.ptr(b), y.data_ptr(),
                                 _lib.dtype_code(y), code.data_ptr(), N, Ci, H, W, Co, K, padding,
                                 _lib.stream_ptr(x.device)),
            "rk_conv_pool_fwd",
        )
        ctx.padding = padding
        ctx.params = (weight, bias)
        ctx.save_for_backward(x, w, code)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib.kernels()
        x, w, code = ctx.saved_tensors
        P = ctx.padding
        N, Ci, H, W = x.shape
        Co, _, K, _ = w.shape
        dy = dy.contiguous()
        if dy.dtype not in (torch.float32, torch.bfloat16):
            dy = dy.float()
        stream = _lib.stream_ptr(x.device)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            _lib.check(
                lib.rk_conv_pool_dgrad(dy.data_ptr(), _lib.dtype_code(dy), code.data_ptr(), w.data_ptr(),
                                       dx.data_ptr(), _lib.dtype_code(dx), N, Ci, H, W, Co, K, P, stream),
                "rk_conv_pool_dgrad",
            )
        weight, bias = ctx.params
        need_w = ctx.needs_input_grad[1]
        need_b = bias is not None and ctx.needs_input_grad[2]
        if need_w or need_b:
            direct = _direct(weight) and (bias is None or _direct(bias))
            if direct:
                gw, gb = weight.grad, (bias.grad if bias is not None else None)
            else:
                gw = torch.zeros(Co, Ci, K, K, dtype=torch.float32, device=x.device)
                gb = torch.zeros(Co, dtype=torch.float32, device=x.device) if bias is not None else None
            _lib.check(
                lib.rk_conv_pool_wgrad(x.data_ptr(), _lib.dtype_code(x), dy.data_ptr(), _lib.dtype_code(dy),
                                       code.data_ptr(), gw.data_ptr(), _lib.ptr(gb), N, Ci, H, W, Co, K, P, stream),
                "rk_conv_pool_wgrad",
            )
            if direct:
                grad_ready(weight)
                if bias is not None:
                    grad_ready(bias)
            else:
                dw = gw if need_w else None
                db = gb if need_b else None
        return dx, dw, db, None, None


def conv_bias_relu_pool(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None, padding: int = 0,
                        out_dtype: torch.dtype | None = None) -> torch.Tensor:
    if x.device.type != "cuda":
        return F.max_pool2d(F.relu(F.conv2d(x, weight, bias, padding=padding)), 2)
    if out_dtype is None:
        out_dtype = torch.bfloat16 if (_autocast_on() or x.dtype == torch.bfloat16) else torch.float32
    return _ConvReluPool.apply(x, weight, bias, padding, out_dtype)
