"""Channels-last bf16 convolutions on the native implicit-GEMM MFMA kernels (``native/kernels/conv.hip``).

:class:`IConv2d` is ``nn.Conv2d`` (same parameters / state_dict) whose forward, input gradient and
weight gradient under bf16 autocast on a HIP device each run as one implicit-GEMM launch (plus the
split-K combine of the weight gradient) — no im2col buffer, no MIOpen solution search, no
``SubTensorOp`` casts:

* forward: gathered NHWC activations x channels_last weights (read as a bf16 copy a fused
  optimizer keeps current: dense bf16 shadow, ``_bf16_copy``);
* dgrad (stride 1): dY gathered with the flipped taps x the weights read K-major per tap;
  strided convs take the library path for their input gradient;
* wgrad: dY x gathered X, split-K over the pixels into f32 slabs, accumulated straight into a
  persistent ``weight.grad`` when the engine provides one.

Shape rules (else the layer is exactly ``nn.Conv2d``): groups = 1, dilation = 1, Cin % 64 == 0
(the stem conv with 3 input channels stays on the library), Cout % 8 == 0.
``ROCKET_CONV=native`` (default) | ``lib``.
"""

from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from torch import nn

from rocket_amd.ops import _lib
from rocket_amd.ops.linear import _autocast_on, _bf16_copy, _direct, grad_ready
from rocket_amd.ops.mgemm import _slab

MODE = os.environ.get("ROCKET_CONV", "native")
N_SLOTS = 512  # resident 128x128 conv blocks (2 per CU)


def _cl(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.bfloat16:
        t = t.to(torch.bfloat16)
    return t.contiguous(memory_format=torch.channels_last)


def _wgrad_split(cout: int, ncol: int, pixels: int) -> int:
    """K-split of a conv weight gradient: few output tiles (Cout x R*S*Cin) over a long pixel
    reduction, so split the pixels until the grid fills the resident slots; each split costs one
    more f32 slab written and re-read by the combine launch."""
    bm = 64 if cout <= 64 else 128
    tiles = -(-cout // bm) * -(-ncol // 128)
    slots = 768 if bm == 64 else N_SLOTS  # 64x128 tile: 48 KiB LDS, 3 blocks per CU
    best, arg = None, 1
    for s in range(1, 257):
        if pixels // s < 512:
            break
        waves = -(-(tiles * s) // slots)
        slab_cost = 0.02 * s * tiles / slots  # combine traffic ~ one extra wave per 50 splits of the grid
        c = waves / s + slab_cost
        if best is None or c < best:
            best, arg = c, s
    return arg


class _IConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, w16, stride: int, pad: int):
        xc = _cl(x)
        N, C, H, W = xc.shape
        Co, _, R, S = w16.shape
        OH = (H + 2 * pad - R) // stride + 1
        OW = (W + 2 * pad - S) // stride + 1
        y = torch.empty((N, Co, OH, OW), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        _lib.check(_lib.kernels().rk_conv_fwd(xc.data_ptr(), w16.data_ptr(), y.data_ptr(), 1, None, N, H, W, C, Co, R, S,
                                               stride, pad, OH, OW, _lib.stream_ptr(x.device)), "rk_conv_fwd")
        ctx.save_for_backward(xc, w16)
        ctx.weight = weight
        ctx.geo = (N, C, H, W, Co, R, S, stride, pad, OH, OW)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, w16 = ctx.saved_tensors
        weight = ctx.weight
        N, C, H, W, Co, R, S, stride, pad, OH, OW = ctx.geo
        dyc = _cl(dy)
        lib = _lib.kernels()
        st = _lib.stream_ptr(dy.device)
        dx = None
        if ctx.needs_input_grad[0]:
            if stride == 1 and Co % 64 == 0:
                dx = torch.empty((N, C, H, W), dtype=torch.bfloat16, device=dy.device, memory_format=torch.channels_last)
                _lib.check(lib.rk_conv_dgrad(dyc.data_ptr(), w16.data_ptr(), dx.data_ptr(), 1, N, H, W, C, Co, R, S,
                                             stride, pad, OH, OW, st), "rk_conv_dgrad")
            else:
                dx = torch.nn.grad.conv2d_input((N, C, H, W), w16, dyc, stride=stride, padding=pad)
        dw = None
        if ctx.needs_input_grad[1]:
            direct = _direct(weight) and weight.grad.is_contiguous(memory_format=torch.channels_last)
            target = weight.grad if direct else torch.empty(weight.shape, dtype=torch.float32, device=dy.device,
                                                            memory_format=torch.channels_last)
            P, ncol = N * OH * OW, R * S * C
            split = _wgrad_split(Co, ncol, P)
            slab = _slab(dy.device, split * Co * ncol) if split > 1 else None
            _lib.check(lib.rk_conv_wgrad(dyc.data_ptr(), xc.data_ptr(), target.data_ptr(), int(direct), None, N, H, W,
                                         C, Co, R, S, stride, pad, OH, OW, split, _lib.ptr(slab), st), "rk_conv_wgrad")
            if direct:
                grad_ready(weight)
            else:
                dw = target
        return dx, dw, None, None, None


def native_ok(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    return (MODE == "native" and x.is_cuda and _autocast_on() and torch.get_autocast_dtype("cuda") == torch.bfloat16
            and conv.groups == 1 and conv.dilation == (1, 1) and conv.bias is None
            and conv.in_channels % 64 == 0 and conv.out_channels % 8 == 0 and conv.stride[0] == conv.stride[1]
            and conv.padding[0] == conv.padding[1] and isinstance(conv.padding[0], int)
            and conv.weight.dtype == torch.float32 and _lib.available())


class IConv2d(nn.Conv2d):
    """``nn.Conv2d`` on the native implicit-GEMM kernels (module docstring)."""

    def forward(self, x):
        if native_ok(self, x):
            if not self.weight.is_contiguous(memory_format=torch.channels_last):
                with torch.no_grad():
                    self.weight.data = self.weight.data.contiguous(memory_format=torch.channels_last)
            w16 = _bf16_copy(self, "_w16", self.weight)
            return _IConvFn.apply(x, self.weight, w16, self.stride[0], self.padding[0])
        return super().forward(x)


def conv2d_reference(x, w, stride, pad):
    """fp32 reference of the same op (tests)."""
    return F.conv2d(x.float(), w.float(), stride=stride, padding=pad)
