"""Channels-last bf16 / fp16 convolutions on the native implicit-GEMM MFMA kernels (``native/kernels/conv.hip``).

:class:`IConv2d` is ``nn.Conv2d`` (same parameters / state_dict) whose forward, input gradient and
weight gradient under bf16 or fp16 autocast on a HIP device each run as one implicit-GEMM launch
(MFMA bf16 / f16 by the autocast dtype, f32 accumulation; plus the
split-K combine of the weight gradient) — no im2col buffer, no MIOpen solution search, no
``SubTensorOp`` casts:

* forward: gathered NHWC activations x channels_last weights (read as a bf16 copy a fused
  optimizer keeps current: dense bf16 / fp16 shadow, ``_lowp_copy``);
* dgrad: dY gathered with the flipped taps x the weights read K-major per tap; stride 2 as the
  four parity classes of dX pixels (each a stride-1 gather over its taps) in one launch;
* wgrad: dY x gathered X, split-K over the pixels into f32 slabs, accumulated straight into a
  persistent ``weight.grad`` when the engine provides one.

Shape rules (else the layer is exactly ``nn.Conv2d``): groups = 1, dilation = 1, Cin % 64 == 0,
Cout % 8 == 0.  The stem conv (Cin <= 8, an input that takes no gradient: the image) runs natively
too (:class:`_StemFn`): the image is padded to 8 channels (one 16-byte chunk per pixel) by one
launch, the forward gathers one tap per chunk (``rk_conv_fwd_c8``, BatchNorm statistics in its
epilogue) and the weight gradient is the ordinary wgrad kernel on the padded image, its pad
columns dropped.  ``ROCKET_CONV=native`` (default) | ``lib``.
"""

from __future__ import annotations

import functools
import os

import torch
import torch.nn.functional as F
from torch import nn

from rocket_amd.ops import _lib
from rocket_amd.ops.linear import _direct, _lowp_copy, grad_ready, native_route
from rocket_amd.ops.mgemm import _slab

MODE = os.environ.get("ROCKET_CONV", "native")
# strided (stride-2) input gradients: native parity-class launch or the library
SDGRAD = os.environ.get("ROCKET_CONV_SDGRAD", "native")
# wgrad split-K combine in the following dgrad launch (conv.hip TailJob); 0: its own launch
DEFER_REDUCE = os.environ.get("ROCKET_CONV_DEFER_REDUCE", "1") != "0"
# residual-block entries (first conv + shortcut) as one autograd node: ROCKET_CONV_ENTRY=0 disables
ENTRY = os.environ.get("ROCKET_CONV_ENTRY", "1") != "0"
N_SLOTS = 512  # resident 128x128 conv blocks (2 per CU)
# bf16 conv outputs / input gradients stored through LDS in row-contiguous chunks (conv.hip
# store_tile_lds); ROCKET_CONV_LDS_EPI=0 stores straight from the MFMA accumulator layout
LDS_EPI = os.environ.get("ROCKET_CONV_LDS_EPI", "1") != "0"
# k-tile pipeline of the bf16 conv kernels (conv.hip rk_conv_set_cfg)
PIPE = int(os.environ.get("ROCKET_CONV_PIPE", "0"))
# tile walk of the conv kernels: tile-rows per group (rk_common.h grouped_tile; 1 = row-major).
# Grouped walks (4 tile-rows) measured neutral-to-slower on ResNet-50/18 (activation panels already
# fit L2): profiles/r4_conv_tile_group_ab.md
TILE_GROUP = int(os.environ.get("ROCKET_CONV_TILE_GROUP", "1"))
_epi_set = False


def _kernels():
    global _epi_set
    lib = _lib.kernels()
    if not _epi_set:
        lib.rk_conv_set_lds_epi(int(LDS_EPI))
        if lib.rk_conv_set_cfg(PIPE):
            raise ValueError(f"ROCKET_CONV_PIPE={PIPE}: no such conv pipeline")
        lib.rk_conv_set_tile_group(TILE_GROUP)
        _epi_set = True
    return lib


_LOWP = (torch.bfloat16, torch.float16)


def _cl(t: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    if t.dtype != dtype:
        t = t.to(dtype)
    return t.contiguous(memory_format=torch.channels_last)


def _dt(t: torch.Tensor) -> int:
    """conv.hip operand dtype code (BF16 = 1, F16 = 2)."""
    return 2 if t.dtype == torch.float16 else 1


# modelled per-CU rate of the wgrad kernel (ROCKET_WGRAD_RATE_CU: the split-K choice's GEMM-vs-slab
# trade-off; 3.5e12 = ~0.9 PF/s over 256 CUs)
WGRAD_RATE_CU = float(os.environ.get("ROCKET_WGRAD_RATE_CU", "3.5e12"))


@functools.lru_cache(maxsize=None)
def _wgrad_split(cout: int, ncol: int, pixels: int) -> int:
    """K-split of a conv weight gradient (few output tiles, long pixel reduction): minimise
    modelled time = waves of resident blocks x per-block MFMA time + the split-K slab traffic
    (each split writes one f32 [Cout][R*S*Cin] slab that the combine launch re-reads)."""
    bm, per_cu = (64, 3) if cout <= 64 else (128, 2)
    tiles = -(-cout // bm) * -(-ncol // 128)
    rate_cu = WGRAD_RATE_CU  # sustained bf16 FLOP/s per CU of this kernel
    best, arg = None, 1
    for s in range(1, 257):
        if s > 1 and pixels // s < 256:
            break
        waves = -(-(tiles * s) // (256 * per_cu))
        t_gemm = waves * (2.0 * bm * 128 * (pixels / s)) * per_cu / rate_cu
        t_slab = 0.0 if s == 1 else (2.0 * s * cout * ncol * 4) / 4.0e12 + 3e-6
        c = t_gemm + t_slab
        if best is None or c < best:
            best, arg = c, s
    return arg


def _sdgrad_ok(R: int, S: int, pad: int) -> bool:
    # every parity class of a stride-2 input gradient needs taps, except the 1x1 / pad-0 case whose
    # three empty classes the (0, 0) tiles zero themselves
    return (R > 1 and S > 1) or (R == 1 and S == 1 and pad == 0)


TILE_ROWS = 64  # rows per wave slice of every conv.hip forward variant (BatchNorm partials granularity)


def _conv_fwd(xc: torch.Tensor, w16: torch.Tensor, stride: int, pad: int, bnpart) -> torch.Tensor:
    N, C, H, W = xc.shape
    Co, _, R, S = w16.shape
    OH = (H + 2 * pad - R) // stride + 1
    OW = (W + 2 * pad - S) // stride + 1
    y = torch.empty((N, Co, OH, OW), dtype=xc.dtype, device=xc.device, memory_format=torch.channels_last)
    _lib.check(_kernels().rk_conv_fwd(_dt(xc), xc.data_ptr(), w16.data_ptr(), y.data_ptr(), _dt(xc), None, N, H, W, C,
                                      Co, R, S,
                                           stride, pad, OH, OW, _lib.ptr(bnpart), _lib.stream_ptr(xc.device)),
               "rk_conv_fwd")
    return y


def _geo(xc: torch.Tensor, w16: torch.Tensor, stride: int, pad: int):
    N, C, H, W = xc.shape
    Co, _, R, S = w16.shape
    return (N, C, H, W, Co, R, S, stride, pad, (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1)


def _bn_src(x: torch.Tensor, stride: int):
    """The :class:`norm.BwdLink` when ``x`` is a fused BatchNorm's output that a stride-1 dgrad can
    finish the backward reduction of (``norm.py`` ``_rocket_bn_bwd_src``), else None."""
    link = getattr(x, "_rocket_bn_bwd_src", None)
    if link is None or link.src is None or stride != 1:
        return None
    z = link.src[0]
    if z.shape != x.shape or z.dtype not in _LOWP or not z.is_contiguous(memory_format=torch.channels_last):
        return None
    return link


def _conv_dgrad(dyc: torch.Tensor, w16: torch.Tensor, geo, dx: torch.Tensor | None, bn=None) -> torch.Tensor:
    """Input gradient of one conv; with ``dx`` given it is ADDED to dx (in place, native epilogue
    accumulate) and dx is returned.  ``bn`` (:func:`_bn_src`): the input is that BatchNorm's output —
    the epilogue also applies its ReLU mask and writes its backward reduction partials, handed to
    the BatchNorm's backward through the link (``norm.BwdLink.done``)."""
    N, C, H, W, Co, R, S, stride, pad, OH, OW = geo
    if (bn is not None and bn.src is not None and stride == 1 and Co % 64 == 0 and C % 8 == 0
            and bn.src[0].dtype == dyc.dtype):
        z, mask, stats = bn.src
        acc = dx is not None
        if dx is None:
            dx = torch.empty((N, C, H, W), dtype=dyc.dtype, device=dyc.device, memory_format=torch.channels_last)
        ntiles = -(-(N * H * W) // 128)  # one partial row per 128-pixel dgrad tile
        part = torch.empty(ntiles * 2 * C, dtype=torch.float32, device=dyc.device)
        _lib.check(_lib.kernels().rk_conv_dgrad_bn(_dt(dyc), dyc.data_ptr(), w16.data_ptr(), dx.data_ptr(), int(acc), N, H, W, C,
                                                   Co, R, S, pad, z.data_ptr(), _lib.ptr(mask), stats[0].data_ptr(),
                                                   stats[1].data_ptr(), part.data_ptr(), _lib.stream_ptr(dyc.device)),
                   "rk_conv_dgrad_bn")
        bn.done = (dx.data_ptr(), dx._version, part, ntiles)
        return dx
    if (stride == 1 or (stride == 2 and SDGRAD == "native" and _sdgrad_ok(R, S, pad))) and Co % 64 == 0:
        acc = dx is not None
        if dx is None:
            dx = torch.empty((N, C, H, W), dtype=dyc.dtype, device=dyc.device, memory_format=torch.channels_last)
        _lib.check(_kernels().rk_conv_dgrad(_dt(dyc), dyc.data_ptr(), w16.data_ptr(), dx.data_ptr(), _dt(dx), int(acc), N, H, W,
                                                C, Co, R, S, stride, pad, OH, OW, _lib.stream_ptr(dyc.device)),
                   "rk_conv_dgrad")
        return dx
    g = torch.nn.grad.conv2d_input((N, C, H, W), w16, dyc, stride=stride, padding=pad)
    return g if dx is None else dx.add_(g)


def _conv_wgrad(dyc: torch.Tensor, xc: torch.Tensor, weight: torch.Tensor, geo, defer: bool = False):
    """Weight gradient, accumulated straight into a persistent ``weight.grad`` when the engine
    provides one (returns None then), else returned.

    ``defer``: the split-K combine is left to the next conv launch on the stream (conv.hip TailJob:
    appended blocks of the dgrad the caller issues next) and a finisher is returned instead — call
    it right after that dgrad: it launches the combine if no conv launch took it, then marks the
    gradient ready (DP bucket hooks) and returns what the plain call would."""
    N, C, H, W, Co, R, S, stride, pad, OH, OW = geo
    direct = _direct(weight) and weight.grad.is_contiguous(memory_format=torch.channels_last)
    target = weight.grad if direct else torch.empty(weight.shape, dtype=torch.float32, device=dyc.device,
                                                    memory_format=torch.channels_last)
    P, ncol = N * OH * OW, R * S * C
    split = _wgrad_split(Co, ncol, P)
    slab = _slab(dyc.device, split * Co * ncol) if split > 1 else None
    lib = _lib.kernels()
    stream = _lib.stream_ptr(dyc.device)
    defer = defer and split > 1
    if defer:
        lib.rk_conv_defer_reduce(1)
    try:
        _lib.check(lib.rk_conv_wgrad(_dt(xc), dyc.data_ptr(), xc.data_ptr(), target.data_ptr(), int(direct), None, N, H,
                                     W, C, Co, R, S, stride, pad, OH, OW, split, _lib.ptr(slab), stream), "rk_conv_wgrad")
    finally:
        if defer:
            lib.rk_conv_defer_reduce(0)

    def finish():
        if defer:
            _lib.check(lib.rk_conv_flush_reduce(stream), "rk_conv_flush_reduce")
        if direct:
            grad_ready(weight)
            return None
        return target

    return finish if defer else finish()



class _IConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, w16, stride: int, pad: int, bnpart, bn=None):
        xc = _cl(x, w16.dtype)
        y = _conv_fwd(xc, w16, stride, pad, bnpart)
        ctx.save_for_backward(xc, w16)
        ctx.weight = weight
        ctx.bn = bn
        ctx.geo = _geo(xc, w16, stride, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, w16 = ctx.saved_tensors
        dyc = _cl(dy, xc.dtype)
        need = ctx.needs_input_grad
        # the wgrad first: its split-K combine rides in the dgrad's launch (DEFER_REDUCE)
        fin = _conv_wgrad(dyc, xc, ctx.weight, ctx.geo, defer=DEFER_REDUCE and need[0]) if need[1] else None
        dx = _conv_dgrad(dyc, w16, ctx.geo, None, ctx.bn) if need[0] else None
        dw = fin() if callable(fin) else fin
        ctx.bn = None
        return dx, dw, None, None, None, None, None


class _EntryFn(torch.autograd.Function):
    """A residual block's entry: ``(conv_a(x), conv_b(x) or x)`` as ONE autograd node.

    x feeds the block's first conv and its shortcut (identity or downsample conv).  As separate
    nodes autograd would sum the two input gradients with an add kernel over x; here the backward
    gets both output gradients at once and the second input gradient is accumulated by the conv
    dgrad epilogue into the first (the shortcut's gradient for an identity)."""

    @staticmethod
    def forward(ctx, x, wa, wa16, sa, pa, parta, wb, wb16, sb, pb, partb, bn=None):
        ctx.bn = bn  # conv_a's dgrad is the last write of dx: it finishes x's BatchNorm reduction
        xc = _cl(x, wa16.dtype)
        ya = _conv_fwd(xc, wa16, sa, pa, parta)
        yb = _conv_fwd(xc, wb16, sb, pb, partb) if wb is not None else xc.view_as(xc)
        ctx.save_for_backward(xc, wa16, wb16 if wb is not None else None)
        ctx.weights = (wa, wb)
        ctx.geo = (_geo(xc, wa16, sa, pa), _geo(xc, wb16, sb, pb) if wb is not None else None)
        return ya, yb

    @staticmethod
    def backward(ctx, ga, gb):
        xc, wa16, wb16 = ctx.saved_tensors
        wa, wb = ctx.weights
        geo_a, geo_b = ctx.geo
        need = ctx.needs_input_grad
        dx = None
        gac = _cl(ga, xc.dtype) if ga is not None else None
        gbc = _cl(gb, xc.dtype) if gb is not None else None
        # each wgrad just before the dgrad of the same conv: its split-K combine rides in that
        # dgrad's launch (DEFER_REDUCE); the finisher runs before the next wgrad is issued
        wa_do = need[1] and gac is not None
        wb_do = wb is not None and need[6] and gbc is not None
        dwa = dwb = None
        if need[0]:
            if gbc is not None:
                # shortcut first: downsample dgrad into a fresh dx / the identity's gradient as dx
                if wb is not None:
                    fin = _conv_wgrad(gbc, xc, wb, geo_b, defer=DEFER_REDUCE) if wb_do else None
                    dx = _conv_dgrad(gbc, wb16, geo_b, None)
                    dwb = fin() if callable(fin) else fin
                    wb_do = False
                else:
                    dx = gbc
            if gac is not None:
                fin = _conv_wgrad(gac, xc, wa, geo_a, defer=DEFER_REDUCE) if wa_do else None
                dx = _conv_dgrad(gac, wa16, geo_a, dx, ctx.bn)
                dwa = fin() if callable(fin) else fin
                wa_do = False
            if dx is None:
                dx = torch.zeros_like(xc)
        if wa_do:
            dwa = _conv_wgrad(gac, xc, wa, geo_a)
        if wb_do:
            dwb = _conv_wgrad(gbc, xc, wb, geo_b)
        ctx.bn = None
        return dx, dwa, None, None, None, None, dwb, None, None, None, None, None


def _stem_weight(weight: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """[Cout][Cin][R][S] fp32 -> bf16 / fp16 [Cout][Kp], taps' 8 (zero-padded) channels in (r, s, c)
    order, K padded to whole 64-deep k-tiles."""
    co, ci, R, S = weight.shape
    kp = -(-(R * S * 8) // 64) * 64
    w8 = torch.zeros(co, kp, dtype=dtype, device=weight.device)
    with torch.no_grad():
        w8[:, : R * S * 8].view(co, R, S, 8)[..., :ci].copy_(weight.detach().permute(0, 2, 3, 1))
    return w8


def _stem_weight_into(weight: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """:func:`_stem_weight` into a buffer kept on the parameter: its zero padding is written once,
    each step only copies the live taps (one launch instead of a fill and a copy).  A buffer first
    needed inside a graph capture is not kept (its memory would belong to the capture's pool)."""
    co, ci, R, S = weight.shape
    kp = -(-(R * S * 8) // 64) * 64
    buf = getattr(weight, "_rocket_w8", None)
    if buf is None or buf.dtype != dtype or buf.device != weight.device or buf.shape != (co, kp):
        if torch.cuda.is_current_stream_capturing():
            return _stem_weight(weight, dtype)
        buf = torch.zeros(co, kp, dtype=dtype, device=weight.device)
        weight._rocket_w8 = buf
    with torch.no_grad():
        buf[:, : R * S * 8].view(co, R, S, 8)[..., :ci].copy_(weight.detach().permute(0, 2, 3, 1))
    return buf


class _StemFn(torch.autograd.Function):
    """Stem conv (Cin <= 8) on the native kernels; the input (the image) takes no gradient."""

    @staticmethod
    def forward(ctx, x, weight, stride: int, pad: int, bnpart):
        N, C, H, W = x.shape
        co, _, R, S = weight.shape
        OH, OW = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
        dev = x.device
        s = _lib.stream_ptr(dev)
        lib = _kernels()
        cdt = torch.get_autocast_dtype("cuda")
        xc = x if x.dtype == cdt else x.to(cdt)
        sn, sc, sh, sw = xc.stride()
        if not (sh == W * sw and (sw == 1 or sw == C)):  # pixels must be evenly strided (NCHW or NHWC)
            xc = xc.contiguous(memory_format=torch.channels_last)
            sn, sc, sh, sw = xc.stride()
        x8 = torch.empty((N, H, W, 8), dtype=cdt, device=dev)
        _lib.check(lib.rk_pad_c8(xc.data_ptr(), x8.data_ptr(), N, C, H, W, sn, sc, sw, s), "rk_pad_c8")
        w8 = _stem_weight_into(weight, cdt)
        y = torch.empty((N, co, OH, OW), dtype=cdt, device=dev, memory_format=torch.channels_last)
        _lib.check(lib.rk_conv_fwd_c8(_dt(x8), x8.data_ptr(), w8.data_ptr(), y.data_ptr(), N, H, W, co, R, S, stride, pad, OH,
                                      OW, _lib.ptr(bnpart), s), "rk_conv_fwd_c8")
        ctx.save_for_backward(x8)
        ctx.weight = weight
        ctx.geo = (N, 8, H, W, co, R, S, stride, pad, OH, OW)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x8,) = ctx.saved_tensors
        weight = ctx.weight
        N, C8, H, W, co, R, S, stride, pad, OH, OW = ctx.geo
        if not ctx.needs_input_grad[1]:
            return None, None, None, None, None
        dyc = _cl(dy, x8.dtype)
        dev = dy.device
        P, ncol = N * OH * OW, R * S * C8
        t8 = torch.empty(co, ncol, dtype=torch.float32, device=dev)
        split = _wgrad_split(co, ncol, P)
        slab = _slab(dev, split * co * ncol) if split > 1 else None
        _lib.check(_lib.kernels().rk_conv_wgrad(_dt(x8), dyc.data_ptr(), x8.data_ptr(), t8.data_ptr(), 0, None, N, H, W, C8, co,
                                                R, S, stride, pad, OH, OW, split, _lib.ptr(slab),
                                                _lib.stream_ptr(dev)), "rk_conv_wgrad(stem)")
        g = t8.view(co, R, S, C8)[..., : weight.shape[1]].permute(0, 3, 1, 2)  # [Cout][Cin][R][S] view
        if _direct(weight):
            weight.grad.add_(g)
            grad_ready(weight)
            return None, None, None, None, None
        return None, g.contiguous(memory_format=torch.channels_last), None, None, None


def stem_ok(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    return (MODE == "native" and x.is_cuda and native_route() and torch.get_autocast_dtype("cuda") in _LOWP
            and conv.groups == 1 and conv.dilation == (1, 1) and conv.bias is None and conv.in_channels <= 8
            and conv.out_channels % 8 == 0 and conv.stride[0] == conv.stride[1] and conv.padding[0] == conv.padding[1]
            and isinstance(conv.padding[0], int) and conv.weight.dtype == torch.float32 and x.dim() == 4
            and not x.requires_grad and _lib.available())


def native_ok(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    return (MODE == "native" and x.is_cuda and native_route() and torch.get_autocast_dtype("cuda") in _LOWP
            and conv.groups == 1 and conv.dilation == (1, 1) and conv.bias is None
            and conv.in_channels % 64 == 0 and conv.out_channels % 8 == 0 and conv.stride[0] == conv.stride[1]
            and conv.kernel_size[0] * conv.kernel_size[1] <= 32  # conv.hip gathers: tap-validity bit masks
            and conv.padding[0] == conv.padding[1] and isinstance(conv.padding[0], int)
            and conv.weight.dtype == torch.float32 and _lib.available())


class IConv2d(nn.Conv2d):
    """``nn.Conv2d`` on the native implicit-GEMM kernels (module docstring).

    ``emit_bn_stats = True`` (set by models whose conv feeds a :class:`BatchNormAct2d`): the
    forward epilogue also writes per-64-pixel BatchNorm partials (sum and sum of squares per
    channel), attached to the output as ``_rocket_bn_partials``; the BatchNorm then merges those
    instead of re-reading the activation for its statistics."""

    emit_bn_stats = False

    def _prep(self, x):
        """(16-bit weight copy in the autocast dtype, BN partials buffer or None) for a native forward."""
        if not self.weight.is_contiguous(memory_format=torch.channels_last):
            with torch.no_grad():
                self.weight.data = self.weight.data.contiguous(memory_format=torch.channels_last)
        w16 = _lowp_copy(self, "_w16", self.weight, torch.get_autocast_dtype("cuda"))
        part = None
        if self.emit_bn_stats:
            N, _, H, W = x.shape
            OH = (H + 2 * self.padding[0] - self.kernel_size[0]) // self.stride[0] + 1
            OW = (W + 2 * self.padding[1] - self.kernel_size[1]) // self.stride[1] + 1
            ntiles = -(-(N * OH * OW) // TILE_ROWS)
            part = torch.empty(ntiles * 2 * self.out_channels, dtype=torch.float32, device=x.device)
        return w16, part

    def _attach(self, y, part):
        if part is not None:
            y._rocket_bn_partials = (part, part.numel() // (2 * self.out_channels), TILE_ROWS)
        return y

    def forward(self, x):
        if stem_ok(self, x):
            part = None
            if self.emit_bn_stats:
                N, _, H, W = x.shape
                OH = (H + 2 * self.padding[0] - self.kernel_size[0]) // self.stride[0] + 1
                OW = (W + 2 * self.padding[1] - self.kernel_size[1]) // self.stride[1] + 1
                part = torch.empty(-(-(N * OH * OW) // TILE_ROWS) * 2 * self.out_channels, dtype=torch.float32,
                                   device=x.device)
            return self._attach(_StemFn.apply(x, self.weight, self.stride[0], self.padding[0], part), part)
        if native_ok(self, x):
            w16, part = self._prep(x)
            return self._attach(_IConvFn.apply(x, self.weight, w16, self.stride[0], self.padding[0], part,
                                               _bn_src(x, self.stride[0])), part)
        return super().forward(x)


def conv_entry(x: torch.Tensor, conv_a: nn.Conv2d, conv_b: nn.Conv2d | None):
    """``(conv_a(x), conv_b(x) if conv_b else x)`` - a residual block's first conv and its shortcut -
    as one autograd node (:class:`_EntryFn`: no add kernel for x's two input gradients), when both
    convs run natively; otherwise the plain modules."""
    if (ENTRY and isinstance(conv_a, IConv2d) and native_ok(conv_a, x)
            and (conv_b is None or (isinstance(conv_b, IConv2d) and native_ok(conv_b, x)))):
        wa16, pa = conv_a._prep(x)
        wb16 = pb = None
        if conv_b is not None:
            wb16, pb = conv_b._prep(x)
        ya, yb = _EntryFn.apply(x, conv_a.weight, wa16, conv_a.stride[0], conv_a.padding[0], pa,
                                conv_b.weight if conv_b is not None else None, wb16,
                                conv_b.stride[0] if conv_b is not None else 1,
                                conv_b.padding[0] if conv_b is not None else 0, pb, _bn_src(x, conv_a.stride[0]))
        conv_a._attach(ya, pa)
        if conv_b is not None:
            conv_b._attach(yb, pb)
        return ya, yb
    return conv_a(x), (conv_b(x) if conv_b is not None else x)


def conv2d_reference(x, w, stride, pad):
    """fp32 reference of the same op (tests)."""
    return F.conv2d(x.float(), w.float(), stride=stride, padding=pad)


# BatchNorm folded into the consuming conv (ROCKET_BN_FOLD=1, opt-in): ``conv(relu(bn(z)))`` with the
# BatchNorm's ``relu(z*scale + shift)`` formed in the conv's operand staging (conv.hip PRO), so the
# BatchNorm output and its ReLU mask are never written: forward = statistics finalize + one conv
# launch, backward = the conv dgrad (ReLU mask recomputed from z in its BatchNorm epilogue) + the
# BatchNorm input-gradient pass + the conv wgrad (the same prologue on its gathered z).
# Measured slower (ResNet-50 10,094 vs 10,609 img/s, ResNet-18 70.2k vs 76.2k; profiles/r5_bn_fold_ab.md):
# an implicit GEMM re-stages every input element once per tap and per output-column tile (9 x 1-16 times
# for a 3x3), so the transform costs several times the VALU work of the one bn_apply pass it replaces,
# while the HBM round trip it saves is cheap at 8 TB/s.
BN_FOLD = os.environ.get("ROCKET_BN_FOLD", "0") == "1"
FOLD_MAX_C = 512  # conv.hip kProMaxC: channels of the prologue's LDS scale / shift table
FOLD_HITS = 0  # folded (BatchNorm, conv) pairs run (tests)


class _BNConvFn(torch.autograd.Function):
    """``conv(relu(bn(z)))`` as one node (module docstring of :func:`bn_relu_conv`)."""

    @staticmethod
    def forward(ctx, z, gamma, beta, running_mean, running_var, nbt, momentum: float, eps: float, partials,
                weight, w16, stride: int, pad: int, bnpart):
        from rocket_amd.ops import norm as _norm

        lib = _kernels()
        dev = z.device
        s = _lib.stream_ptr(dev)
        zc = _cl(z, w16.dtype)
        C = zc.shape[1]
        R = zc.numel() // C
        stats = torch.empty(4, C, dtype=torch.float32, device=dev)  # mean, invstd, scale, shift
        ws = torch.empty(int(lib.rk_bn_workspace(R, C)), dtype=torch.float32, device=dev)
        nctr = int(lib.rk_bn_counters(C))
        counters = _lib.Workspace.get(dev).counter_array(f"bn{nctr}", nctr)
        g, b = gamma.detach(), beta.detach()
        args = (_lib.ptr(g), _lib.ptr(b), stats[0].data_ptr(), stats[1].data_ptr(), stats[2].data_ptr(),
                stats[3].data_ptr(), _lib.ptr(running_mean), _lib.ptr(running_var), _lib.ptr(nbt), float(momentum),
                float(eps), ws.data_ptr(), counters, s)
        if partials is not None:
            tp, ntiles, tile_rows = partials
            _lib.check(lib.rk_bn_finalize(tp.data_ptr(), ntiles, tile_rows, R, C, *args), "rk_bn_finalize")
        else:
            _lib.check(lib.rk_bn_stats(_norm._dt(zc), _norm._rows_view(zc).data_ptr(), R, C, *args), "rk_bn_stats")
        lib.rk_conv_set_bn_prologue(stats[2].data_ptr())  # [scale][shift] rows: the [2][C] table
        y = _conv_fwd(zc, w16, stride, pad, bnpart)
        ctx.save_for_backward(zc, w16, stats)
        ctx.params = (gamma, beta, weight)
        ctx.geo = _geo(zc, w16, stride, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        from rocket_amd.ops.lenet import _finish, _grad_targets

        global FOLD_HITS
        FOLD_HITS += 1
        zc, w16, stats = ctx.saved_tensors
        gamma, beta, weight = ctx.params
        N, C, H, W, Co, R, S, stride, pad, OH, OW = ctx.geo
        dev = zc.device
        s = _lib.stream_ptr(dev)
        lib = _kernels()
        dyc = _cl(dy, zc.dtype)
        rows = N * H * W
        # dX' = relu-mask(z) * (dY (*) W^T), with the BatchNorm backward's per-tile reductions
        dxp = torch.empty_like(zc)
        ntiles = -(-rows // 128)
        part = torch.empty(ntiles * 2 * C, dtype=torch.float32, device=dev)
        lib.rk_conv_set_bn_prologue(stats[2].data_ptr())
        _lib.check(lib.rk_conv_dgrad_bn(_dt(dyc), dyc.data_ptr(), w16.data_ptr(), dxp.data_ptr(), 0, N, H, W, C, Co, R, S,
                                        pad, zc.data_ptr(), None, stats[0].data_ptr(), stats[1].data_ptr(),
                                        part.data_ptr(), s), "rk_conv_dgrad_bn(fold)")
        # dz from dX' and the partials (BatchNorm input gradient; dgamma / dbeta into their grads)
        bufs, direct = _grad_targets([gamma, beta], dev)
        dz = torch.empty_like(zc)
        ws = torch.empty(int(lib.rk_bn_workspace(rows, C)), dtype=torch.float32, device=dev)
        coef = torch.empty(3 * C, dtype=torch.float32, device=dev)
        nctr = int(lib.rk_bn_counters(C))
        counters = _lib.Workspace.get(dev).counter_array(f"bn{nctr}", nctr)
        _lib.check(lib.rk_bn_bwd_partials(_dt(zc), _dt(dxp), dxp.data_ptr(), zc.data_ptr(), part.data_ptr(), ntiles,
                                          rows, C, stats[0].data_ptr(), stats[1].data_ptr(), stats[2].data_ptr(),
                                          bufs[0].data_ptr(), bufs[1].data_ptr(), dz.data_ptr(), None,
                                          ws.data_ptr(), coef.data_ptr(), counters, s), "rk_bn_bwd_partials(fold)")
        gg, gb = _finish([gamma, beta], bufs, direct)
        # the conv's weight gradient over relu(z*scale + shift), formed by the same prologue
        dw = None
        if ctx.needs_input_grad[9]:
            lib.rk_conv_set_bn_prologue(stats[2].data_ptr())
            dw = _conv_wgrad(dyc, zc, weight, ctx.geo)
        return dz, gg, gb, None, None, None, None, None, None, dw, None, None, None, None


def fold_ok(bn: nn.Module, conv: nn.Module, z: torch.Tensor) -> bool:
    """Whether ``conv(bn(z))`` runs as :class:`_BNConvFn`: a training BatchNorm(+ReLU) with
    affine parameters and running statistics feeding a stride-1 native conv, over <= 512 16-bit
    channels-last channels."""
    from rocket_amd.ops.norm import BatchNormAct2d

    return (BN_FOLD and isinstance(bn, BatchNormAct2d) and isinstance(conv, IConv2d) and bn.training and bn.relu
            and not bn.maxpool and bn.affine and bn.track_running_stats and bn.momentum is not None
            and z.dim() == 4 and z.dtype in _LOWP and z.dtype == torch.get_autocast_dtype("cuda")
            and z.is_contiguous(memory_format=torch.channels_last) and z.shape[1] <= FOLD_MAX_C
            and bn._fused_ok(z, None) and native_ok(conv, z) and conv.stride[0] == 1
            and conv.out_channels % 64 == 0)


def bn_relu_conv(bn: nn.Module, conv: nn.Module, z: torch.Tensor) -> torch.Tensor:
    """``conv(bn(z))`` for a ReLU BatchNorm feeding a conv: folded into the conv (:class:`_BNConvFn`)
    when :func:`fold_ok`, else the two modules."""
    if not fold_ok(bn, conv, z):
        return conv(bn(z))
    partials = getattr(z, "_rocket_bn_partials", None)
    if partials is not None and partials[0].numel() != 2 * partials[1] * z.shape[1]:
        partials = None
    w16, part = conv._prep(z)
    y = _BNConvFn.apply(z, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.num_batches_tracked,
                        bn.momentum, bn.eps, partials, conv.weight, w16, conv.stride[0], conv.padding[0], part)
    return conv._attach(y, part)
