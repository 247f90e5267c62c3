"""Fused normalisation ops (``native/kernels/norm.hip``).

* :class:`BatchNormAct2d` — ``nn.BatchNorm2d`` whose training forward is two HIP
  launches over channels-last activations (statistics with an in-launch grid
  reduction + running-stat update, then one fused ``x*a + b (+ residual) (ReLU)``
  pass) and whose backward is two launches (per-channel reductions, then the
  input gradient and the residual gradient).  ResNet blocks call
  ``bn(x, residual=identity, relu=True)`` so the block epilogue
  ``relu(bn(conv(x)) + identity)`` is one pass over HBM.
* :class:`FusedLayerNorm` — ``nn.LayerNorm`` with a one-wave-per-row forward that
  can emit bf16 directly for the following GEMM, and a backward that fuses the
  dgamma/dbeta column reduction (block partials + last block).

Parameter gradients accumulate straight into persistent ``.grad`` buffers when the
engine provides them (graph capture), otherwise they are returned to autograd.
On CPU (or for layouts the kernels do not cover) the modules run the PyTorch
reference implementation; on a HIP device the kernels are mandatory.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

import os

import rocket_amd.ops as _ops
from rocket_amd.ops import _lib
from rocket_amd.ops.lenet import _finish, _grad_targets
from rocket_amd.ops.linear import _direct


# ROCKET_BN_BWD_FUSE (default 1): a BatchNorm whose output feeds a stride-1 native conv leaves its
# backward reduction to that conv's LDS-staged dgrad epilogue (conv.hip store_tile_lds<BNB>), which
# already holds dy' on chip: the bn_bwd_reduce pass over (dy, x, mask) disappears for 44 of ResNet-50's
# 53 BatchNorms (9,625 -> 9,900 img/s; profiles/r2_bn_bwd_fusion_ab.md).  0: a separate reduction pass.
BWD_FUSE = os.environ.get("ROCKET_BN_BWD_FUSE", "1") != "0"


def _dt(t: torch.Tensor) -> int:
    return _lib.dtype_code(t)


def _rows_view(x: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels-last (or [N, C]) -> [R, C] view, no copy."""
    if x.dim() == 4:
        return x.permute(0, 2, 3, 1).reshape(-1, x.shape[1])
    return x.reshape(-1, x.shape[-1])


def _channels_last(x: torch.Tensor) -> torch.Tensor:
    if x.dim() == 4:
        return x.contiguous(memory_format=torch.channels_last)
    return x.contiguous()


LINK_HITS = 0  # BatchNorm backwards that used a conv dgrad epilogue's reductions (tests)


class BwdLink:
    """Hand-off between a fused BatchNorm and the conv that consumes its output.

    ``src`` = (BatchNorm input, ReLU mask, stats), set by the BatchNorm forward; ``done`` =
    (dy data_ptr, dy version, partials, ntiles), set by the consuming stride-1 conv's dgrad
    (iconv.py) when its epilogue already did this BatchNorm's backward reductions, and consumed by
    the BatchNorm's backward when its incoming gradient is exactly that tensor, unmodified.  The
    link lives on the autograd graph (the BatchNorm's ctx and its output), so a pruned or partial
    backward leaves nothing behind that a later step could pick up."""

    __slots__ = ("src", "done")

    def __init__(self):
        self.src = None
        self.done = None


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, nbt, momentum, eps, relu, partials,
                pool=False, box=None):
        lib = _lib.kernels()
        x = _channels_last(x)
        C = x.shape[1]
        xr = _rows_view(x)
        R = xr.shape[0]
        dev = x.device
        out_dtype = residual.dtype if residual is not None else x.dtype
        y = torch.empty_like(x, dtype=out_dtype, memory_format=torch.channels_last if x.dim() == 4 else torch.contiguous_format)
        stats = torch.empty(4, C, dtype=torch.float32, device=dev)  # mean, invstd, scale, shift
        ws = torch.empty(int(lib.rk_bn_workspace(R, C)), dtype=torch.float32, device=dev)
        nctr = int(lib.rk_bn_counters(C))
        counters = _lib.Workspace.get(dev).counter_array(f"bn{nctr}", nctr)
        w = weight.detach() if weight is not None else None
        b = bias.detach() if bias is not None else None
        s = _lib.stream_ptr(dev)
        if partials is not None:  # the producing conv's epilogue already reduced its output tiles
            tp, ntiles, tile_rows = partials
            _lib.check(lib.rk_bn_finalize(tp.data_ptr(), ntiles, tile_rows, R, C, _lib.ptr(w), _lib.ptr(b),
                                          stats[0].data_ptr(), stats[1].data_ptr(), stats[2].data_ptr(),
                                          stats[3].data_ptr(), _lib.ptr(running_mean), _lib.ptr(running_var),
                                          _lib.ptr(nbt), float(momentum), float(eps), ws.data_ptr(), counters, s),
                       "rk_bn_finalize")
        else:
            _lib.check(lib.rk_bn_stats(_dt(x), xr.data_ptr(), R, C, _lib.ptr(w), _lib.ptr(b), stats[0].data_ptr(),
                                       stats[1].data_ptr(), stats[2].data_ptr(), stats[3].data_ptr(),
                                       _lib.ptr(running_mean), _lib.ptr(running_var), _lib.ptr(nbt), float(momentum),
                                       float(eps), ws.data_ptr(), counters, s), "rk_bn_stats")
        if pool:  # stem: relu(bn(x)) max-pooled 3x3/s2/p1 in the same pass (codes instead of a mask)
            N, _, H, W = x.shape
            OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
            y = torch.empty((N, C, OH, OW), dtype=x.dtype, device=dev, memory_format=torch.channels_last)
            code = torch.empty((N, OH, OW, C), dtype=torch.uint8, device=dev)
            _lib.check(lib.rk_bn_relu_maxpool(_dt(x), x.data_ptr(), stats[2].data_ptr(), stats[3].data_ptr(),
                                              y.data_ptr(), code.data_ptr(), N, H, W, C, OH, OW, s),
                       "rk_bn_relu_maxpool")
            ctx.params = (weight, bias)
            ctx.relu, ctx.has_res, ctx.out_dtype, ctx.pool = True, False, x.dtype, True
            ctx.link = None
            ctx.save_for_backward(x, code, stats)
            return y
        res = None
        if residual is not None:
            res = _channels_last(residual)
        # fused ReLU: a 1-bit [y > 0] mask (R*C/8 bytes) is all the backward needs of y
        mask = torch.empty(R * C // 8, dtype=torch.uint8, device=dev) if relu else None
        _lib.check(lib.rk_bn_apply(_dt(x), _dt(y), xr.data_ptr(), _lib.ptr(_rows_view(res)) if res is not None else None,
                                   stats[2].data_ptr(), stats[3].data_ptr(), _rows_view(y).data_ptr(), _lib.ptr(mask),
                                   R, C, int(relu), s), "rk_bn_apply")
        ctx.params = (weight, bias)
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.out_dtype = out_dtype
        ctx.pool = False
        ctx.save_for_backward(x, mask, stats)
        ctx.link = box
        if box is not None:  # what a consuming conv's dgrad epilogue needs to do this backward's reduction
            box.src = (x, mask, stats)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib.kernels()
        x, mask, stats = ctx.saved_tensors
        weight, bias = ctx.params
        C = x.shape[1]
        dev = x.device
        dy = _channels_last(dy if dy.dtype == ctx.out_dtype else dy.to(ctx.out_dtype))
        if ctx.pool:  # route the pooled gradient through the codes: the ReLU-masked d(bn output)
            N, _, H, W = x.shape
            OH, OW = dy.shape[2], dy.shape[3]
            dfull = torch.empty_like(x)
            _lib.check(lib.rk_maxpool_bwd(_dt(x), dy.data_ptr(), mask.data_ptr(), dfull.data_ptr(), N, H, W, C, OH, OW,
                                          _lib.stream_ptr(dev)), "rk_maxpool_bwd")
            dy, mask = dfull, None
        link, ctx.link = ctx.link, None
        done = None
        if link is not None:
            done, link.done, link.src = link.done, None, None
        xr, dyr = _rows_view(x), _rows_view(dy)
        R = xr.shape[0]
        params = [p for p in (weight, bias) if p is not None]
        bufs, direct = _grad_targets(params, dev) if params else ([], False)
        dgamma = bufs[0] if weight is not None else None
        dbeta = bufs[-1] if bias is not None else None
        dx = torch.empty_like(x)
        ws = torch.empty(int(lib.rk_bn_workspace(R, C)), dtype=torch.float32, device=dev)
        coef = torch.empty(3 * C, dtype=torch.float32, device=dev)
        nctr = int(lib.rk_bn_counters(C))
        counters = _lib.Workspace.get(dev).counter_array(f"bn{nctr}", nctr)
        if done is not None and done[0] == dy.data_ptr() and done[1] == dy._version:
            global LINK_HITS
            LINK_HITS += 1
            # dy is the masked gradient the conv dgrad epilogue stored, its reductions are in done[2];
            # the residual's gradient IS that masked dy: handed on as is, not copied
            dres = dy if ctx.has_res else None
            _lib.check(lib.rk_bn_bwd_partials(_dt(x), _dt(dy), dyr.data_ptr(), xr.data_ptr(), done[2].data_ptr(),
                                              done[3], R, C, stats[0].data_ptr(), stats[1].data_ptr(),
                                              stats[2].data_ptr(), _lib.ptr(dgamma), _lib.ptr(dbeta),
                                              _rows_view(dx).data_ptr(), None, ws.data_ptr(),
                                              coef.data_ptr(), counters, _lib.stream_ptr(dev)), "rk_bn_bwd_partials")
        else:
            dres = torch.empty_like(dy) if ctx.has_res else None
            _lib.check(lib.rk_bn_bwd(_dt(x), _dt(dy), dyr.data_ptr(), xr.data_ptr(), _lib.ptr(mask), R, C,
                                     stats[0].data_ptr(), stats[1].data_ptr(), stats[2].data_ptr(), _lib.ptr(dgamma),
                                     _lib.ptr(dbeta), _rows_view(dx).data_ptr(),
                                     _rows_view(dres).data_ptr() if dres is not None else None, ws.data_ptr(),
                                     coef.data_ptr(), counters, _lib.stream_ptr(dev)), "rk_bn_bwd")
        g = _finish(params, bufs, direct) if params else []
        gw = g[0] if weight is not None else None
        gb = g[-1] if bias is not None else None
        return dx, gw, gb, dres, None, None, None, None, None, None, None, None, None


class BatchNormAct2d(nn.BatchNorm2d):
    """``BatchNorm2d`` with optional fused residual add and ReLU: ``relu?(bn(x) + residual?)``."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True, relu=False,
                 maxpool=False, **kw):
        super().__init__(num_features, eps=eps, momentum=momentum, affine=affine,
                         track_running_stats=track_running_stats, **kw)
        self.relu = relu or maxpool
        # ``maxpool``: the ImageNet ResNet stem's max_pool2d(3, 2, 1) after the ReLU, fused into the
        # same pass (the full-resolution activation is never written)
        self.maxpool = maxpool

    def _fused_ok(self, x, residual) -> bool:
        return (
            _ops.fused_enabled() and x.is_cuda and self.training and x.dim() in (2, 4) and x.shape[1] % 8 == 0 and x.shape[1] <= 2048
            and x.dtype in (torch.float32, torch.bfloat16, torch.float16) and self.momentum is not None
            and (residual is None or residual.shape == x.shape)
            and (not self.maxpool or (residual is None and x.dim() == 4 and 256 % (x.shape[1] // 8) == 0))
        )

    def forward(self, x, residual=None):
        if self._fused_ok(x, residual):
            if residual is not None and residual.dtype != x.dtype:
                residual = residual.to(x.dtype)
            partials = getattr(x, "_rocket_bn_partials", None)
            if partials is not None and not (x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)
                                             and partials[0].numel() == 2 * partials[1] * x.shape[1]):
                partials = None
            box = (BwdLink() if (BWD_FUSE and not self.maxpool and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float16))
                   else None)
            y = _BNAct.apply(x, self.weight, self.bias, residual,
                             self.running_mean if self.track_running_stats else None,
                             self.running_var if self.track_running_stats else None,
                             self.num_batches_tracked if self.track_running_stats else None,
                             self.momentum, self.eps, self.relu, partials, self.maxpool, box)
            if box is not None and box.src is not None:
                y._rocket_bn_bwd_src = box  # for a consuming conv's dgrad (BwdLink)
            return y
        if x.is_cuda and self.training and _ops.fused_enabled():
            _lib.kernels()  # a HIP device without the native library is an error, not a fallback
        y = super().forward(x)
        if residual is not None:
            y = y + residual
        y = F.relu(y) if self.relu else y
        return F.max_pool2d(y, 3, 2, 1) if self.maxpool else y


class _LN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, out_dtype):
        lib = _lib.kernels()
        x = x.contiguous()
        C = x.shape[-1]
        rows = x.numel() // C
        dev = x.device
        y = torch.empty(x.shape, dtype=out_dtype, device=dev)
        mean = torch.empty(rows, dtype=torch.float32, device=dev)
        rstd = torch.empty(rows, dtype=torch.float32, device=dev)
        w = weight.detach() if weight is not None else None
        b = bias.detach() if bias is not None else None
        _lib.check(lib.rk_ln_fwd(_dt(x), _dt(y), x.data_ptr(), None, None, _lib.ptr(w), _lib.ptr(b), y.data_ptr(),
                                 mean.data_ptr(), rstd.data_ptr(), rows, C, float(eps), _lib.stream_ptr(dev)),
                   "rk_ln_fwd")
        ctx.params = (weight, bias)
        ctx.save_for_backward(x, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib.kernels()
        x, mean, rstd = ctx.saved_tensors
        weight, bias = ctx.params
        dy = dy.contiguous()
        C = x.shape[-1]
        rows = x.numel() // C
        dev = x.device
        params = [p for p in (weight, bias) if p is not None]
        bufs, direct = _grad_targets(params, dev) if params else ([], False)
        dgamma = bufs[0] if weight is not None else None
        dbeta = bufs[-1] if bias is not None else None
        dx = torch.empty_like(x)
        ws = torch.empty(int(lib.rk_ln_workspace(rows, C)), dtype=torch.float32, device=dev)
        counter = _lib.Workspace.get(dev).counter("ln_bwd")
        w = weight.detach() if weight is not None else None
        _lib.check(lib.rk_ln_bwd(_dt(x), _dt(dy), dy.data_ptr(), x.data_ptr(), _lib.ptr(w), mean.data_ptr(),
                                 rstd.data_ptr(), dx.data_ptr(), None, None, _lib.ptr(dgamma), _lib.ptr(dbeta), None,
                                 None, rows, C, ws.data_ptr(), counter, _lib.stream_ptr(dev)), "rk_ln_bwd")
        g = _finish(params, bufs, direct) if params else []
        gw = g[0] if weight is not None else None
        gb = g[-1] if bias is not None else None
        return dx, gw, gb, None, None


class BiasLink:
    """Hand-off between a linear layer whose output ``r`` feeds ONLY an add-LayerNorm and that
    LayerNorm: the LN backward already streams dr (= the linear's output gradient), so it also
    forms dr's column sums — the linear's bias gradient — into ``db``; the linear's backward uses
    them when its incoming gradient is exactly that dr, unmodified (:meth:`take`), instead of a column-sum pass
    over its output gradient.  Lives on the autograd graph (both ctxs), like :class:`BwdLink`."""

    __slots__ = ("bias", "db", "dr", "dr_ver", "applied")

    def __init__(self, bias):
        self.bias = bias
        self.db = None
        self.dr = None  # the LN's dr (held: its storage cannot be recycled under another tensor)
        self.dr_ver = None
        self.applied = False  # the LN kernel already added db into the persistent bias.grad

    def take(self, dy: torch.Tensor):
        """The finished bias gradient for incoming gradient ``dy``, or None (compute it yourself).

        ``dy`` must BE the LN's dr, unmodified: same storage, same shape, and the same version
        counter value.  When the linear's output also feeds another op, autograd's input buffer may
        sum that op's gradient into dr in place before handing it over (same pointer, bumped
        ``_version``): then the link's column sums miss that contribution and are refused."""
        db, dr, ver, applied = self.db, self.dr, self.dr_ver, self.applied
        self.db = self.dr = self.dr_ver = None
        self.applied = False
        ok = (db is not None and dr is not None and dy.data_ptr() == dr.data_ptr()
              and dy.numel() == dr.numel() and dy._version == ver)
        if applied and not ok:
            self.bias.grad.sub_(db)  # refused: back out what the LN kernel already added
        return db if ok else None


def attach_bias_link(y: torch.Tensor, bias) -> "BiasLink | None":
    """Tag a linear layer's output with a :class:`BiasLink` (bias that needs a gradient only)."""
    if bias is None or not bias.requires_grad or not torch.is_grad_enabled():
        return None
    link = BiasLink(bias)
    y._rocket_bias_link = link
    return link


class _AddLN(torch.autograd.Function):
    """(s, y) = (x + r, LayerNorm(x + r)): the pre-norm transformer's residual add fused into its LN.

    Backward: dx = LN_bwd(dy) + ds (the residual stream's own gradient) and dr = dx, both written
    by the same kernel — no separate add / cast / gradient-accumulation passes; with a
    :class:`BiasLink` on r, the same kernel also sums dr's columns (r's producer's bias gradient)."""

    @staticmethod
    def forward(ctx, x, r, weight, bias, eps, out_dtype, link=None):
        lib = _lib.kernels()
        x = x.contiguous()
        r = r.contiguous()
        C = x.shape[-1]
        rows = x.numel() // C
        dev = x.device
        ssum = torch.empty_like(x)
        y = torch.empty(x.shape, dtype=out_dtype, device=dev)
        mean = torch.empty(rows, dtype=torch.float32, device=dev)
        rstd = torch.empty(rows, dtype=torch.float32, device=dev)
        w = weight.detach() if weight is not None else None
        b = bias.detach() if bias is not None else None
        _lib.check(lib.rk_ln_fwd(_dt(x), _dt(y), x.data_ptr(), r.data_ptr(), ssum.data_ptr(), _lib.ptr(w),
                                 _lib.ptr(b), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), rows, C, float(eps),
                                 _lib.stream_ptr(dev)), "rk_ln_fwd(add)")
        ctx.params = (weight, bias)
        ctx.r_dtype = r.dtype
        ctx.link = link
        ctx.save_for_backward(ssum, mean, rstd)
        return ssum, y

    @staticmethod
    def backward(ctx, ds, dy):
        lib = _lib.kernels()
        ssum, mean, rstd = ctx.saved_tensors
        weight, bias = ctx.params
        C = ssum.shape[-1]
        rows = ssum.numel() // C
        dev = ssum.device
        if dy is None:
            dy = torch.zeros(ssum.shape, dtype=ctx.r_dtype, device=dev)
        dy = dy.contiguous()
        if dy.dtype != ctx.r_dtype:
            dy = dy.to(ctx.r_dtype)
        ds = ds.contiguous() if ds is not None else None
        params = [p for p in (weight, bias) if p is not None]
        bufs, direct = _grad_targets(params, dev) if params else ([], False)
        dgamma = bufs[0] if weight is not None else None
        dbeta = bufs[-1] if bias is not None else None
        dx = torch.empty_like(ssum)
        dr = torch.empty(ssum.shape, dtype=ctx.r_dtype, device=dev)
        ws = torch.empty(int(lib.rk_ln_workspace(rows, C)), dtype=torch.float32, device=dev)
        counter = _lib.Workspace.get(dev).counter("ln_bwd")
        w = weight.detach() if weight is not None else None
        link, ctx.link = ctx.link, None
        rsum = torch.empty(C, dtype=torch.float32, device=dev) if link is not None else None  # written by the kernel
        # a persistent fp32 bias.grad takes the sums in the same launch (the linear then only
        # confirms the hand-off, or backs the sums out again if it refuses it: BiasLink.take)
        acc = (link.bias.grad if link is not None and _direct(link.bias) and link.bias.grad.dtype == torch.float32
               else None)
        _lib.check(lib.rk_ln_bwd(_dt(ssum), _dt(dy), dy.data_ptr(), ssum.data_ptr(), _lib.ptr(w), mean.data_ptr(),
                                 rstd.data_ptr(), dx.data_ptr(), _lib.ptr(ds), dr.data_ptr(), _lib.ptr(dgamma),
                                 _lib.ptr(dbeta), _lib.ptr(rsum), _lib.ptr(acc), rows, C, ws.data_ptr(), counter,
                                 _lib.stream_ptr(dev)), "rk_ln_bwd(add)")
        if link is not None:
            link.db, link.dr, link.dr_ver, link.applied = rsum, dr, dr._version, acc is not None
        g = _finish(params, bufs, direct) if params else []
        gw = g[0] if weight is not None else None
        gb = g[-1] if bias is not None else None
        return dx, dr, gw, gb, None, None, None


def _ln_out_dtype(x: torch.Tensor) -> torch.dtype:
    """LayerNorm output dtype: the autocast compute dtype (bf16 or fp16: the output feeds a GEMM),
    else the input's 16-bit dtype, else fp32."""
    if torch.is_autocast_enabled("cuda"):
        return torch.get_autocast_dtype("cuda")
    return x.dtype


class FusedLayerNorm(nn.LayerNorm):
    """``LayerNorm`` over the last dim; under autocast the output is in the autocast dtype (it
    feeds a GEMM).

    ``add_forward(x, r)`` returns ``(x + r, LN(x + r))`` with the residual add fused (pre-norm
    transformer blocks); ``r=None`` is a plain LN that passes ``x`` through.
    """

    def add_forward(self, x, r=None):
        if r is None:
            return x, self(x)
        C = x.shape[-1]
        if (_ops.fused_enabled() and x.is_cuda and len(self.normalized_shape) == 1 and C % 4 == 0 and C <= 4096
                and x.dtype in (torch.float32, torch.bfloat16, torch.float16) and r.shape == x.shape):
            out_dtype = _ln_out_dtype(x)
            if {x.dtype, out_dtype} == {torch.bfloat16, torch.float16}:
                x = x.to(out_dtype)
            link = getattr(r, "_rocket_bias_link", None)
            if r.dtype != out_dtype:
                r, link = r.to(out_dtype), None  # the producer then sees a different gradient tensor
            return _AddLN.apply(x, r, self.weight, self.bias, self.eps, out_dtype, link)
        s = x + r
        return s, self(s)

    def forward(self, x):
        C = x.shape[-1]
        if (_ops.fused_enabled() and x.is_cuda and len(self.normalized_shape) == 1 and C % 4 == 0 and C <= 4096
                and x.dtype in (torch.float32, torch.bfloat16, torch.float16)):
            out_dtype = _ln_out_dtype(x)
            if {x.dtype, out_dtype} == {torch.bfloat16, torch.float16}:
                x = x.to(out_dtype)
            return _LN.apply(x, self.weight, self.bias, self.eps, out_dtype)
        if x.is_cuda and _ops.fused_enabled():
            _lib.kernels()
        return super().forward(x)
