"""Fused linear layer on the MFMA GEMM kernel (``native/kernels/gemm.hip``).

``linear(x, weight, bias, activation)`` = ``act(x @ weight.T + bias)`` with
bf16 MFMA math and f32 accumulation.  ``weight``/``bias`` are the fp32 master
parameters (converted while staging, so no per-step cast kernels).

Backward (one launch each):

* dgrad  ``dx = (dy ⊙ act'(·)) @ W``        — the activation mask is applied
  while staging ``dy`` (no threshold_backward kernel);
* wgrad  ``dW = (dy ⊙ act'(·))ᵀ @ x``       — split-K over the batch with f32
  atomics when the tile grid is small, bias gradient fused as the row sums of
  the staged ``dyᵀ`` tile.

When a parameter owns a persistent gradient buffer (``param._rocket_direct_grad``,
set by the engine for flat gradient buckets / graph capture) the kernels
accumulate straight into ``param.grad`` and notify the data-parallel reducer;
otherwise they return fresh gradient tensors to autograd.
"""

from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from rocket_amd.ops import _lib

_ACT = {None: 0, "none": 0, "relu": 1, "gelu": 2}


def _direct(p: torch.Tensor | None) -> bool:
    return p is not None and getattr(p, "_rocket_direct_grad", False) and p.grad is not None


def _autocast_on() -> bool:
    try:
        return torch.is_autocast_enabled("cuda")
    except TypeError:  # older signature
        return torch.is_autocast_enabled()


def native_route() -> bool:
    """bf16/fp16 autocast is on and the fused kernels are enabled (``rocket_amd.ops.set_fused``):
    the model-level layers (IConv2d, MLinear, MMlp, LibLinear, PatchEmbed) take their native paths;
    otherwise they are exactly the stock torch modules (the ``--impl torch`` A/B and parity runs)."""
    from rocket_amd.ops import fused_enabled

    return fused_enabled() and _autocast_on()


def grad_ready(p: torch.Tensor) -> None:
    hook = getattr(p, "_rocket_grad_hook", None)
    if hook is not None:
        hook(p)


def gemm(a, b, c, *, a_trans=False, b_trans=False, M, N, K, lda, ldb, ldc, mask=None, mask_mode=0, ld_mask=0,
         bias=None, act=0, accumulate=False, c_pre=None, rowsum=None, splitk=1, cfg=0):
    lib = _lib.kernels()
    _lib.check(
        lib.rk_gemm(a.data_ptr(), _lib.dtype_code(a), lda, int(a_trans), _lib.ptr(mask),
                    _lib.dtype_code(mask) if mask is not None else 0, ld_mask, mask_mode, b.data_ptr(),
                    _lib.dtype_code(b), ldb, int(b_trans), c.data_ptr(), _lib.dtype_code(c), ldc, _lib.ptr(c_pre),
                    _lib.ptr(bias), act, int(accumulate), _lib.ptr(rowsum), M, N, K, splitk, cfg,
                    _lib.stream_ptr(c.device)),
        "rk_gemm",
    )


def _tiles(M, N, t):
    return ((M + t - 1) // t) * ((N + t - 1) // t)


def _cfg(M, N):
    return 0 if _tiles(M, N, 64) >= 128 else 1


def _splitk(M, N, K):
    tiles = _tiles(M, N, 64)
    if tiles >= 128 or K < 256:
        return 1
    return int(max(1, min(K // 128, (256 + tiles - 1) // tiles)))


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, act: int, out_dtype):
        shape = x.shape
        K = shape[-1]
        x2 = x.reshape(-1, K)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        if x2.dtype not in (torch.float32, torch.bfloat16):
            x2 = x2.float()
        M, N = x2.shape[0], weight.shape[0]
        w = weight if weight.is_contiguous() else weight.contiguous()
        y = torch.empty(M, N, dtype=out_dtype, device=x.device)
        pre = torch.empty_like(y) if act == 2 else None
        gemm(x2, w, y, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, bias=bias, act=act, c_pre=pre, cfg=_cfg(M, N))
        ctx.act = act
        ctx.params = (weight, bias)
        ctx.shape = shape
        ctx.x_dtype = x2.dtype
        mask = y if act == 1 else pre
        ctx.save_for_backward(x2, w, bias if bias is not None else None, mask)
        return y.reshape(*shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w, bias, mask = ctx.saved_tensors
        act = ctx.act
        M, K = x2.shape
        N = w.shape[0]
        dy2 = dy.reshape(M, N)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        if dy2.dtype not in (torch.float32, torch.bfloat16):
            dy2 = dy2.float()
        mmode = act if mask is not None else 0
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, dtype=ctx.x_dtype, device=dy.device)
            gemm(dy2, w, dx, b_trans=True, M=M, N=K, K=N, lda=N, ldb=K, ldc=K, mask=mask, mask_mode=mmode, ld_mask=N,
                 cfg=_cfg(M, K))
            dx = dx.reshape(ctx.shape)
        need_w = ctx.needs_input_grad[1]
        need_b = bias is not None and ctx.needs_input_grad[2]
        if need_w or need_b:
            wparam = ctx.params
            direct = _direct(wparam[0]) and (not need_b or _direct(wparam[1]))
            sk = _splitk(N, K, M)
            if direct:
                wp, bp = wparam
                gemm(dy2, x2, wp.grad, a_trans=True, b_trans=True, M=N, N=K, K=M, lda=N, ldb=K, ldc=K, mask=mask,
                     mask_mode=mmode, ld_mask=N, accumulate=True, rowsum=bp.grad if need_b else None,
                     splitk=sk, cfg=0)
                grad_ready(wp)
                if need_b:
                    grad_ready(bp)
            else:
                dw = torch.zeros(N, K, dtype=torch.float32, device=dy.device) if sk > 1 else \
                    torch.empty(N, K, dtype=torch.float32, device=dy.device)
                db = torch.zeros(N, dtype=torch.float32, device=dy.device) if need_b else None
                gemm(dy2, x2, dw, a_trans=True, b_trans=True, M=N, N=K, K=M, lda=N, ldb=K, ldc=K, mask=mask,
                     mask_mode=mmode, ld_mask=N, accumulate=False, rowsum=db, splitk=sk, cfg=0)
                dw = dw if need_w else None
        return dx, dw, db, None, None


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None, activation: str | None = None,
           out_dtype: torch.dtype | None = None) -> torch.Tensor:
    act = _ACT[activation]
    if x.device.type != "cuda":
        y = F.linear(x, weight, bias)
        if act == 1:
            y = F.relu(y)
        elif act == 2:
            y = F.gelu(y)
        return y
    if out_dtype is None:
        out_dtype = torch.bfloat16 if (_autocast_on() or x.dtype == torch.bfloat16) else torch.float32
    if weight.dtype != torch.float32 and weight.dtype != torch.bfloat16:
        weight = weight.float()
    if x.dtype != torch.float32 and x.dtype != torch.bfloat16:  # the kernel reads bf16 / f32 operands
        x = x.float()
    return _Linear.apply(x, weight, bias, act, out_dtype)


class FusedLinear(torch.nn.Linear):
    """``nn.Linear`` (same parameters / state_dict keys) with an optional fused activation."""

    def __init__(self, in_features, out_features, bias=True, activation: str | None = None, device=None, dtype=None):
        super().__init__(in_features, out_features, bias=bias, device=device, dtype=dtype)
        self.activation = activation

    def forward(self, x):
        return linear(x, self.weight, self.bias, self.activation)


def _wgrad_splits(M: int, N: int, K: int) -> int:
    """K-split of a weight-gradient GEMM dW[N, K] = dY^T X (reduction over M rows): the output
    has few tiles (ViT: 18-144 tiles of 128x128 for 256 CUs), so the rows are cut into S chunks
    computed as ONE strided-batched GEMM and summed in fp32.  ``ROCKET_WGRAD_SPLITK=0`` disables."""
    if os.environ.get("ROCKET_WGRAD_SPLITK", "1") == "0" or M < 4096:
        return 1
    tiles = ((N + 127) // 128) * ((K + 127) // 128)
    s = 1
    while s < 16 and tiles * s * 2 <= 640 and M % (2 * s) == 0 and M // (2 * s) >= 1024:
        s *= 2
    return s


def _wgrad(dy2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """fp32 dW = dy2^T @ x2 (bf16 operands, fp32 accumulation)."""
    M, N = dy2.shape
    K = x2.shape[1]
    s = _wgrad_splits(M, N, K)
    if s == 1:
        return (dy2.t() @ x2).float()
    part = torch.bmm(dy2.view(s, M // s, N).transpose(1, 2), x2.view(s, M // s, K))  # [s, N, K]
    return part.sum(0, dtype=torch.float32)


# ROCKET_WGRAD_F32=1: the split-K partial products come out of the library GEMM in fp32 (bmm with
# out_dtype) instead of bf16 - exact partials for twice the combine traffic.
_WGRAD_F32 = os.environ.get("ROCKET_WGRAD_F32", "0") == "1"


def wgrad_into(dy2: torch.Tensor, x2: torch.Tensor, target: torch.Tensor, accumulate: bool) -> None:
    """target (+)= dy2^T @ x2 in fp32 (target: contiguous fp32 [N, K], e.g. a persistent
    ``weight.grad``): the library GEMM's split-K partial products are summed (and accumulated)
    by ONE ``rk_slab_acc`` launch - no reduction temporary, no separate accumulation add."""
    M, N = dy2.shape
    K = x2.shape[1]
    s = _wgrad_splits(M, N, K)
    if s == 1:
        part = torch.mm(dy2.t(), x2, out_dtype=torch.float32) if _WGRAD_F32 else dy2.t() @ x2
    else:
        a, b = dy2.view(s, M // s, N).transpose(1, 2), x2.view(s, M // s, K)
        part = torch.bmm(a, b, out_dtype=torch.float32) if _WGRAD_F32 else torch.bmm(a, b)
    part = part.contiguous()
    if (N * K) % 8 or target.data_ptr() % 16 or part.data_ptr() % 16:
        # the combine kernel moves 8 floats per thread from 16-byte aligned rows; a small head's grad
        # packed into a flat gradient bucket at an odd offset is summed here instead
        red = (part if s == 1 else part.sum(0)).float().view_as(target)
        if accumulate:
            target.add_(red)
        else:
            target.copy_(red)
        return
    _lib.check(_lib.kernels().rk_slab_acc(part.data_ptr(), _lib.dtype_code(part), s, N * K, target.data_ptr(),
                                          int(accumulate), _lib.stream_ptr(dy2.device)), "rk_slab_acc")


def bias_grad_into(dy2: torch.Tensor, target: torch.Tensor) -> None:
    """target += column sums of dy2 [M, N] (fp32 target, e.g. a persistent ``bias.grad``)."""
    M, N = dy2.shape
    if N % 8:  # the column-sum kernel reads 8 channels per thread; small heads (10 classes) reduce here
        target.add_(dy2.float().sum(0))
        return
    lib = _lib.kernels()
    ws = torch.empty(int(lib.rk_bn_workspace(M, N)), dtype=torch.float32, device=dy2.device)
    nctr = int(lib.rk_bn_counters(N))
    _lib.check(lib.rk_colsum_acc(_lib.dtype_code(dy2), dy2.data_ptr(), M, N, target.data_ptr(), ws.data_ptr(),
                                 _lib.Workspace.get(dy2.device).counter_array(f"bn{nctr}", nctr),
                                 _lib.stream_ptr(dy2.device)), "rk_colsum_acc")


class _LibLinear(torch.autograd.Function):
    """``x @ W^T + b`` on the library GEMM (hipBLASLt, bf16 under autocast) whose bias gradient is
    the column-sum kernel (``rk_colsum_acc``) instead of a generic reduction over the rows of
    d(out); accumulated straight into a persistent ``bias.grad`` when the engine provides one."""

    @staticmethod
    def forward(ctx, x, weight, bias, cdtype, w16, b16):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        w = w16 if w16 is not None else weight.to(cdtype)
        y = torch.addmm(b16 if b16 is not None else bias.to(cdtype), x2.to(cdtype), w.t())
        ctx.save_for_backward(x2, w)
        ctx.weight = weight
        ctx.bias = bias
        ctx.shape = shape
        return y.reshape(*shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        bias = ctx.bias
        N = w.shape[0]
        dy2 = dy.reshape(-1, N)
        if dy2.dtype != w.dtype:
            dy2 = dy2.to(w.dtype)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = (dy2 @ w).reshape(ctx.shape) if ctx.needs_input_grad[0] else None
        dw, db = lib_param_grads(dy2, x2.to(w.dtype), ctx.weight, bias, ctx.needs_input_grad[1],
                                 ctx.needs_input_grad[2])
        return dx, dw, db, None, None, None


def lib_param_grads(dy2: torch.Tensor, x2: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None,
                    need_w: bool, need_b: bool):
    """Library-GEMM weight gradient + column-sum bias gradient, written straight into persistent
    ``weight.grad`` / ``bias.grad`` when the engine provides them (returns None for those), else
    returned as new fp32 tensors."""
    M, N = dy2.shape
    K = x2.shape[1]
    dw = db = None
    if need_w:
        if _direct(weight) and weight.grad.is_contiguous():
            wgrad_into(dy2, x2, weight.grad, True)
            grad_ready(weight)
        else:
            dw = torch.empty(N, K, dtype=torch.float32, device=dy2.device)
            wgrad_into(dy2, x2, dw, False)
    if need_b:
        direct = _direct(bias)
        target = bias.grad if direct else torch.zeros(N, dtype=torch.float32, device=dy2.device)
        bias_grad_into(dy2, target)
        if direct:
            grad_ready(bias)
        else:
            db = target
    return dw, db


def _shadow_copy(module, name: str, p: torch.Tensor, dtype: torch.dtype):
    """16-bit (bf16 / fp16) copy of parameter ``p``, registered as its dense shadow: a fused
    optimizer keeps it current while updating ``p`` (no per-forward cast).  Re-cast here whenever
    ``p`` was written by anything else (its autograd version moved), no fused optimizer maintains
    it, or the parameter's registered shadow is another buffer (autocast dtype switched)."""
    buf = getattr(module, name, None)
    if (buf is None or buf.dtype != dtype or buf.shape != p.shape or buf.device != p.device
            or buf.stride() != p.stride()):
        buf = torch.empty_like(p, dtype=dtype)
        setattr(module, name, buf)
        setattr(module, name + "_version", None)
    sh = getattr(p, "_rocket_bf16_shadow", None)
    if sh is None or sh[1] is not buf:
        p._rocket_bf16_shadow = (None, buf)
        setattr(module, name + "_version", None)  # the optimizer maintained another buffer so far
    if not (getattr(p, "_rocket_shadow_live", False) and getattr(module, name + "_version") == p._version):
        with torch.no_grad():
            buf.copy_(p)
        setattr(module, name + "_version", p._version)
    return buf


def _bf16_copy(module, name: str, p: torch.Tensor):
    """bf16 copy of ``p`` maintained by the fused optimizer (:func:`_shadow_copy`)."""
    return _shadow_copy(module, name, p, torch.bfloat16)


def _lowp_copy(module, name: str, p: torch.Tensor, dtype: torch.dtype):
    """16-bit copy of parameter ``p`` in the autocast compute dtype, optimizer-maintained in both
    cases (dense bf16 or dense fp16 shadow); the fp16 copy lives under ``name + "_f16"``."""
    return _shadow_copy(module, name if dtype == torch.bfloat16 else name + "_f16", p, dtype)


class LibLinear(torch.nn.Linear):
    """``nn.Linear`` (same parameters / state_dict) for the large projections that stay on the
    library GEMM: under bf16 autocast on a HIP device the bias gradient is one column-sum launch
    (``rk_colsum_acc``, fp32, into ``bias.grad``) instead of a row reduction plus a bf16->fp32
    cast and an add, and the GEMM reads a bf16 weight copy that a fused optimizer maintains
    (dense bf16 shadow) instead of casting the fp32 master every forward; elsewhere it is exactly
    ``nn.Linear``."""

    def forward(self, x):
        if (x.is_cuda and self.bias is not None and native_route()
                and (self.out_features * self.in_features) % 8 == 0 and torch.is_grad_enabled()):
            cdtype = torch.get_autocast_dtype("cuda")
            w16 = b16 = None
            if (cdtype in (torch.bfloat16, torch.float16) and self.weight.dtype == torch.float32
                    and self.weight.is_contiguous()):
                w16 = _lowp_copy(self, "_w16", self.weight, cdtype)
                b16 = _lowp_copy(self, "_b16", self.bias, cdtype)
            return _LibLinear.apply(x, self.weight, self.bias, cdtype, w16, b16)
        return super().forward(x)


class _PatchEmbedFn(torch.autograd.Function):
    """Non-overlapping patch embedding (conv with stride == kernel) as patchify + ONE library GEMM:
    the im2col of a stride-k / kernel-k conv is a pure permutation of the image (no duplication), so
    the conv is ``patches [B*P, C*k*k] @ W^T + b``.  Backward: weight/bias gradients only (the image
    takes no gradient), straight into persistent grads."""

    @staticmethod
    def forward(ctx, x, weight, bias, w16, b16, k):
        B, C, H, W = x.shape
        gh, gw = H // k, W // k
        if (k % 8 == 0 and x.dtype in (torch.float32, w16.dtype) and x.is_contiguous()
                and w16.dtype in (torch.bfloat16, torch.float16)):
            # one native pass: cast + im2col permutation (norm.hip rk_patchify)
            p = torch.empty(B * gh * gw, C * k * k, dtype=w16.dtype, device=x.device)
            _lib.check(_lib.kernels().rk_patchify(_lib.dtype_code(x), _lib.dtype_code(p), x.data_ptr(), p.data_ptr(),
                                                  B, C, H, W, k, _lib.stream_ptr(x.device)), "rk_patchify")
        else:
            p = x.to(w16.dtype).reshape(B, C, gh, k, gw, k).permute(0, 2, 4, 1, 3, 5).reshape(B * gh * gw, C * k * k)
        from rocket_amd.ops import mlinear as _ml

        w2d = w16.reshape(w16.shape[0], -1)
        if _ml.MODE == "x5" and p.dtype == torch.bfloat16 and _ml._x5_shape(w2d.shape[0], w2d.shape[1]):
            y = _ml._x5(p, w2d, bias, p.shape[0], w2d.shape[0], w2d.shape[1])  # bias inside the MFMAs
        else:
            y = torch.addmm(b16, p, w2d.t())
        ctx.save_for_backward(p)
        ctx.params = (weight, bias)
        return y.view(B, gh * gw, -1)

    @staticmethod
    def backward(ctx, dy):
        (p,) = ctx.saved_tensors
        weight, bias = ctx.params
        N = weight.shape[0]
        dy2 = dy.reshape(-1, N)
        if dy2.dtype != p.dtype:
            dy2 = dy2.to(p.dtype)
        dy2 = dy2.contiguous()
        w2 = _FlatParam(weight)
        from rocket_amd.ops import mlinear as _ml

        if _ml.MODE == "x5" and dy2.dtype == torch.bfloat16:  # native split-K wgrad + bias grad
            dw, db = _ml._wgrad(dy2, p, w2, bias, ctx.needs_input_grad[1], ctx.needs_input_grad[2])
        else:
            dw, db = lib_param_grads(dy2, p, w2, bias, ctx.needs_input_grad[1], ctx.needs_input_grad[2])
        return None, (dw.view_as(weight) if dw is not None else None), db, None, None, None


class _FlatParam:
    """A [N, K] view of a conv weight (and of its persistent grad) for :func:`lib_param_grads`."""

    def __init__(self, p: torch.Tensor):
        self._p = p
        self.grad = p.grad.view(p.shape[0], -1) if p.grad is not None else None
        self._rocket_direct_grad = getattr(p, "_rocket_direct_grad", False)
        hook = getattr(p, "_rocket_grad_hook", None)
        if hook is not None:
            self._rocket_grad_hook = lambda _q: hook(p)


class PatchEmbed(torch.nn.Conv2d):
    """``nn.Conv2d(C, D, k, stride=k)`` (same parameters / state_dict) whose forward under bf16 or
    fp16 autocast on a HIP device returns the token matrix ``[B, (H/k)*(W/k), D]`` from one patchify
    copy + one library GEMM (:class:`_PatchEmbedFn`); elsewhere ``conv(x).flatten(2).transpose(1, 2)``."""

    def __init__(self, in_chans: int, dim: int, patch: int):
        super().__init__(in_chans, dim, patch, stride=patch)

    def forward(self, x):
        k = self.kernel_size[0]
        cdtype = torch.get_autocast_dtype("cuda") if x.is_cuda else None
        if (x.is_cuda and native_route() and cdtype in (torch.bfloat16, torch.float16) and x.dim() == 4
                and x.shape[2] % k == 0 and x.shape[3] % k == 0 and self.weight.is_contiguous()
                and self.weight.dtype == torch.float32):
            w16 = _lowp_copy(self, "_w16", self.weight, cdtype)
            b16 = _lowp_copy(self, "_b16", self.bias, cdtype)
            return _PatchEmbedFn.apply(x, self.weight, self.bias, w16, b16, k)
        return super().forward(x).flatten(2).transpose(1, 2)
