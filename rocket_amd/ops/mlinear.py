"""Linear layers on the native MFMA GEMM (``native/kernels/mgemm.hip``) for the transformer path.

:class:`MLinear` is ``nn.Linear`` (same parameters and state_dict) whose forward, dgrad and wgrad
under bf16 autocast on a HIP device are each ONE ``rk_mgemm`` launch (plus the split-K combine
launch of the wgrad):

* forward ``y = x W^T + b``: bias in the epilogue, bf16 out;
* dgrad ``dx = dy W``: W read K-major straight from the [N, K] weight (no transpose copy);
* wgrad ``dW = dy^T x``: both operands read token-major, split-K over the tokens into f32 slabs,
  combined straight into a persistent ``weight.grad`` (``_rocket_direct_grad``); the bias gradient
  ``db = sum_tokens dy`` comes out of the same launch (MFMAs against a ones fragment), so there is
  no column-sum kernel.

:class:`MMlp` fuses ``fc2(gelu(fc1(x)))``: fc1's epilogue applies GELU and keeps the pre-activation,
and fc2's dgrad epilogue multiplies by ``gelu'(pre)`` — the GELU forward and backward kernels
disappear.  The weights are read as bf16 copies that a fused optimizer keeps current (dense bf16
shadows, :func:`rocket_amd.ops.linear._bf16_copy`), so there is no per-step cast either.

Everywhere else (CPU, no autocast, odd shapes) they are exactly ``nn.Linear`` / the unfused MLP.
Reference anchor: the Linear layers of ``/root/reference/examples/mnist.py:49-51``.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from rocket_amd.ops import _lib
from rocket_amd.ops.linear import _autocast_on, _bf16_copy, _direct, grad_ready
from rocket_amd.ops.mgemm import mgemm, pick_split

# forward/dgrad tile per operand layout (bench/mgemm_probe.py at the ViT-B/16 shapes): the
# 4-wave 128x128 tile wins the wide (N >= 2048) forwards, the 8-wave one everything else
_TILE_WIDE_FWD, _TILE_DEFAULT = 4, 0


def _fwd_tile(N: int) -> int:
    return _TILE_WIDE_FWD if N >= 2048 else _TILE_DEFAULT


def _ok(x: torch.Tensor, N: int, K: int) -> bool:
    # features % 8 (16-byte rows); the token count is free (the wgrad reads tokens as k-rows)
    return x.is_cuda and K % 8 == 0 and N % 8 == 0 and _lib.available()


def _as_bf16_2d(t: torch.Tensor, K: int) -> torch.Tensor:
    t = t.reshape(-1, K)
    if t.dtype != torch.bfloat16:
        t = t.to(torch.bfloat16)
    return t if t.is_contiguous() else t.contiguous()


def _wgrad(dy: torch.Tensor, x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None, need_w: bool,
           need_b: bool):
    """dW = dy^T x (f32) and db = column sums of dy, accumulated into persistent grads when the
    engine provides them (returns None for those), else returned as new tensors."""
    M, N = dy.shape
    K = x.shape[1]
    direct = (not need_w or _direct(weight)) and (not need_b or _direct(bias))
    if direct:
        dw = weight.grad if need_w else torch.empty(N, K, dtype=torch.float32, device=dy.device)
        db = bias.grad if need_b else None
    else:
        dw = torch.empty(N, K, dtype=torch.float32, device=dy.device)
        db = torch.zeros(N, dtype=torch.float32, device=dy.device) if need_b else None
    tile, split = pick_split(N, K, M)
    mgemm(dy, x, dw, M=N, N=K, K=M, lda=N, ldb=K, ldc=K, a_kmaj=True, b_kmaj=True, rowsum=db,
          accumulate=direct and need_w, splitk=split, tile=tile)
    if direct:
        if need_w:
            grad_ready(weight)
        if need_b:
            grad_ready(bias)
        return None, None
    return (dw if need_w else None), db


class _MLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, w16):
        shape = x.shape
        K = shape[-1]
        N = w16.shape[0]
        x2 = _as_bf16_2d(x, K)
        M = x2.shape[0]
        y = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
        mgemm(x2, w16, y, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, bias=bias, tile=_fwd_tile(N))
        ctx.save_for_backward(x2, w16)
        ctx.params = (weight, bias)
        ctx.shape = shape
        return y.reshape(*shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w16 = ctx.saved_tensors
        weight, bias = ctx.params
        M, K = x2.shape
        N = w16.shape[0]
        dy2 = _as_bf16_2d(dy, N)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, dtype=torch.bfloat16, device=dy.device)
            mgemm(dy2, w16, dx, M=M, N=K, K=N, lda=N, ldb=K, ldc=K, b_kmaj=True, tile=_TILE_DEFAULT)
            dx = dx.reshape(ctx.shape)
        need_b = bias is not None and ctx.needs_input_grad[2]
        dw = db = None
        if ctx.needs_input_grad[1] or need_b:
            dw, db = _wgrad(dy2, x2, weight, bias, ctx.needs_input_grad[1], need_b)
        return dx, dw, db, None


class _MMlpFn(torch.autograd.Function):
    """y = fc2(gelu(fc1(x))) with GELU in fc1's epilogue and gelu' in fc2's dgrad epilogue."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w1_16, w2_16):
        shape = x.shape
        K = shape[-1]
        H, N = w1_16.shape[0], w2_16.shape[0]
        x2 = _as_bf16_2d(x, K)
        M = x2.shape[0]
        pre = torch.empty(M, H, dtype=torch.bfloat16, device=x.device)
        h = torch.empty(M, H, dtype=torch.bfloat16, device=x.device)
        mgemm(x2, w1_16, h, M=M, N=H, K=K, lda=K, ldb=K, ldc=H, bias=b1, epi="gelu", c_pre=pre, tile=_fwd_tile(H))
        y = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
        mgemm(h, w2_16, y, M=M, N=N, K=H, lda=H, ldb=H, ldc=N, bias=b2, tile=_fwd_tile(N))
        ctx.save_for_backward(x2, pre, h, w1_16, w2_16)
        ctx.params = (w1, b1, w2, b2)
        ctx.shape = shape
        return y.reshape(*shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, pre, h, w1_16, w2_16 = ctx.saved_tensors
        w1, b1, w2, b2 = ctx.params
        M, K = x2.shape
        H, N = w1_16.shape[0], w2_16.shape[0]
        dy2 = _as_bf16_2d(dy, N)
        # d(pre) = (dy W2) * gelu'(pre): the GELU backward is fc2's dgrad epilogue
        dpre = torch.empty(M, H, dtype=torch.bfloat16, device=dy.device)
        mgemm(dy2, w2_16, dpre, M=M, N=H, K=N, lda=N, ldb=H, ldc=H, b_kmaj=True, epi="mul_gelu_grad", aux=pre,
              tile=_TILE_DEFAULT)
        g = ctx.needs_input_grad
        dw2, db2 = _wgrad(dy2, h, w2, b2, g[3], b2 is not None and g[4])
        dx = None
        if g[0]:
            dx = torch.empty(M, K, dtype=torch.bfloat16, device=dy.device)
            mgemm(dpre, w1_16, dx, M=M, N=K, K=H, lda=H, ldb=K, ldc=K, b_kmaj=True, tile=_TILE_DEFAULT)
            dx = dx.reshape(ctx.shape)
        dw1, db1 = _wgrad(dpre, x2, w1, b1, g[1], b1 is not None and g[2])
        return dx, dw1, db1, dw2, db2, None, None


def _native(module: nn.Linear, x: torch.Tensor) -> bool:
    return (x.is_cuda and _autocast_on() and torch.get_autocast_dtype("cuda") == torch.bfloat16
            and module.weight.dtype == torch.float32 and module.weight.is_contiguous()
            and _ok(x, module.out_features, module.in_features))


class MLinear(nn.Linear):
    """``nn.Linear`` on the native MFMA GEMM under bf16 autocast (module docstring)."""

    def forward(self, x):
        if _native(self, x):
            w16 = _bf16_copy(self, "_w16", self.weight)
            return _MLinearFn.apply(x, self.weight, self.bias, w16)
        return super().forward(x)


class MMlp(nn.Module):
    """Transformer MLP ``fc2(gelu(fc1(x)))`` (``fc1``/``fc2`` state_dict keys, erf GELU) with the
    activation fused into the GEMMs (module docstring)."""

    def __init__(self, dim: int, hidden: int):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x):
        if _native(self.fc1, x) and _ok(x, self.fc2.out_features, self.fc2.in_features) and \
                self.fc2.weight.is_contiguous() and self.fc1.bias is not None and self.fc2.bias is not None:
            w1 = _bf16_copy(self.fc1, "_w16", self.fc1.weight)
            w2 = _bf16_copy(self.fc2, "_w16", self.fc2.weight)
            return _MMlpFn.apply(x, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias, w1, w2)
        return self.fc2(F.gelu(self.fc1(x)))
