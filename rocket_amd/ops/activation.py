"""GELU and row softmax on HIP (``native/kernels/act.hip``) + the attention composite.

* :func:`gelu` — exact (erf) GELU; backward recomputes the derivative from the saved input.
* :func:`softmax` — ``softmax(x * scale)`` over the last dim in one read/one write, with the
  fused backward ``scale * y * (dy - <dy, y>)`` (rows up to 1024 long).
* :func:`attention` — ``softmax(q k^T * scale) v`` for short sequences (ViT: 197 tokens):
  the two batched GEMMs run on the library (hipBLASLt) path, the scaled softmax on the
  kernel above, so the score matrix is read and written once per direction.
* :func:`attention_qkv` — the fused MFMA attention of ``native/kernels/attn.hip`` working
  directly on the QKV projection output (token-major, no head permutes, scores never leave
  the CU): one launch forward, two backward, writing d(qkv) as one tensor.
"""

from __future__ import annotations

import math
import os

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
    if (_ops.fused_enabled() and x.is_cuda and x.dtype in (torch.float32, torch.bfloat16, torch.float16)
            and x.numel() % 4 == 0):
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


# waves per (batch, head) block of the attention kernels: fwd,bwd_q,bwd_kv (4 or 8 each; 82 = 8 waves
# register-bounded to 128 VGPRs so two blocks share a CU; profiles/r2_attn_waves_ab.txt)
ATTN_WAVES = tuple(int(v) for v in os.environ.get("ROCKET_ATTN_WAVES", "8,82,82").split(","))
# backward: "fused" (default: one kernel per (batch, head), S / dP computed once, one wave per key
# tile, dQ from the per-chunk dS image), "stream" (the same with only K staged whole and the query
# chunks' Q / dO / O streamed by LDS-DMA one chunk ahead) or "split" (the dQ and dK/dV kernels,
# each recomputing S and dP)
ATTN_BWD = os.environ.get("ROCKET_ATTN_BWD", "fused")
_BWD_MODES = {"split": 0, "fused": 1, "stream": 2}
_waves_set = False


def _attn_lib():
    global _waves_set
    lib = _lib.kernels()
    if not _waves_set:
        _lib.check(lib.rk_attn_set_waves(*ATTN_WAVES), "rk_attn_set_waves")
        _lib.check(lib.rk_attn_set_bwd_fused(_BWD_MODES[ATTN_BWD]), "rk_attn_set_bwd_fused")
        _waves_set = True
    return lib


class _AttnQKV(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, heads: int, scale: float):
        lib = _attn_lib()
        qkv = qkv.contiguous()
        B, L, C3 = qkv.shape
        HD = C3 // 3
        out = torch.empty(B, L, HD, dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(B * heads, L, dtype=torch.float32, device=qkv.device)
        base, es = qkv.data_ptr(), qkv.element_size()
        hf = int(qkv.dtype == torch.float16)
        _lib.check(lib.rk_attn_fwd16(hf, base, base + HD * es, base + 2 * HD * es, C3, out.data_ptr(), HD,
                                     lse.data_ptr(), B, L, heads, float(scale), _lib.stream_ptr(qkv.device)),
                   "rk_attn_fwd16")
        ctx.cfg = (heads, scale)
        ctx.save_for_backward(qkv, out, lse)
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = _attn_lib()
        qkv, out, lse = ctx.saved_tensors
        heads, scale = ctx.cfg
        B, L, C3 = qkv.shape
        HD = C3 // 3
        dout = dout.contiguous()
        if dout.dtype != qkv.dtype:
            dout = dout.to(qkv.dtype)
        dqkv = torch.empty_like(qkv)
        delta = torch.empty(B * heads, L, dtype=torch.float32, device=qkv.device)  # (split backward)
        base, gbase, es = qkv.data_ptr(), dqkv.data_ptr(), qkv.element_size()
        _lib.check(lib.rk_attn_bwd16(int(qkv.dtype == torch.float16), base, base + HD * es, base + 2 * HD * es, C3,
                                     out.data_ptr(), dout.data_ptr(), HD, lse.data_ptr(), delta.data_ptr(), gbase,
                                     gbase + HD * es, gbase + 2 * HD * es, C3, B, L, heads, float(scale),
                                     _lib.stream_ptr(qkv.device)), "rk_attn_bwd16")
        return dqkv, None, None


def attention_qkv(qkv: torch.Tensor, heads: int, scale: float | None = None) -> torch.Tensor:
    """Multi-head self-attention from the packed projection ``qkv`` [B, L, 3*H*D] -> [B, L, H*D]."""
    B, L, C3 = qkv.shape
    D = C3 // (3 * heads)
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    # fp16: the default kernel configuration only (8-wave forward, fused backward)
    f16_ok = qkv.dtype == torch.float16 and ATTN_BWD == "fused"  # fp16 backward: the fused kernel
    if (_ops.fused_enabled() and qkv.is_cuda and (qkv.dtype == torch.bfloat16 or f16_ok) and D == 64
            and L <= _lib.kernels().rk_attn_max_len()):
        return _AttnQKV.apply(qkv, heads, scale)
    t = qkv.view(B, L, 3, heads, D).permute(2, 0, 3, 1, 4)
    o = attention(t[0], t[1], t[2], scale)
    return o.transpose(1, 2).reshape(B, L, heads * D)
