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

:class:`MMlp` is ``fc2(gelu(fc1(x)))`` as one autograd node (pre-activation saved once, GELU
forward/backward as single streaming kernels).  The weights are read as bf16 copies that a fused
optimizer keeps current (dense bf16 shadows, :func:`rocket_amd.ops.linear._bf16_copy`), so there
is no per-step cast either.  Which engine runs each product: ``MODE`` below.

Everywhere else (CPU, no autocast, odd shapes) they are exactly ``nn.Linear`` / the unfused MLP.
Reference anchor: the Linear layers of ``/root/reference/examples/mnist.py:49-51``.
"""

from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from torch import nn

from rocket_amd.ops import _lib
from rocket_amd.ops.linear import native_route, _bf16_copy, _direct, _lowp_copy, grad_ready, lib_param_grads
from rocket_amd.ops.mgemm import mgemm, pick_split

# Which engine runs each product.  ROCKET_VIT_GEMM:
#   lib            every product on the library GEMM (hipBLASLt with the shipped TunableOp table:
#                  tuned 256-wide tiles, K-split strided-batched wgrad) - the fastest routing
#                  measured in-model on 1x MI355X: ViT-B/16 5,058 img/s vs 4,629 hybrid and 4,290
#                  native (profiles/r2_vit_gemm_routing.md);
#   native         every product on mgemm (forward, K-major dgrad, split-K wgrad + fused bias grad);
#   hybrid         mgemm where it won the isolated per-shape probe (bench/mgemm_probe.py): all
#                  wgrads, the <= 2048-wide dgrads and the K = 3072 forward; the library elsewhere.
#   libw           forward / dgrad on the library, every weight gradient on mgemm (split-K with the
#                  bias gradient from the same launch: no K-split batched GEMM + slab sums + colsum)
#   libd           forward / wgrad on the library, every input gradient (K-major weight read, no
#                  transpose) on mgemm
#   x              every product on the macro-tile kernels of native/kernels/xgemm.hip (persistent
#                  256x256 / 256x128 tiles, buffer-load LDS-DMA ring; forward + bias, K-major-weight
#                  dgrad, split-K wgrad with the bias gradient from the same launch); the only route
#                  with fp16 operands (the GELU runs as its own streaming kernel)
#   x5             forward and input gradient on the persistent kernel of native/kernels/xgemm5.hip
#                  (bias inside the MFMAs; the input gradient reads a per-step transposed bf16 weight
#                  copy), products it does not take (N % 128, K < 320: the classifier head) on mgemm;
#                  weight gradients on mgemm (split-K over the tokens, bias gradient from the same
#                  launch) - no library GEMM anywhere
#   mixed (default) x5 for the products where it beat the library IN-MODEL (ViT-B/16, 1x MI355X,
#                  profiles/r6_vit_gemm_inmodel.md): the forward and input gradient with >= 2048 output
#                  features (256x256 tiles: qkv / fc1 forward, fc2 input gradient) and mgemm for the
#                  small products (classifier heads, <= 2^30 MACs); the library for the 768-wide outputs
#                  and the weight gradients
MODE = os.environ.get("ROCKET_VIT_GEMM", "mixed")
_X5_WIDE = 2048  # mixed: output width from which the forward / input gradient runs on xgemm5
_SMALL = 1 << 30  # mixed: products of at most this many MACs (classifier heads) run on mgemm


def _small(M: int, N: int, K: int, dtype: torch.dtype) -> bool:
    """mixed: a small bf16 product (classifier head) for mgemm (bf16 operands only)."""
    return MODE == "mixed" and dtype == torch.bfloat16 and M * N * K <= _SMALL
# The transformer MLP's two GEMMs whose neighbours are streaming GELU passes run on the native 256x256
# kernel (native/kernels/xgemm4.hip) with the GELU fused into their epilogues, beside any MODE:
#   fc1 forward       z = x W1^T + b1 and h = gelu(z) from ONE launch (no gelu_fwd pass);
#   fc2 input grad    dz = (dy W2) * gelu'(z) and db1 += colsum(dz) from ONE launch (no GELU-backward
#                     + column-sum pass; W2 read through a per-step transposed bf16 copy).
# Opt-in (ROCKET_VIT_X4_MLP=1): the fused launches are correct (tests/kernels/test_xgemm4.py) but the
# 256x256 core runs these short-K shapes at ~2/3 of hipBLASLt's rate, and the saved GELU passes do not
# pay for it: ViT-B/16 5,163 img/s fused vs 5,782 separate (profiles/r5_vit_b16_x4_mlp.md).
X4_MLP = os.environ.get("ROCKET_VIT_X4_MLP", "0") == "1"
_TILE_WIDE_FWD, _TILE_DEFAULT = 4, 0


def _fwd_tile(N: int) -> int:
    return _TILE_WIDE_FWD if N >= 2048 else _TILE_DEFAULT


def _x_tile(M: int, N: int, dtype: torch.dtype, splitk: int = 1) -> int:
    """xgemm config for an M x N output: the 256x256 tile unless the 256x128 one leaves fewer CU
    rounds (wave quantisation over the persistent grid); + 16 for fp16 operands."""
    from rocket_amd.ops.mgemm import N_CU, XTILE

    def rounds(bm, bn):
        return -(-(-(-M // bm) * -(-N // bn) * splitk) // N_CU)

    t = XTILE if rounds(256, 256) * 2 <= rounds(256, 128) * 1.25 else XTILE + 1
    return t + (16 if dtype == torch.float16 else 0)


def _x_split(M: int, N: int, K: int) -> int:
    """K splits of an xgemm wgrad (long K, few tiles): fill the CUs, each split a whole number of
    32-deep units, priced with the f32 slab each split writes and the combine reads."""
    from rocket_amd.ops.mgemm import N_CU

    tiles = -(-M // 256) * -(-N // 256)
    best = None
    for s in range(1, 33):
        rounds = -(-(tiles * s) // N_CU)
        cost = rounds * (K / s) + 0.08 * (s - 1) * K / 8
        if best is None or cost < best[0]:
            best = (cost, s)
    return best[1]


def _x5_shape(N: int, K: int) -> bool:
    """Output width / reduction depth rk_xgemm5 takes (N % 128, K % 64, K >= 320)."""
    return N % 128 == 0 and K % 64 == 0 and K >= 320


def _x5(a: torch.Tensor, b: torch.Tensor, bias, M: int, N: int, K: int) -> torch.Tensor:
    """C = a b^T (+ bias) on rk_xgemm5: a [M, K], b [N, K] bf16, C bf16."""
    c = torch.empty(M, N, dtype=a.dtype, device=a.device)
    _lib.check(_lib.kernels().rk_xgemm5(a.data_ptr(), K, b.data_ptr(), K, c.data_ptr(), N, _lib.dtype_code(c),
                                        _lib.ptr(bias), M, N, K, _lib.stream_ptr(a.device)), "rk_xgemm5")
    return c


def _transposed16(w16: torch.Tensor) -> torch.Tensor:
    """w16^T as a dense 16-bit copy (one launch): the input-gradient GEMM's K-contiguous B operand."""
    N, K = w16.shape
    wt = torch.empty(K, N, dtype=w16.dtype, device=w16.device)
    _lib.check(_lib.kernels().rk_transpose16(w16.data_ptr(), N, K, wt.data_ptr(), _lib.stream_ptr(w16.device)),
               "rk_transpose16")
    return wt


def _lib_fwd(K: int) -> bool:
    return MODE in ("lib", "libw", "libd", "mixed") or (MODE == "hybrid" and K < 2048)


def _lib_dgrad(N_in: int) -> bool:
    return MODE in ("lib", "libw", "mixed") or (MODE == "hybrid" and N_in > 2048)


def _x5_fwd(N: int, K: int, dtype: torch.dtype) -> bool:
    return dtype == torch.bfloat16 and _x5_shape(N, K) and (MODE == "x5" or (MODE == "mixed" and N >= _X5_WIDE))


def _ok(x: torch.Tensor, N: int, K: int) -> bool:
    # features % 8 (16-byte rows); the token count is free (the wgrad reads tokens as k-rows);
    # xgemm: row-layout operands move in 32-deep k-units (features % 32)
    if MODE == "x" and (K % 32 or N % 32):
        return False
    return x.is_cuda and K % 8 == 0 and N % 8 == 0 and _lib.available()


def _as_16_2d(t: torch.Tensor, K: int, dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    t = t.reshape(-1, K)
    if t.dtype != dtype:
        t = t.to(dtype)
    return t if t.is_contiguous() else t.contiguous()


_as_bf16_2d = _as_16_2d


def _linear_fwd(x2: torch.Tensor, w16: torch.Tensor, bias: torch.Tensor, b16: torch.Tensor) -> torch.Tensor:
    M, K = x2.shape
    N = w16.shape[0]
    if MODE == "x":
        y = torch.empty(M, N, dtype=x2.dtype, device=x2.device)
        mgemm(x2, w16, y, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, bias=bias, tile=_x_tile(M, N, x2.dtype))
        return y
    if _x5_fwd(N, K, x2.dtype):
        return _x5(x2, w16, bias, M, N, K)
    if _lib_fwd(K) and not _small(M, N, K, x2.dtype):
        return torch.addmm(b16, x2, w16.t())
    y = torch.empty(M, N, dtype=torch.bfloat16, device=x2.device)
    mgemm(x2, w16, y, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, bias=bias, tile=_fwd_tile(N))
    return y


def _linear_dgrad(dy2: torch.Tensor, w16: torch.Tensor, gelu_of: torch.Tensor | None = None) -> torch.Tensor:
    """dx = dy W (bf16); with ``gelu_of`` = z (native route only) the epilogue also multiplies by
    gelu'(z): the input gradient of a GELU whose input z fed this layer, in the same launch."""
    M, N = dy2.shape
    K = w16.shape[1]
    if MODE == "x":
        assert gelu_of is None
        dx = torch.empty(M, K, dtype=dy2.dtype, device=dy2.device)
        mgemm(dy2, w16, dx, M=M, N=K, K=N, lda=N, ldb=K, ldc=K, b_kmaj=True, tile=_x_tile(M, K, dy2.dtype))
        return dx
    if gelu_of is None and _x5_fwd(K, N, dy2.dtype):
        return _x5(dy2, _transposed16(w16), None, M, K, N)
    if _lib_dgrad(K) and not _small(M, N, K, dy2.dtype):
        assert gelu_of is None
        return dy2 @ w16
    dx = torch.empty(M, K, dtype=torch.bfloat16, device=dy2.device)
    mgemm(dy2, w16, dx, M=M, N=K, K=N, lda=N, ldb=K, ldc=K, b_kmaj=True, tile=_TILE_DEFAULT,
          aux=gelu_of, epi="none" if gelu_of is None else "mul_gelu_grad")
    return dx


def _wgrad(dy: torch.Tensor, x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None, need_w: bool,
           need_b: bool):
    """dW = dy^T x (f32) and db = column sums of dy, accumulated into persistent grads when the
    engine provides them (returns None for those), else returned as new tensors."""
    M, N = dy.shape
    K = x.shape[1]
    if MODE in ("lib", "libd") or (MODE == "mixed" and not _small(M, N, K, dy.dtype)):
        return lib_param_grads(dy, x, weight, bias, need_w, need_b)
    direct = (not need_w or _direct(weight)) and (not need_b or _direct(bias))
    if direct:
        dw = weight.grad if need_w else torch.empty(N, K, dtype=torch.float32, device=dy.device)
        db = bias.grad if need_b else None
    else:
        dw = torch.empty(N, K, dtype=torch.float32, device=dy.device)
        db = torch.zeros(N, dtype=torch.float32, device=dy.device) if need_b else None
    if MODE == "x":
        split = _x_split(N, K, M)
        tile = _x_tile(N, K, dy.dtype, split)
    else:
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


BIAS_LINK_HITS = 0  # bias gradients taken from a consuming add-LayerNorm (tests)


def _bias_from_link(link, dy: torch.Tensor, bias) -> tuple:
    """(handled, db): the bias gradient the consuming add-LayerNorm already formed (BiasLink), put
    into a persistent ``bias.grad`` (db None) or returned; handled False -> compute it here."""
    applied = link is not None and link.applied
    db = link.take(dy) if link is not None else None
    if db is None:
        return False, None
    global BIAS_LINK_HITS
    BIAS_LINK_HITS += 1
    if applied:  # the LN kernel added db into the persistent bias.grad already
        grad_ready(bias)
        return True, None
    if _direct(bias):
        bias.grad.add_(db)
        grad_ready(bias)
        return True, None
    return True, db


def _new_link(bias):
    from rocket_amd.ops.norm import BiasLink

    return BiasLink(bias) if (bias is not None and bias.requires_grad and torch.is_grad_enabled()) else None


class _MLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, w16, b16, link=None):
        shape = x.shape
        K = shape[-1]
        N = w16.shape[0]
        x2 = _as_16_2d(x, K, w16.dtype)
        y = _linear_fwd(x2, w16, bias, b16)
        ctx.save_for_backward(x2, w16)
        ctx.params = (weight, bias)
        ctx.shape = shape
        ctx.link = link
        return y.reshape(*shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w16 = ctx.saved_tensors
        weight, bias = ctx.params
        N = w16.shape[0]
        dy2 = _as_16_2d(dy, N, w16.dtype)
        dx = _linear_dgrad(dy2, w16).reshape(ctx.shape) if ctx.needs_input_grad[0] else None
        need_b = bias is not None and ctx.needs_input_grad[2]
        dw = db = None
        link, ctx.link = ctx.link, None
        if need_b:
            done, db = _bias_from_link(link, dy, bias)
            need_b = not done
        if ctx.needs_input_grad[1] or need_b:
            dw, db_ = _wgrad(dy2, x2, weight, bias, ctx.needs_input_grad[1], need_b)
            db = db_ if need_b else db
        return dx, dw, db, None, None, None


def _gelu_fwd(z: torch.Tensor) -> torch.Tensor:
    h = torch.empty_like(z)
    dt = _lib.dtype_code(z)
    _lib.check(_lib.kernels().rk_gelu_fwd(dt, dt, z.data_ptr(), h.data_ptr(), z.numel(),
                                          _lib.stream_ptr(z.device)), "rk_gelu_fwd")
    return h


def _gelu_bwd(dh: torch.Tensor, z: torch.Tensor) -> torch.Tensor:
    dz = torch.empty_like(z)
    _lib.check(_lib.kernels().rk_gelu_bwd(_lib.dtype_code(z), _lib.dtype_code(dh), dh.data_ptr(), z.data_ptr(),
                                          dz.data_ptr(), z.numel(), _lib.stream_ptr(z.device)), "rk_gelu_bwd")
    return dz


def _x4_ok(x2: torch.Tensor, K: int, N: int) -> bool:
    """Shapes / dtype the fused-epilogue x4 kernel takes: bf16 operands, K % 64, N % 8."""
    return X4_MLP and x2.dtype == torch.bfloat16 and K % 64 == 0 and N % 8 == 0 and x2.data_ptr() % 16 == 0


def _x4_fwd_gelu(x2: torch.Tensor, w16: torch.Tensor, bias: torch.Tensor):
    """(z, h = gelu(z)) of ``x2 @ w16^T + bias`` from one launch (rk_xgemm4_epi, GELU epilogue)."""
    M, K = x2.shape
    N = w16.shape[0]
    z = torch.empty(M, N, dtype=x2.dtype, device=x2.device)
    h = torch.empty_like(z)
    b = bias.detach().float().contiguous()
    _lib.check(_lib.kernels().rk_xgemm4_epi(x2.data_ptr(), K, w16.data_ptr(), K, h.data_ptr(), N,
                                            _lib.dtype_code(h), b.data_ptr(), z.data_ptr(), None, None, 1, M, N, K,
                                            _lib.stream_ptr(x2.device)), "rk_xgemm4_epi")
    return z, h


def _x4_dgrad_gelu(dy2: torch.Tensor, w16: torch.Tensor, z: torch.Tensor, bias: torch.Tensor | None):
    """dz = (dy2 @ w16) * gelu'(z) with the bias gradient of the layer that produced z (column sums
    of dz) accumulated by the same launch; returns (dz, db) with db None when it went straight into
    a persistent ``bias.grad`` (or when ``bias`` is None)."""
    M, N = dy2.shape
    K = w16.shape[1]  # dz columns
    wt = torch.empty(K, N, dtype=w16.dtype, device=w16.device)  # w16^T: the forward layout's B operand
    lib = _lib.kernels()
    stream = _lib.stream_ptr(dy2.device)
    _lib.check(lib.rk_transpose16(w16.data_ptr(), N, K, wt.data_ptr(), stream), "rk_transpose16")
    dz = torch.empty(M, K, dtype=dy2.dtype, device=dy2.device)
    db = None
    if bias is not None:
        direct = _direct(bias)
        db = bias.grad if direct else torch.zeros(K, dtype=torch.float32, device=dy2.device)
    _lib.check(lib.rk_xgemm4_epi(dy2.data_ptr(), N, wt.data_ptr(), N, dz.data_ptr(), K, _lib.dtype_code(dz), None,
                                 None, z.data_ptr(), _lib.ptr(db), 2, M, K, N, stream), "rk_xgemm4_epi")
    if bias is not None and _direct(bias):
        grad_ready(bias)
        return dz, None
    return dz, db


def _gelu_bwd_bias(dh: torch.Tensor, z: torch.Tensor, bias: torch.Tensor):
    """(dz = dh * gelu'(z), column sums of dz added to the bias gradient) in one launch; returns
    (dz, db) with db None when it went straight into a persistent ``bias.grad``."""
    M, N = z.shape
    direct = _direct(bias)
    target = bias.grad if direct else torch.zeros(N, dtype=torch.float32, device=z.device)
    dz = torch.empty_like(z)
    lib = _lib.kernels()
    ws = torch.empty(int(lib.rk_bn_workspace(M, N)), dtype=torch.float32, device=z.device)
    nctr = int(lib.rk_bn_counters(N))
    if dh.dtype != z.dtype:
        dh = dh.to(z.dtype)
    _lib.check(lib.rk_gelu_bwd_colsum16(_lib.dtype_code(z), dh.data_ptr(), z.data_ptr(), dz.data_ptr(), M, N,
                                        target.data_ptr(), ws.data_ptr(),
                                        _lib.Workspace.get(z.device).counter_array(f"bn{nctr}", nctr),
                                        _lib.stream_ptr(z.device)), "rk_gelu_bwd_colsum16")
    if direct:
        grad_ready(bias)
        return dz, None
    return dz, target


class _MMlpFn(torch.autograd.Function):
    """y = fc2(gelu(fc1(x))): GELU forward/backward as one streaming HIP kernel each (a GELU
    epilogue inside the K = 768 GEMM costs more than that: the erf math runs in phase with the
    MFMAs of every block instead of overlapping them)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w1_16, b1_16, w2_16, b2_16, link=None):
        shape = x.shape
        K = shape[-1]
        N = w2_16.shape[0]
        x2 = _as_16_2d(x, K, w1_16.dtype)
        if MODE != "x" and _x4_ok(x2, K, w1_16.shape[0]):
            z, h = _x4_fwd_gelu(x2, w1_16, b1)  # GELU in the GEMM epilogue
        else:
            z = _linear_fwd(x2, w1_16, b1, b1_16)
            h = _gelu_fwd(z)
        y = _linear_fwd(h, w2_16, b2, b2_16)
        ctx.save_for_backward(x2, z, h, w1_16, w2_16)
        ctx.params = (w1, b1, w2, b2)
        ctx.shape = shape
        ctx.link = link
        return y.reshape(*shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, z, h, w1_16, w2_16 = ctx.saved_tensors
        w1, b1, w2, b2 = ctx.params
        N = w2_16.shape[0]
        dy2 = _as_16_2d(dy, N, w2_16.dtype)
        g = ctx.needs_input_grad
        need_b1 = b1 is not None and g[2]
        db1 = None
        if MODE == "x":
            # dz = gelu'(z) * (dy W2) by the streaming kernel; fc1's bias gradient comes out of
            # its wgrad launch (row sums of dz)
            dz = _gelu_bwd(_linear_dgrad(dy2, w2_16), z)
        elif MODE != "x" and _x4_ok(dy2, N, z.shape[1]) and z.dtype == torch.bfloat16:
            # gelu'(z) and fc1's bias gradient in fc2's input-gradient GEMM epilogue
            dz, db1 = _x4_dgrad_gelu(dy2, w2_16, z, b1 if need_b1 else None)
            need_b1 = False
        elif MODE in ("lib", "x5", "mixed") and need_b1:
            # GELU backward and fc1's bias gradient in one pass over the [tokens, hidden] gradient
            dz, db1 = _gelu_bwd_bias(_linear_dgrad(dy2, w2_16), z, b1)
            need_b1 = False
        elif not _lib_dgrad(z.shape[1]):
            # native fc2 input gradient with gelu'(z) in its epilogue: dz straight out of the GEMM
            dz = _linear_dgrad(dy2, w2_16, gelu_of=z)
        else:
            dz = _gelu_bwd(_linear_dgrad(dy2, w2_16), z)
        need_b2 = b2 is not None and g[4]
        link, ctx.link = ctx.link, None
        db2 = None
        if need_b2:
            done, db2 = _bias_from_link(link, dy, b2)
            need_b2 = not done
        dw2, db2_ = _wgrad(dy2, h, w2, b2, g[3], need_b2)
        db2 = db2_ if need_b2 else db2
        dx = _linear_dgrad(dz, w1_16).reshape(ctx.shape) if g[0] else None
        dw1, db1_ = _wgrad(dz, x2, w1, b1, g[1], need_b1)
        return dx, dw1, (db1 if db1_ is None else db1_), dw2, db2, None, None, None, None, None


def _cdtype() -> torch.dtype:
    return torch.get_autocast_dtype("cuda")


def _native(module: nn.Linear, x: torch.Tensor) -> bool:
    dt = _cdtype()
    # fp16: the library routes (hipBLASLt fp16 GEMMs beside the fp16 attention / LayerNorm / GELU
    # kernels) and the xgemm route; the mgemm routes are bf16-only
    return (x.is_cuda and native_route() and (dt == torch.bfloat16 or (dt == torch.float16 and MODE in ("x", "lib", "mixed")))
            and module.weight.dtype == torch.float32 and module.weight.is_contiguous()
            and _ok(x, module.out_features, module.in_features))


# classifier heads whose class count is not a multiple of 8 (head.hip): one forward, one backward
# launch, fp32 logits.  ROCKET_HEAD=0: nn.Linear (the library route under autocast)
HEAD = os.environ.get("ROCKET_HEAD", "1") != "0"
_HEAD_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def _head_ok(module: nn.Linear, x: torch.Tensor) -> bool:
    N, K = module.out_features, module.in_features
    return (HEAD and x.is_cuda and native_route() and N % 8 != 0 and N <= 128 and x.dtype in _HEAD_DT
            and x.shape[-1] == K and x.numel() < (1 << 31) and module.weight.dtype == torch.float32
            and module.weight.is_contiguous() and (module.bias is None or module.bias.dtype == torch.float32)
            and _lib.available())


class _HeadFn(torch.autograd.Function):
    """y = x W^T + b (fp32 logits) and its backward in one launch each (head.hip)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        N, K = weight.shape
        x2 = x.reshape(-1, K)
        x2 = x2 if x2.is_contiguous() else x2.contiguous()
        M = x2.shape[0]
        y = torch.empty(M, N, dtype=torch.float32, device=x.device)
        _lib.check(_lib.kernels().rk_head_fwd(_HEAD_DT[x2.dtype], x2.data_ptr(), weight.data_ptr(), _lib.ptr(bias),
                                              y.data_ptr(), M, N, K, 1, None, _lib.stream_ptr(x.device)),
                   "rk_head_fwd")
        ctx.save_for_backward(x2, weight)
        ctx.bias = bias
        ctx.xshape = x.shape
        ctx.hw = 1
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        bias = ctx.bias
        N, K = weight.shape
        M = x2.shape[0]
        dy2 = dy.reshape(M, N)
        if dy2.dtype != torch.float32 or not dy2.is_contiguous():
            dy2 = dy2.float().contiguous()
        need_x, need_w, need_b = ctx.needs_input_grad
        need_b = need_b and bias is not None
        dev = x2.device
        hw = ctx.hw
        if need_x:
            dx = torch.empty_like(x2) if hw == 1 else torch.empty(ctx.xshape, dtype=x2.dtype, device=x2.device,
                                                                   memory_format=torch.channels_last)
        else:
            dx = None
        direct_w = need_w and _direct(weight) and weight.grad.is_contiguous()
        direct_b = need_b and _direct(bias)
        dw = weight.grad if direct_w else (torch.empty(N, K, dtype=torch.float32, device=dev)
                                           if (need_w or need_b) else None)  # db rides on the dW blocks
        db = (bias.grad if direct_b else torch.empty(N, dtype=torch.float32, device=dev)) if need_b else None
        lib = _lib.kernels()
        part = cnt = None
        if dw is not None:  # dW partials per 64-row chunk + the chunk-combine tickets (left zeroed)
            part = torch.empty(int(lib.rk_head_bwd_scratch(M, N, K)), dtype=torch.float32, device=dev)
            kb = -(-K // 64)
            cnt = _lib.Workspace.get(dev).counter_array(f"head{kb}", kb)
        _lib.check(lib.rk_head_bwd(_HEAD_DT[x2.dtype], dy2.data_ptr(), x2.data_ptr(), weight.data_ptr(),
                                   _lib.ptr(dx), _lib.ptr(dw), _lib.ptr(db), int(direct_w), int(direct_b),
                                   M, N, K, _lib.ptr(part), cnt, hw, _lib.stream_ptr(dev)), "rk_head_bwd")
        if direct_w:
            grad_ready(weight)
        if direct_b:
            grad_ready(bias)
        return (dx.view(ctx.xshape) if need_x and hw == 1 else dx, dw if need_w and not direct_w else None,
                db if need_b and not direct_b else None)


class _PooledHeadFn(_HeadFn):
    """``head(global_avg_pool(x))`` for a channels-last ``[N, C, H, W]`` activation: the pool runs
    inside the head's forward launch (pooled rows kept for the weight gradient) and its backward
    (the ``dy / HW`` broadcast) inside the head's backward launch — two launches fewer than
    ``ops.pool.global_avg_pool`` + :class:`_HeadFn`, same rounding."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        N, C, H, W = x.shape
        Nc, K = weight.shape
        xpool = torch.empty(N, C, dtype=x.dtype, device=x.device)
        y = torch.empty(N, Nc, dtype=torch.float32, device=x.device)
        _lib.check(_lib.kernels().rk_head_fwd(_HEAD_DT[x.dtype], x.data_ptr(), weight.data_ptr(), _lib.ptr(bias),
                                              y.data_ptr(), N, Nc, K, H * W, xpool.data_ptr(),
                                              _lib.stream_ptr(x.device)), "rk_head_fwd(pooled)")
        ctx.save_for_backward(xpool, weight)
        ctx.bias = bias
        ctx.xshape = x.shape
        ctx.hw = H * W
        return y


def pooled_head_ok(module: nn.Module, x: torch.Tensor) -> bool:
    """Whether ``module(global_avg_pool(x))`` can run as :class:`_PooledHeadFn`."""
    return (isinstance(module, MLinear) and x.dim() == 4 and x.shape[1] == module.in_features
            and x.is_contiguous(memory_format=torch.channels_last) and x.shape[2] * x.shape[3] > 1
            and _head_ok(module, x.new_empty(0, module.in_features)))


def pooled_head(module: nn.Linear, x: torch.Tensor) -> torch.Tensor:
    return _PooledHeadFn.apply(x, module.weight, module.bias)


class MLinear(nn.Linear):
    """``nn.Linear`` on the native MFMA GEMM under bf16 autocast (module docstring); class counts
    that are not a multiple of 8 on the head kernels (:class:`_HeadFn`, fp32 logits)."""

    def forward(self, x):
        if _head_ok(self, x):
            return _HeadFn.apply(x, self.weight, self.bias)
        if _native(self, x) and self.bias is not None:
            dt = _cdtype()
            w16 = _lowp_copy(self, "_w16", self.weight, dt)
            b16 = _lowp_copy(self, "_b16", self.bias, dt)
            link = _new_link(self.bias)
            y = _MLinearFn.apply(x, self.weight, self.bias, w16, b16, link)
            if link is not None:
                y._rocket_bias_link = link  # a consuming add-LayerNorm may form the bias gradient
            return y
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
            f1, f2 = self.fc1, self.fc2
            dt = _cdtype()
            link = _new_link(f2.bias)
            y = _MMlpFn.apply(x, f1.weight, f1.bias, f2.weight, f2.bias, _lowp_copy(f1, "_w16", f1.weight, dt),
                              _lowp_copy(f1, "_b16", f1.bias, dt), _lowp_copy(f2, "_w16", f2.weight, dt),
                              _lowp_copy(f2, "_b16", f2.bias, dt), link)
            if link is not None:
                y._rocket_bias_link = link  # a consuming add-LayerNorm may form fc2's bias gradient
            return y
        return self.fc2(F.gelu(self.fc1(x)))
