"""Fused LeNet building blocks (``native/kernels/lenet_conv.hip`` and ``mlp.hip``).

* :func:`lenet_features` — conv(1→6,5×5,p2)+ReLU+pool → conv(6→16,5×5)+ReLU+pool on
  MFMA, one launch forward, one launch backward (conv2 dgrad + both weight/bias
  gradients).  Returns the flattened ``[N, 400]`` bf16 feature map.
* :func:`mlp_head` — a 3-layer ReLU MLP (``fc1-ReLU-fc2-ReLU-fc3``): one launch for
  the forward chain, one for the input-gradient chain, then the three weight
  gradients on the MFMA GEMM (split-K, fused bias-gradient).

Both are ordinary autograd Functions over fp32 master parameters.  Weight
gradients accumulate directly into persistent ``param.grad`` buffers when the
engine provides them (graph capture / flat gradient buckets), otherwise they
are returned to autograd.
"""

from __future__ import annotations

from typing import List, Sequence

import ctypes

import torch

from rocket_amd.ops import _lib
from rocket_amd.ops.linear import _direct, gemm, grad_ready


def _grad_targets(params: Sequence[torch.nn.Parameter], device):
    """Return (buffers, direct): persistent grads, or one zeroed flat buffer split per param."""
    if all(_direct(p) for p in params):
        return [p.grad for p in params], True
    flat = torch.zeros(sum(p.numel() for p in params), dtype=torch.float32, device=device)
    out, off = [], 0
    for p in params:
        out.append(flat[off : off + p.numel()].view_as(p))
        off += p.numel()
    return out, False


def _finish(params, bufs, direct):
    if direct:
        for p in params:
            grad_ready(p)
        return [None] * len(params)
    return bufs


class _LeNetFeatures(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        lib = _lib.kernels()
        x = x.contiguous().float()
        N = x.shape[0]
        assert tuple(x.shape[1:]) == (1, 28, 28), "lenet_features expects [N,1,28,28]"
        dev = x.device
        a1 = torch.empty(N, 1176, dtype=torch.bfloat16, device=dev)
        c1 = torch.empty(N, 1176, dtype=torch.uint8, device=dev)
        a2 = torch.empty(N, 400, dtype=torch.bfloat16, device=dev)
        c2 = torch.empty(N, 400, dtype=torch.uint8, device=dev)
        w1c, b1c, w2c, b2c = (t.detach().float().contiguous() for t in (w1, b1, w2, b2))
        _lib.check(lib.rk_lenet_conv_fwd(x.data_ptr(), w1c.data_ptr(), b1c.data_ptr(), w2c.data_ptr(), b2c.data_ptr(),
                                         a1.data_ptr(), c1.data_ptr(), a2.data_ptr(), c2.data_ptr(), N,
                                         _lib.stream_ptr(dev)), "rk_lenet_conv_fwd")
        ctx.params = (w1, b1, w2, b2)
        ctx.save_for_backward(x, a1, c1, c2, w2c)
        return a2

    @staticmethod
    def backward(ctx, da2):
        lib = _lib.kernels()
        x, a1, c1, c2, w2c = ctx.saved_tensors
        N = x.shape[0]
        da2 = da2.contiguous()
        if da2.dtype != torch.bfloat16:
            da2 = da2.to(torch.bfloat16)
        params = ctx.params
        bufs, direct = _grad_targets(params, x.device)
        rounds = max(1, N // 2048)
        _lib.check(lib.rk_lenet_conv_bwd(x.data_ptr(), a1.data_ptr(), c1.data_ptr(), da2.data_ptr(), c2.data_ptr(),
                                         w2c.data_ptr(), bufs[0].data_ptr(), bufs[1].data_ptr(), bufs[2].data_ptr(),
                                         bufs[3].data_ptr(), N, rounds, _lib.stream_ptr(x.device)), "rk_lenet_conv_bwd")
        return (None, *_finish(params, bufs, direct))


def lenet_features(x, w1, b1, w2, b2):
    return _LeNetFeatures.apply(x, w1, b1, w2, b2)


class _MLPHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w3, b3):
        lib = _lib.kernels()
        x = x.contiguous()
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        M, K0 = x.shape
        N1, N2, N3 = w1.shape[0], w2.shape[0], w3.shape[0]
        dev = x.device
        bf = dict(dtype=torch.bfloat16, device=dev)
        xT = torch.empty(K0, M, **bf)
        h1T = torch.empty(N1, M, **bf)
        h2T = torch.empty(N2, M, **bf)
        y = torch.empty(M, N3, dtype=torch.float32, device=dev)
        ws = [t.detach().float().contiguous() for t in (w1, b1, w2, b2, w3, b3)]
        _lib.check(lib.rk_mlp3_fwd(x.data_ptr(), K0, ws[0].data_ptr(), ws[1].data_ptr(), N1, ws[2].data_ptr(),
                                   ws[3].data_ptr(), N2, ws[4].data_ptr(), ws[5].data_ptr(), N3, xT.data_ptr(),
                                   h1T.data_ptr(), h2T.data_ptr(), y.data_ptr(), M, _lib.stream_ptr(dev)),
                   "rk_mlp3_fwd")
        ctx.params = (w1, b1, w2, b2, w3, b3)
        ctx.save_for_backward(xT, h1T, h2T, ws[0], ws[2], ws[4])
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib.kernels()
        xT, h1T, h2T, w1, w2, w3 = ctx.saved_tensors
        K0, M = xT.shape
        N1, N2, N3 = w1.shape[0], w2.shape[0], w3.shape[0]
        dev = xT.device
        dy = dy.contiguous().float()
        bf = dict(dtype=torch.bfloat16, device=dev)
        dyT = torch.empty(N3, M, **bf)
        d2T = torch.empty(N2, M, **bf)
        d1T = torch.empty(N1, M, **bf)
        dx = torch.empty(M, K0, **bf) if ctx.needs_input_grad[0] else None
        stream = _lib.stream_ptr(dev)
        _lib.check(lib.rk_mlp3_dgrad(dy.data_ptr(), N3, w3.data_ptr(), N2, h2T.data_ptr(), w2.data_ptr(), N1,
                                     h1T.data_ptr(), w1.data_ptr(), K0, dyT.data_ptr(), d2T.data_ptr(),
                                     d1T.data_ptr(), _lib.ptr(dx), M, stream), "rk_mlp3_dgrad")
        params = ctx.params
        bufs, direct = _grad_targets(params, dev)
        probs = ((dyT, h2T, bufs[4], bufs[5], N3, N2), (d2T, h1T, bufs[2], bufs[3], N2, N1),
                 (d1T, xT, bufs[0], bufs[1], N1, K0))
        if M % 8 == 0:
            P = ctypes.c_void_p * 3
            I = ctypes.c_int * 3
            _lib.check(lib.rk_mlp3_wgrad(3, P(*[p[0].data_ptr() for p in probs]), P(*[p[1].data_ptr() for p in probs]),
                                         P(*[p[2].data_ptr() for p in probs]), P(*[p[3].data_ptr() for p in probs]),
                                         I(*[p[4] for p in probs]), I(*[p[5] for p in probs]), M, stream),
                       "rk_mlp3_wgrad")
        else:  # generic MFMA GEMM: dW[n][k] += sum_m dT[n][m] xT[k][m]
            for dT, inT, wbuf, bbuf, n_out, k_in in probs:
                gemm(dT, inT, wbuf, M=n_out, N=k_in, K=M, lda=M, ldb=M, ldc=k_in, accumulate=True, rowsum=bbuf,
                     cfg=0)
        return (dx, *_finish(params, bufs, direct))


class _LeNetFused(torch.autograd.Function):
    """The whole LeNet: conv stack + classifier forward in ONE launch (after a tiny weight-fragment
    prep launch), classifier input-gradient chain + conv backward in ONE launch, the three
    classifier weight gradients in one grouped launch.  Needs N % 8 == 0."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, f1w, f1b, f2w, f2b, f3w, f3b):
        lib = _lib.kernels()
        x = x.contiguous().float()
        N = x.shape[0]
        assert tuple(x.shape[1:]) == (1, 28, 28) and N % 8 == 0, "fused LeNet expects [N,1,28,28], N % 8 == 0"
        dev = x.device
        stream = _lib.stream_ptr(dev)
        cw = [t.detach().float().contiguous() for t in (w1, b1, w2, b2, f1w, f1b, f2w, f2b, f3w, f3b)]
        frag = torch.empty(int(lib.rk_lenet_frag_bytes()), dtype=torch.uint8, device=dev)
        _lib.check(lib.rk_lenet_prep(cw[4].data_ptr(), cw[6].data_ptr(), cw[8].data_ptr(), frag.data_ptr(), stream),
                   "rk_lenet_prep")
        bf = dict(dtype=torch.bfloat16, device=dev)
        a1 = torch.empty(N, 1176, **bf)
        c1 = torch.empty(N, 1176, dtype=torch.uint8, device=dev)
        c2 = torch.empty(N, 400, dtype=torch.uint8, device=dev)
        a2T = torch.empty(400, N, **bf)
        h1T = torch.empty(120, N, **bf)
        h2T = torch.empty(84, N, **bf)
        logits = torch.empty(N, 10, dtype=torch.float32, device=dev)
        _lib.check(lib.rk_lenet_fwd(x.data_ptr(), cw[0].data_ptr(), cw[1].data_ptr(), cw[2].data_ptr(),
                                    cw[3].data_ptr(), frag.data_ptr(), cw[5].data_ptr(), cw[7].data_ptr(),
                                    cw[9].data_ptr(), a1.data_ptr(), c1.data_ptr(), c2.data_ptr(), a2T.data_ptr(),
                                    h1T.data_ptr(), h2T.data_ptr(), logits.data_ptr(), N, stream), "rk_lenet_fwd")
        ctx.params = (w1, b1, w2, b2, f1w, f1b, f2w, f2b, f3w, f3b)
        ctx.save_for_backward(x, a1, c1, c2, a2T, h1T, h2T, frag, cw[2])
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        lib = _lib.kernels()
        x, a1, c1, c2, a2T, h1T, h2T, frag, w2c = ctx.saved_tensors
        N = x.shape[0]
        dev = x.device
        stream = _lib.stream_ptr(dev)
        dy = dlogits.contiguous().float()
        bf = dict(dtype=torch.bfloat16, device=dev)
        dyT = torch.empty(10, N, **bf)
        d2T = torch.empty(84, N, **bf)
        d1T = torch.empty(120, N, **bf)
        params = ctx.params
        bufs, direct = _grad_targets(params, dev)
        rounds = 2 if N % 16 == 0 and N >= 4096 else 1
        _lib.check(lib.rk_lenet_bwd(x.data_ptr(), a1.data_ptr(), c1.data_ptr(), c2.data_ptr(), w2c.data_ptr(),
                                    frag.data_ptr(), dy.data_ptr(), h1T.data_ptr(), h2T.data_ptr(), dyT.data_ptr(),
                                    d2T.data_ptr(), d1T.data_ptr(), bufs[0].data_ptr(), bufs[1].data_ptr(),
                                    bufs[2].data_ptr(), bufs[3].data_ptr(), N, rounds, stream), "rk_lenet_bwd")
        probs = ((dyT, h2T, bufs[8], bufs[9], 10, 84), (d2T, h1T, bufs[6], bufs[7], 84, 120),
                 (d1T, a2T, bufs[4], bufs[5], 120, 400))
        P = ctypes.c_void_p * 3
        I = ctypes.c_int * 3
        _lib.check(lib.rk_mlp3_wgrad(3, P(*[q[0].data_ptr() for q in probs]), P(*[q[1].data_ptr() for q in probs]),
                                     P(*[q[2].data_ptr() for q in probs]), P(*[q[3].data_ptr() for q in probs]),
                                     I(*[q[4] for q in probs]), I(*[q[5] for q in probs]), N, stream),
                   "rk_mlp3_wgrad")
        return (None, *_finish(params, bufs, direct))


def lenet_forward(x, conv1, conv2, fc1, fc2, fc3):
    """Fused LeNet logits (N % 8 == 0)."""
    return _LeNetFused.apply(x, conv1.weight, conv1.bias, conv2.weight, conv2.bias, fc1.weight, fc1.bias,
                             fc2.weight, fc2.bias, fc3.weight, fc3.bias)


def mlp_head(x, layers: List[torch.nn.Linear]):
    (l1, l2, l3) = layers
    return _MLPHead.apply(x, l1.weight, l1.bias, l2.weight, l2.bias, l3.weight, l3.bias)
