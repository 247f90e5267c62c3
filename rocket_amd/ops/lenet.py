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
import os

import torch

from rocket_amd.ops import _lib
from rocket_amd.ops.linear import _direct, gemm, grad_ready


def half_mode(device) -> bool:
    """True under fp16 autocast on ``device``: the fused LeNet then runs its fp16 kernel build
    (``*_h`` entries of lenet_conv_h.hip / mlp_h.hip: fp16 activations, fragments and MFMA
    operands, fp32 accumulation), otherwise bf16."""
    dt = device.type if isinstance(device, torch.device) else str(device)
    return torch.is_autocast_enabled(dt) and torch.get_autocast_dtype(dt) == torch.float16


def _k(lib, name: str, half: bool):
    """The bf16 or fp16 build of a fused-LeNet entry point."""
    return getattr(lib, name + "_h" if half else name)


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
    def forward(ctx, x, w1, b1, w2, b2, half=False):
        lib = _lib.kernels()
        x = x.contiguous().float()
        N = x.shape[0]
        assert tuple(x.shape[1:]) == (1, 28, 28), "lenet_features expects [N,1,28,28]"
        dev = x.device
        dt = torch.float16 if half else torch.bfloat16
        a1 = torch.empty(N, 1176, dtype=dt, device=dev)
        c1 = torch.empty(N, 1176, dtype=torch.uint8, device=dev)
        a2 = torch.empty(N, 400, dtype=dt, device=dev)
        c2 = torch.empty(N, 400, dtype=torch.uint8, device=dev)
        w1c, b1c, w2c, b2c = (t.detach().float().contiguous() for t in (w1, b1, w2, b2))
        _lib.check(_k(lib, "rk_lenet_conv_fwd", half)(x.data_ptr(), w1c.data_ptr(), b1c.data_ptr(), w2c.data_ptr(), b2c.data_ptr(),
                                         a1.data_ptr(), c1.data_ptr(), a2.data_ptr(), c2.data_ptr(), N,
                                         _lib.stream_ptr(dev)), "rk_lenet_conv_fwd")
        ctx.params = (w1, b1, w2, b2)
        ctx.half = half
        ctx.save_for_backward(x, a1, c1, c2, w2c)
        return a2

    @staticmethod
    def backward(ctx, da2):
        lib = _lib.kernels()
        x, a1, c1, c2, w2c = ctx.saved_tensors
        N = x.shape[0]
        da2 = da2.contiguous()
        if da2.dtype != a1.dtype:
            da2 = da2.to(a1.dtype)
        params = ctx.params
        bufs, direct = _grad_targets(params, x.device)
        rounds = max(1, N // 2048)
        _lib.check(_k(lib, "rk_lenet_conv_bwd", ctx.half)(x.data_ptr(), a1.data_ptr(), c1.data_ptr(), da2.data_ptr(), c2.data_ptr(),
                                         w2c.data_ptr(), bufs[0].data_ptr(), bufs[1].data_ptr(), bufs[2].data_ptr(),
                                         bufs[3].data_ptr(), N, rounds, _lib.stream_ptr(x.device)), "rk_lenet_conv_bwd")
        return (None, *_finish(params, bufs, direct), None)


def lenet_features(x, w1, b1, w2, b2):
    return _LeNetFeatures.apply(x, w1, b1, w2, b2, half_mode(x.device))


class _MLPHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w3, b3):
        lib = _lib.kernels()
        x = x.contiguous()
        half = x.dtype == torch.float16  # fp16 features (fp16 autocast) -> fp16 kernel build
        if not half and x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        M, K0 = x.shape
        N1, N2, N3 = w1.shape[0], w2.shape[0], w3.shape[0]
        dev = x.device
        bf = dict(dtype=x.dtype, device=dev)
        xT = torch.empty(K0, M, **bf)
        h1T = torch.empty(N1, M, **bf)
        h2T = torch.empty(N2, M, **bf)
        y = torch.empty(M, N3, dtype=torch.float32, device=dev)
        ws = [t.detach().float().contiguous() for t in (w1, b1, w2, b2, w3, b3)]
        _lib.check(_k(lib, "rk_mlp3_fwd", half)(x.data_ptr(), K0, ws[0].data_ptr(), ws[1].data_ptr(), N1, ws[2].data_ptr(),
                                   ws[3].data_ptr(), N2, ws[4].data_ptr(), ws[5].data_ptr(), N3, xT.data_ptr(),
                                   h1T.data_ptr(), h2T.data_ptr(), y.data_ptr(), M, _lib.stream_ptr(dev)),
                   "rk_mlp3_fwd")
        ctx.params = (w1, b1, w2, b2, w3, b3)
        ctx.half = half
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
        half = ctx.half
        bf = dict(dtype=xT.dtype, device=dev)
        dyT = torch.empty(N3, M, **bf)
        d2T = torch.empty(N2, M, **bf)
        d1T = torch.empty(N1, M, **bf)
        dx = torch.empty(M, K0, **bf) if ctx.needs_input_grad[0] else None
        stream = _lib.stream_ptr(dev)
        _lib.check(_k(lib, "rk_mlp3_dgrad", half)(dy.data_ptr(), N3, w3.data_ptr(), N2, h2T.data_ptr(), w2.data_ptr(), N1,
                                     h1T.data_ptr(), w1.data_ptr(), K0, dyT.data_ptr(), d2T.data_ptr(),
                                     d1T.data_ptr(), _lib.ptr(dx), M, stream), "rk_mlp3_dgrad")
        params = ctx.params
        bufs, direct = _grad_targets(params, dev)
        probs = ((dyT, h2T, bufs[4], bufs[5], N3, N2), (d2T, h1T, bufs[2], bufs[3], N2, N1),
                 (d1T, xT, bufs[0], bufs[1], N1, K0))
        if M % 8 == 0:
            P = ctypes.c_void_p * 3
            I = ctypes.c_int * 3
            _lib.check(_k(lib, "rk_mlp3_wgrad", half)(3, P(*[p[0].data_ptr() for p in probs]), P(*[p[1].data_ptr() for p in probs]),
                                         P(*[p[2].data_ptr() for p in probs]), P(*[p[3].data_ptr() for p in probs]),
                                         I(*[p[4] for p in probs]), I(*[p[5] for p in probs]), M, None, 0, 0, None,
                                         None, stream), "rk_mlp3_wgrad")
        else:  # generic MFMA GEMM: dW[n][k] += sum_m dT[n][m] xT[k][m]
            if half:
                raise NotImplementedError("fused fp16 MLP head needs M % 8 == 0")
            for dT, inT, wbuf, bbuf, n_out, k_in in probs:
                gemm(dT, inT, wbuf, M=n_out, N=k_in, K=M, lda=M, ldb=M, ldc=k_in, accumulate=True, rowsum=bbuf,
                     cfg=0)
        return (dx, *_finish(params, bufs, direct))


# fragment-table geometry (mirror of lenet_conv.hip: OFF_* / NFRAG)
_OFF_F1, _OFF_F2, _OFF_F3, _OFF_B3, _OFF_B2, _OFF_B1 = 0, 104, 128, 131, 137, 161
_OFF_C1, _OFF_C2, _OFF_D2, _NFRAG = 261, 262, 269, 282


def _frag_index_maps():
    """Where every weight element lands in the bf16 fragment table built by ``lenet_prep``.

    Returns int32 arrays [numel, 2] for (fc1.w, fc2.w, fc3.w, conv1.w, conv2.w): column 0 = the
    forward-layout slot, column 1 = the input-gradient-layout slot (-1 where absent); a slot is
    an element index of the table viewed as bf16.  Mirrors lenet_prep_kernel exactly (checked
    bitwise by tests/kernels: optimizer-maintained table == freshly prepped table)."""
    import numpy as np

    shapes = {"f1": (120, 400), "f2": (84, 120), "f3": (10, 84), "c1": (6 * 25,), "c2": (16 * 150,)}
    maps = {k: np.full((int(np.prod(v)), 2), -1, dtype=np.int32) for k, v in shapes.items()}
    lane = np.arange(64)
    lo, hi = lane & 15, lane >> 4
    for f in range(_NFRAG):
        for j in range(8):
            slot = (f * 64 + lane) * 8 + j
            if f >= _OFF_C1:
                if f == _OFF_C1:
                    k = 8 * hi + j
                    kh, kw = k // 6, k % 6
                    ok = (lo < 6) & (k < 30) & (kw < 5)
                    elem, key, col = lo * 25 + kh * 5 + kw, "c1", 0
                elif f < _OFF_D2:
                    kk = 4 * (f - _OFF_C2) + hi
                    ok = (kk < 25) & (j < 6)
                    elem, key, col = (lo * 6 + j) * 25 + kk, "c2", 0
                else:  # plain [kk][ci 8][co 16] dgrad weights, 16-byte unit u = (kk, ci, co half)
                    u = (f - _OFF_D2) * 64 + lane
                    kk, ci, co = u >> 4, (u >> 1) & 7, 8 * (u & 1) + j
                    ok = (kk < 25) & (ci < 6)
                    elem, key, col = (co * 6 + ci) * 25 + kk, "c2", 1
            else:
                if f < _OFF_F2:
                    key, tile, ks, bwd = "f1", (f - _OFF_F1) // 13, (f - _OFF_F1) % 13, 0
                elif f < _OFF_F3:
                    key, tile, ks, bwd = "f2", (f - _OFF_F2) // 4, (f - _OFF_F2) % 4, 0
                elif f < _OFF_B3:
                    key, tile, ks, bwd = "f3", 0, f - _OFF_F3, 0
                elif f < _OFF_B2:
                    key, tile, ks, bwd = "f3", f - _OFF_B3, 0, 1
                elif f < _OFF_B1:
                    key, tile, ks, bwd = "f2", (f - _OFF_B2) // 3, (f - _OFF_B2) % 3, 1
                else:
                    key, tile, ks, bwd = "f1", (f - _OFF_B1) // 4, (f - _OFF_B1) % 4, 1
                nout, nin = shapes[key]
                a = 32 * ks + 8 * hi + j if bwd else 16 * tile + lo
                b = 16 * tile + lo if bwd else 32 * ks + 8 * hi + j
                ok = (a < nout) & (b < nin)
                elem, col = a * nin + b, bwd
            elem = np.broadcast_to(elem, lane.shape)
            maps[key][elem[ok], col] = slot[ok]
    return [maps[k] for k in ("f1", "f2", "f3", "c1", "c2")]


class LeNetFragments:
    """Persistent 16-bit MFMA fragment table of a fused LeNet (one per model and precision: bf16,
    or fp16 under fp16 autocast).

    The table is rebuilt by the ``lenet_prep`` launch only when needed.  It is registered as the
    bf16 shadow of the five weight tensors (``_rocket_bf16_shadow``), so a fused optimizer
    (:mod:`rocket_amd.ops.optim`) rewrites the affected table entries while updating the
    weights, and the next forward skips the prep launch.  Any other writer of the weights bumps
    their autograd version counter, which forces a prep on the next forward."""

    _maps_host = None
    #: speculative whole-step launch (see _LeNetFused); paused after MAX_MISSES unused speculations
    #: in a row (e.g. a plain loss), resumed when a fused cross-entropy is attached again
    SPECULATE = os.environ.get("ROCKET_LENET_SPEC", "1") != "0"
    MAX_MISSES = 2

    def __init__(self, device, half: bool = False):
        lib = _lib.kernels()
        self.half = half
        self.frag = torch.empty(int(lib.rk_lenet_frag_bytes()) // 2, dtype=torch.float16 if half else torch.bfloat16,
                                device=device)
        if LeNetFragments._maps_host is None:
            LeNetFragments._maps_host = _frag_index_maps()
        self.maps = [torch.from_numpy(m).to(device) for m in LeNetFragments._maps_host]
        self.versions = None
        self.params = None
        self.spec_misses = 0
        # the device loss scale (fp16 AMP) the last fused cross-entropy multiplied d(logits) by;
        # the speculative forward launch applies the same one (before any fused cross-entropy:
        # the live fp16 scaler's, runtime/amp.py active_loss_scale)
        self.dev_scale = None
        self.dev_scale_known = False

    @property
    def spec_ok(self) -> bool:
        return self.SPECULATE and self.spec_misses < self.MAX_MISSES

    def ensure(self, fc1w, fc2w, fc3w, conv1w, conv2w, stream) -> torch.Tensor:
        params = (fc1w, fc2w, fc3w, conv1w, conv2w)
        versions = tuple(p._version for p in params)
        # live: the table is the registered shadow of all five weights (a table of the other
        # precision may have registered itself since) and a fused optimizer keeps it current
        live = (self.params is not None and all(a is b for a, b in zip(params, self.params))
                and versions == self.versions
                and all(getattr(p, "_rocket_shadow_live", False)
                        and getattr(p, "_rocket_bf16_shadow", (None, None))[1] is self.frag for p in params))
        if not live:
            cw = [p.detach().float().contiguous() for p in params]
            _lib.check(_k(_lib.kernels(), "rk_lenet_prep", self.half)(cw[0].data_ptr(), cw[1].data_ptr(), cw[2].data_ptr(),
                                                    cw[3].data_ptr(), cw[4].data_ptr(), self.frag.data_ptr(), stream),
                       "rk_lenet_prep")
            for p, m in zip(params, self.maps):
                if p.dtype == torch.float32 and p.is_contiguous() and \
                        getattr(p, "_rocket_bf16_shadow", (None, None))[1] is not self.frag:
                    p._rocket_bf16_shadow = (m, self.frag)  # the fp16 table: an fp16 mapped shadow
                    p._rocket_shadow_live = False  # until a fused optimizer prepares with it
            self.params = params
            self.versions = versions
        return self.frag


class _LenetCE(ctypes.Structure):
    """Mirror of ``struct LenetCE`` (lenet_conv.hip): softmax cross-entropy fused into the backward."""

    _fields_ = [("logits", ctypes.c_void_p), ("target", ctypes.c_void_p), ("ignore_index", ctypes.c_int64),
                ("grad_scale", ctypes.c_float), ("partials", ctypes.c_void_p), ("counter", ctypes.c_void_p),
                ("loss_out", ctypes.c_void_p), ("acc", ctypes.c_void_p), ("ring", ctypes.c_void_p),
                ("slot", ctypes.c_void_p), ("ring_size", ctypes.c_int), ("acc_scale", ctypes.c_float),
                ("sync", ctypes.c_int), ("defer_loss", ctypes.c_int), ("gscale_dev", ctypes.c_void_p)]


class _RowSrc(ctypes.Structure):
    """Mirror of ``struct RowSrc`` (lenet_conv.hip): the batch gathered by the step kernel itself."""

    _fields_ = [("rows", ctypes.c_void_p), ("xsrc", ctypes.c_void_p), ("ysrc", ctypes.c_void_p),
                ("ydst", ctypes.c_void_p), ("target", ctypes.c_void_p), ("keep", ctypes.c_int)]


def _claim_rows(x, target):
    """The deferred device-loader batch ``(x, target)`` (runtime/data.py PendingRows), claimed for
    the step kernel to gather itself: ``(_RowSrc, record)``; None when the batch is an ordinary one
    (or not exactly these two buffers: then it is gathered now).  The weight-gradient launch of the
    step performs the record's cursor advance."""
    from rocket_amd.runtime.data import pending_rows

    p = pending_rows((x, target))
    if p is None:
        return None
    ok = (len(p.bufs) == 2 and p.bufs[0] is x and p.bufs[1] is target and p.n == x.shape[0]
          and p.loader.dataset.tensors[0].dtype == torch.float32
          and p.loader.dataset.tensors[1].dtype == torch.int64
          and tuple(p.loader.dataset.tensors[0].shape[1:]) == (1, 28, 28))
    if not ok:
        p.materialize()
        return None
    (xs, ys), rows = p.claim()
    return _RowSrc(rows.data_ptr(), xs.data_ptr(), ys.data_ptr(), target.data_ptr()), p


class _LossFin(ctypes.Structure):
    """Mirror of ``struct LossFin`` (mlp.hip): the batch loss finalised by the wgrad launch from the
    backward's per-block partials (no last-block ticket at the tail of the backward)."""

    _fields_ = [("partials", ctypes.c_void_p), ("nparts", ctypes.c_int), ("loss_out", ctypes.c_void_p),
                ("acc", ctypes.c_void_p), ("ring", ctypes.c_void_p), ("slot", ctypes.c_void_p),
                ("ring_size", ctypes.c_int), ("acc_scale", ctypes.c_float), ("sync", ctypes.c_int)]


class _TensorRec(ctypes.Structure):
    """Mirror of ``rk_opt::TensorRec`` (optim_common.h)."""

    _fields_ = [(n, ctypes.c_int64) for n in ("p", "g", "s0", "s1", "n", "group", "shadow_map", "shadow_buf")]


class _WgradEpi(ctypes.Structure):
    """Mirror of ``struct WgradEpi`` (mlp.hip): the optimizer update applied by the wgrad launch."""

    _fields_ = [("hyper", ctypes.c_void_p), ("step", ctypes.c_void_p), ("counter", ctypes.c_void_p),
                ("ngroups", ctypes.c_int), ("zero_grads", ctypes.c_int), ("rdw", _TensorRec * 3),
                ("rdb", _TensorRec * 3), ("rsl", _TensorRec * 4)]


def _optimizer_epilogue(params, direct):
    """The armed fused optimizer's update records for the 10 LeNet parameters (or None): the weight-
    gradient launch then applies the step's Adam update as each final gradient element is formed."""
    opt = getattr(params[4], "_rocket_optimizer", None)
    if opt is None or not getattr(opt, "epilogue_armed", False) or not direct:
        return None, None
    spec = opt.epilogue(params)
    if spec is None:
        return None, None
    ngroups, hyper, step, counter, recs = spec
    r = [_TensorRec(*rec) for rec in recs]  # params order: w1 b1 w2 b2 f1w f1b f2w f2b f3w f3b
    epi = _WgradEpi(hyper, step, counter, ngroups, 1, (_TensorRec * 3)(r[8], r[6], r[4]),
                    (_TensorRec * 3)(r[9], r[7], r[5]), (_TensorRec * 4)(r[0], r[1], r[2], r[3]))
    return epi, opt


def _spec_matches(spec, target, dev_scale=None) -> bool:
    t, ver = spec[0], spec[1]
    return (target.data_ptr() == t.data_ptr() and target.shape == t.shape and target.dtype == t.dtype
            and target._version == ver and spec[8] is dev_scale)


class _LeNetFused(torch.autograd.Function):
    """The whole LeNet: conv stack + classifier forward in ONE launch (after a tiny weight-fragment
    prep launch), classifier input-gradient chain + conv backward in ONE launch, the three
    classifier weight gradients in one grouped launch.  Needs N % 8 == 0.

    Training fast path: :func:`fuse_cross_entropy` attaches a mean softmax-cross-entropy to the
    logits' backward node; the backward launch then computes loss and d(logits) itself (the
    incoming gradient is ignored) — forward, loss and backward are 3 launches + the wgrad.

    Speculative whole step (``target`` given, i.e. the model saw the batch's labels, under grad
    mode): the forward launch already runs the cross-entropy and the backward of its block's
    samples (``rk_lenet_train``: no sample's backward depends on another block, so the forward ->
    backward kernel boundary goes), for a unit upstream gradient.  If the loss then attached is
    exactly that cross-entropy on the same targets, the backward only launches the weight-gradient
    kernel, scaled by the loss's gradient scale; otherwise the speculation is dropped (its outputs
    are unused, the regular backward runs on the forward state the kernel also wrote) and, after
    two such misses in a row, paused until a fused cross-entropy is attached again (the engine's
    eager warm-up step uses the plain loss, its captured steps the fused one)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, f1w, f1b, f2w, f2b, f3w, f3b, frags, target=None):
        half = frags.half
        lib = _lib.kernels()
        x = x.contiguous().float()
        N = x.shape[0]
        assert tuple(x.shape[1:]) == (1, 28, 28) and N % 8 == 0, "fused LeNet expects [N,1,28,28], N % 8 == 0"
        dev = x.device
        stream = _lib.stream_ptr(dev)
        cw = [t.detach().float().contiguous() for t in (w1, b1, w2, b2, f1w, f1b, f2w, f2b, f3w, f3b)]
        frag = frags.ensure(f1w, f2w, f3w, w1, w2, stream)
        bf = dict(dtype=torch.float16 if half else torch.bfloat16, device=dev)
        a1 = torch.empty(N, 1176, **bf)
        c1 = torch.empty(N, 1176, dtype=torch.uint8, device=dev)
        c2 = torch.empty(N, 400, dtype=torch.uint8, device=dev)
        a2T = torch.empty(400, N, **bf)
        h1T = torch.empty(120, N, **bf)
        h2T = torch.empty(84, N, **bf)
        logits = torch.empty(N, 10, dtype=torch.float32, device=dev)
        ctx.spec = None
        # (grad mode is off inside Function.forward: whether a backward can follow is needs_input_grad)
        if (target is not None and frags.spec_ok and any(ctx.needs_input_grad[1:11]) and N <= 65536 and target.dim() == 1
                and target.numel() == N and target.dtype == torch.int64 and target.is_contiguous()
                and target.device == dev):
            dyT, d2T, d1T = torch.empty(10, N, **bf), torch.empty(84, N, **bf), torch.empty(120, N, **bf)
            slab = torch.empty(N // 4, int(lib.rk_lenet_slab_width()), dtype=torch.float32, device=dev)
            partials = torch.empty(2 * (N // 4), dtype=torch.float32, device=dev)  # loss sums, valid counts
            loss_out = torch.empty(2, dtype=torch.float32, device=dev)
            if frags.dev_scale_known:
                dscale = frags.dev_scale
            else:
                from rocket_amd.runtime.amp import active_loss_scale

                dscale = active_loss_scale(dev)
            ce = _LenetCE(logits.data_ptr(), target.data_ptr(), -100, 1.0, partials.data_ptr(),
                          _lib.Workspace.get(dev).counter("lenet_ce"), loss_out.data_ptr(), None, None, None, 0,
                          0.0, 0, 1, _lib.ptr(dscale))
            claimed = _claim_rows(x, target)  # a deferred loader batch: this launch gathers it
            rows = claimed[0] if claimed is not None else None
            ctx.rows_pend = claimed[1] if claimed is not None else None
            _lib.check(_k(lib, "rk_lenet_train", half)(x.data_ptr(), cw[1].data_ptr(), cw[3].data_ptr(), frag.data_ptr(),
                                          cw[5].data_ptr(), cw[7].data_ptr(), cw[9].data_ptr(), a1.data_ptr(),
                                          c1.data_ptr(), c2.data_ptr(), a2T.data_ptr(), h1T.data_ptr(), h2T.data_ptr(),
                                          logits.data_ptr(), dyT.data_ptr(), d2T.data_ptr(), d1T.data_ptr(),
                                          slab.data_ptr(), N, ctypes.byref(ce),
                                          ctypes.byref(rows) if rows is not None else None, stream),
                       "rk_lenet_train")
            ctx.spec = (target, target._version, dyT, d2T, d1T, slab, partials, loss_out, dscale)
        else:
            from rocket_amd.runtime.data import materialize_batch

            materialize_batch((x, target) if target is not None else x)  # a deferred loader batch: gather it now
            _lib.check(_k(lib, "rk_lenet_fwd", half)(x.data_ptr(), cw[0].data_ptr(), cw[1].data_ptr(), cw[2].data_ptr(),
                                        cw[3].data_ptr(), frag.data_ptr(), cw[5].data_ptr(), cw[7].data_ptr(),
                                        cw[9].data_ptr(), a1.data_ptr(), c1.data_ptr(), c2.data_ptr(), a2T.data_ptr(),
                                        h1T.data_ptr(), h2T.data_ptr(), logits.data_ptr(), N, stream), "rk_lenet_fwd")
        if ctx.spec is None:
            ctx.rows_pend = None
        ctx.params = (w1, b1, w2, b2, f1w, f1b, f2w, f2b, f3w, f3b)
        ctx.frags = frags
        ctx.save_for_backward(x, a1, c1, c2, a2T, h1T, h2T, frag, cw[2], logits)
        ctx.ce_spec = None
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        lib = _lib.kernels()
        x, a1, c1, c2, a2T, h1T, h2T, frag, w2c, logits = ctx.saved_tensors
        N = x.shape[0]
        dev = x.device
        stream = _lib.stream_ptr(dev)
        rounds = 1  # one block per 4 samples (the kernel keeps no state across sample groups)
        ce, keep, fin, dev_scale = None, None, None, None
        spec, ctx.spec = ctx.spec, None
        gscale = 1.0
        if ctx.ce_spec is not None and spec is not None and _spec_matches(spec, ctx.ce_spec[0], ctx.ce_spec[4]):
            # the forward launch already ran this loss's backward for a unit upstream gradient
            # (times the same device loss scale)
            target, grad_scale, accum, loss_out, dev_scale = ctx.ce_spec
            ctx.ce_spec = None
            _, _, dyT, d2T, d1T, slab, partials, _, _ = spec
            acc = ring = slot = None
            acc_scale, sync = 0.0, 0
            if accum is not None:
                acc, ring, slot, acc_scale, sync = accum
            keep = (partials, target)
            fin = _LossFin(partials.data_ptr(), N // 4, loss_out.data_ptr(), _lib.ptr(acc), _lib.ptr(ring),
                           _lib.ptr(slot), ring.numel() if ring is not None else 0, float(acc_scale), int(sync))
            gscale = float(grad_scale)
            ctx.frags.spec_misses = 0
            return _LeNetFused._wgrad(ctx, lib, N, dev, stream, dyT, d2T, d1T, a2T, h1T, h2T, slab, fin, gscale, keep,
                                      dev_scale)
        if spec is not None:
            ctx.frags.spec_misses += 1  # the loss was not the fused cross-entropy on those targets
            # the whole-step launch kept a1 and the code maps in LDS (no global copies): the
            # regular backward below needs them, so the forward launch recomputes them (same values)
            cw = [p.detach().float().contiguous() for p in ctx.params]
            _lib.check(_k(lib, "rk_lenet_fwd", ctx.frags.half)(
                x.data_ptr(), cw[0].data_ptr(), cw[1].data_ptr(), cw[2].data_ptr(), cw[3].data_ptr(), frag.data_ptr(),
                cw[5].data_ptr(), cw[7].data_ptr(), cw[9].data_ptr(), a1.data_ptr(), c1.data_ptr(), c2.data_ptr(),
                a2T.data_ptr(), h1T.data_ptr(), h2T.data_ptr(), logits.data_ptr(), N, stream), "rk_lenet_fwd")
        if ctx.ce_spec is not None:
            target, grad_scale, accum, loss_out, dev_scale = ctx.ce_spec
            ctx.ce_spec = None
            acc = ring = slot = None
            acc_scale, sync = 0.0, 0
            if accum is not None:
                acc, ring, slot, acc_scale, sync = accum
            partials = torch.empty(2 * (N // 4), dtype=torch.float32, device=dev)  # loss sums, valid counts
            keep = (partials, target)
            ce = _LenetCE(logits.data_ptr(), target.data_ptr(), -100, float(grad_scale), partials.data_ptr(),
                          _lib.Workspace.get(dev).counter("lenet_ce"), loss_out.data_ptr(), _lib.ptr(acc),
                          _lib.ptr(ring), _lib.ptr(slot), ring.numel() if ring is not None else 0, float(acc_scale),
                          int(sync), 1, _lib.ptr(dev_scale))
            fin = _LossFin(partials.data_ptr(), N // 4, loss_out.data_ptr(), _lib.ptr(acc), _lib.ptr(ring),
                           _lib.ptr(slot), ring.numel() if ring is not None else 0, float(acc_scale), int(sync))
            dy = logits  # unread
        else:
            dy = dlogits.contiguous().float()
        bf = dict(dtype=a1.dtype, device=dev)
        dyT = torch.empty(10, N, **bf)
        d2T = torch.empty(84, N, **bf)
        d1T = torch.empty(120, N, **bf)
        # conv weight/bias gradients: one slab row per backward block, summed by the wgrad launch
        slab = torch.empty(N // 4, int(lib.rk_lenet_slab_width()), dtype=torch.float32, device=dev)
        _lib.check(_k(lib, "rk_lenet_bwd", ctx.frags.half)(x.data_ptr(), a1.data_ptr(), c1.data_ptr(), c2.data_ptr(), w2c.data_ptr(),
                                    frag.data_ptr(), dy.data_ptr(), h1T.data_ptr(), h2T.data_ptr(), dyT.data_ptr(),
                                    d2T.data_ptr(), d1T.data_ptr(), slab.data_ptr(), N, rounds,
                                    ctypes.byref(ce) if ce is not None else None, stream), "rk_lenet_bwd")
        return _LeNetFused._wgrad(ctx, lib, N, dev, stream, dyT, d2T, d1T, a2T, h1T, h2T, slab, fin, gscale, keep,
                                  dev_scale)

    @staticmethod
    def _wgrad(ctx, lib, N, dev, stream, dyT, d2T, d1T, a2T, h1T, h2T, slab, fin, gscale, keep, dev_scale=None):
        """The grouped weight-gradient launch (+ loss finalisation, + the armed optimizer's update,
        or under the device fp16 scaler the non-finite check of the gradients it writes)."""
        params = ctx.params
        half = ctx.frags.half
        bufs, direct = _grad_targets(params, dev)
        probs = ((dyT, h2T, bufs[8], bufs[9], 10, 84), (d2T, h1T, bufs[6], bufs[7], 84, 120),
                 (d1T, a2T, bufs[4], bufs[5], 120, 400))
        P = ctypes.c_void_p * 3
        I = ctypes.c_int * 3
        # slab columns [dW1 150 | db1 6 | dW2 2400 | db2 16] -> conv1.weight/bias, conv2.weight/bias
        sizes = [bufs[i].numel() for i in range(4)]
        assert sum(sizes) == int(lib.rk_lenet_slab_cols()), "fused LeNet expects conv1 6x1x5x5 / conv2 16x6x5x5"
        bounds = (ctypes.c_int * 5)(0, sizes[0], sizes[0] + sizes[1], sizes[0] + sizes[1] + sizes[2], sum(sizes))
        epi, opt = _optimizer_epilogue(params, direct)
        amp_opt = None
        amp_state = getattr(dev_scale, "_rocket_amp_state", None) if dev_scale is not None else None
        if epi is None and amp_state is not None and direct:
            o = getattr(params[4], "_rocket_optimizer", None)
            if o is not None and o.amp_fold_target(params):
                amp_opt = o
                found = amp_state[2:3]  # runtime/amp.py FOUND
                _lib.check(_k(lib, "rk_mlp3_set_amp_found", half)(found.data_ptr()), "rk_mlp3_set_amp_found")
        pend, ctx.rows_pend = getattr(ctx, "rows_pend", None), None
        rows_staged = pend is not None and not pend.advanced
        if rows_staged:  # the step's batch cursor, as one more block of this launch
            _lib.check(_k(lib, "rk_mlp3_set_rows", half)(*pend.advance_args()), "rk_mlp3_set_rows")
        _lib.check(_k(lib, "rk_mlp3_wgrad_loss", half)(3, P(*[q[0].data_ptr() for q in probs]), P(*[q[1].data_ptr() for q in probs]),
                                          P(*[q[2].data_ptr() for q in probs]), P(*[q[3].data_ptr() for q in probs]),
                                          I(*[q[4] for q in probs]), I(*[q[5] for q in probs]), N, slab.data_ptr(),
                                          N // 4, slab.shape[1],
                                          (ctypes.c_void_p * 4)(*[bufs[i].data_ptr() for i in range(4)]), bounds,
                                          ctypes.byref(fin) if fin is not None else None,
                                          ctypes.byref(epi) if epi is not None else None, float(gscale),
                                          int(fin is not None), stream),
                   "rk_mlp3_wgrad_loss")
        if rows_staged:
            pend.mark_advanced()  # only once the launch that advances the cursor was accepted
        if opt is not None:
            opt.epilogue_done = True  # the optimizer's own launch for this step is skipped
        if amp_opt is not None:
            amp_opt.amp_checked = True  # the scaler skips its check launch for this step
        del keep  # partials: read by the wgrad launch (stream-ordered before any reuse)
        return (None, *_finish(params, bufs, direct), None, None)


def lenet_forward(x, conv1, conv2, fc1, fc2, fc3, target=None):
    """Fused LeNet logits (N % 8 == 0).  The bf16 fragment table lives on ``conv1``
    (:class:`LeNetFragments`), kept current by a fused optimizer between steps; under fp16
    autocast the fp16 kernel build runs with its own (per-forward) fp16 table."""
    half = half_mode(x.device)
    attr = "_rocket_fragments_h" if half else "_rocket_fragments"
    frags = getattr(conv1, attr, None)
    if frags is None or frags.frag.device != x.device:
        frags = LeNetFragments(x.device, half)
        setattr(conv1, attr, frags)
    return _LeNetFused.apply(x, conv1.weight, conv1.bias, conv2.weight, conv2.bias, fc1.weight, fc1.bias,
                             fc2.weight, fc2.bias, fc3.weight, fc3.bias, frags, target)


def fuse_cross_entropy(logits, target, grad_scale: float, accum=None, dev_scale=None):
    """Attach a mean cross-entropy (ignore_index -100) to fused-LeNet ``logits`` so the backward
    launch computes loss and d(logits) in-kernel.  Returns ``(loss[0-d], dummy_grad)`` to pass to
    ``torch.autograd.backward([logits], [dummy_grad])``, or None if ``logits`` is not a fused-LeNet
    output (or ``N > 65536``).  ``accum`` as in :func:`rocket_amd.ops.cross_entropy.ce_train`.
    ``dev_scale``: optional 1-element fp32 device tensor (the fp16 loss scale) that d(logits) is
    multiplied by in-kernel, as ``scaler.scale(loss).backward()`` would (the loss stays unscaled)."""
    fn = logits.grad_fn
    if (fn is None or type(fn).__name__ != "_LeNetFusedBackward" or logits.dim() != 2 or logits.shape[0] > 65536
            or target.dim() != 1 or target.dtype.is_floating_point):
        return None
    target = target.contiguous().to(torch.int64)
    spec = getattr(fn, "spec", None)
    frags = getattr(fn, "frags", None)
    if frags is not None:
        frags.dev_scale = dev_scale  # the next speculative forward scales d(logits) the same way
        frags.dev_scale_known = True
    if spec is not None and _spec_matches(spec, target, dev_scale):
        loss_out = spec[7]  # the speculative forward launch already wrote this loss's partials
    else:
        loss_out = torch.empty(2, dtype=torch.float32, device=logits.device)
        if frags is not None:
            frags.spec_misses = 0  # the fused loss is in use: speculate on the next forward
    fn.ce_spec = (target, float(grad_scale), accum, loss_out, dev_scale)
    # the incoming gradient is never read (the kernel derives d(logits) itself): no fill launch
    return loss_out[0], torch.empty((), dtype=logits.dtype, device=logits.device).expand_as(logits)


def mlp_head(x, layers: List[torch.nn.Linear]):
    (l1, l2, l3) = layers
    return _MLPHead.apply(x, l1.weight, l1.bias, l2.weight, l2.bias, l3.weight, l3.bias)
