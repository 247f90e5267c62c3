"""BatchNorm (+residual +ReLU) and LayerNorm HIP kernels vs a PyTorch fp32 reference."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("relu,residual", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("shape", [(8, 64, 14, 14), (4, 200, 7, 7), (64, 24, 32, 32)])
def test_batchnorm_act(dtype, relu, residual, shape):
    from rocket_amd.ops.norm import BatchNormAct2d

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    C = shape[1]
    bn = BatchNormAct2d(C, relu=relu).to(dev)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    x32 = (torch.randn(shape, device=dev) * 3 + 1).to(memory_format=torch.channels_last)
    r32 = torch.randn(shape, device=dev).to(memory_format=torch.channels_last) if residual else None
    x = x32.to(dtype).requires_grad_(True)
    r = r32.to(dtype).requires_grad_(True) if residual else None
    y = bn(x, residual=r)
    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    gy = torch.randn_like(y)
    y.backward(gy)

    # fp32 reference on the same (rounded) inputs
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True) if residual else None
    w = bn.weight.detach().clone().requires_grad_(True)
    b = bn.bias.detach().clone().requires_grad_(True)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    ref = F.batch_norm(xr, rm, rv, w, b, training=True, momentum=0.1, eps=1e-5)
    if residual:
        ref = ref + rr
    if relu:
        ref = F.relu(ref)
    ref.backward(gy.float())
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert _rel(y, ref) < tol
    assert _rel(bn.running_mean, rm) < 1e-5 and _rel(bn.running_var, rv) < 1e-4
    assert int(bn.num_batches_tracked) == 1
    gtol = 1e-4 if dtype == torch.float32 else 3e-2
    assert _rel(x.grad, xr.grad) < gtol
    assert _rel(bn.weight.grad, w.grad) < gtol
    assert _rel(bn.bias.grad, b.grad) < gtol
    if residual:
        assert _rel(r.grad, rr.grad) < gtol


@pytest.mark.parametrize("in_dtype,autocast", [(torch.float32, False), (torch.float32, True), (torch.bfloat16, False)])
@pytest.mark.parametrize("C", [768, 256, 100])
def test_layernorm(in_dtype, autocast, C):
    from rocket_amd.ops.norm import FusedLayerNorm

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ln = FusedLayerNorm(C).to(dev)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.5, 0.5)
    x = (torch.randn(3, 197, C, device=dev) * 2 + 0.5).to(in_dtype).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        y = ln(x)
    expect = torch.bfloat16 if (autocast or in_dtype == torch.bfloat16) else torch.float32
    assert y.dtype == expect
    gy = torch.randn(y.shape, device=dev)
    y.backward(gy.to(y.dtype))
    xr = x.detach().float().requires_grad_(True)
    w = ln.weight.detach().clone().requires_grad_(True)
    b = ln.bias.detach().clone().requires_grad_(True)
    ref = F.layer_norm(xr, (C,), w, b, 1e-5)
    ref.backward(gy.to(y.dtype).float())
    tol = 1e-5 if expect == torch.float32 else 1e-2
    assert _rel(y, ref) < tol
    gtol = 1e-4 if in_dtype == torch.float32 and expect == torch.float32 else 3e-2
    assert _rel(x.grad, xr.grad) < gtol
    assert _rel(ln.weight.grad, w.grad) < gtol
    assert _rel(ln.bias.grad, b.grad) < gtol


def test_fused_add_layernorm():
    """(s, y) = (x + r, LN(x + r)) with the residual add fused; gradients of x, r, gamma, beta."""
    from rocket_amd.ops.norm import FusedLayerNorm

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    C = 768
    ln = FusedLayerNorm(C).to(dev)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.5, 0.5)
    x = torch.randn(2, 197, C, device=dev).requires_grad_(True)
    r = torch.randn(2, 197, C, device=dev).to(torch.bfloat16).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        s, y = ln.add_forward(x, r)
    assert s.dtype == torch.float32 and y.dtype == torch.bfloat16
    gs, gy = torch.randn_like(s), torch.randn(y.shape, device=dev).to(torch.bfloat16)
    torch.autograd.backward([s, y], [gs, gy])
    xr = x.detach().clone().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True)
    w = ln.weight.detach().clone().requires_grad_(True)
    b = ln.bias.detach().clone().requires_grad_(True)
    sr = xr + rr
    yr = F.layer_norm(sr, (C,), w, b, 1e-5)
    torch.autograd.backward([sr, yr], [gs, gy.float()])
    assert _rel(s, sr) < 1e-6 and _rel(y, yr) < 1e-2
    assert _rel(x.grad, xr.grad) < 1e-2 and _rel(r.grad, rr.grad) < 1e-2
    assert _rel(ln.weight.grad, w.grad) < 3e-2 and _rel(ln.bias.grad, b.grad) < 3e-2


@pytest.mark.parametrize("bwd", ["fused", "stream", "split"])
@pytest.mark.parametrize("B,L,H", [(2, 197, 12), (3, 50, 4), (1, 224, 2), (2, 17, 3), (2, 208, 2)])
def test_fused_attention_qkv(B, L, H, bwd):
    """Fused MFMA attention (fwd + dQ/dK/dV) vs fp32 softmax attention on the same bf16 inputs, with
    the one-kernel backward (dQ reduced over key-tile waves in LDS) and the two-kernel backward."""
    from rocket_amd.ops import _lib
    from rocket_amd.ops.activation import _attn_lib, attention_qkv

    _attn_lib()
    _lib.kernels().rk_attn_set_bwd_fused({"split": 0, "fused": 1, "stream": 2}[bwd])

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    D = 64
    qkv = (torch.randn(B, L, 3 * H * D, device=dev) * 1.5).to(torch.bfloat16).requires_grad_(True)
    o = attention_qkv(qkv, H)
    g = torch.randn_like(o)
    o.backward(g)
    ref_in = qkv.detach().float().requires_grad_(True)
    t = ref_in.view(B, L, 3, H, D).permute(2, 0, 3, 1, 4)
    p = torch.softmax(t[0] @ t[1].transpose(-2, -1) / D ** 0.5, dim=-1)
    ref = (p @ t[2]).transpose(1, 2).reshape(B, L, H * D)
    ref.backward(g.float())
    assert o.shape == (B, L, H * D)
    assert _rel(o, ref) < 1.5e-2, _rel(o, ref)
    gq, gr = qkv.grad.view(B, L, 3, H * D), ref_in.grad.view(B, L, 3, H * D)
    _lib.kernels().rk_attn_set_bwd_fused(1)
    for i, name in enumerate("qkv"):
        assert _rel(gq[:, :, i], gr[:, :, i]) < 3e-2, (name, _rel(gq[:, :, i], gr[:, :, i]))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(8, 64, 28, 28), (4, 32, 15, 15), (2, 256, 9, 10)])
def test_batchnorm_relu_maxpool(dtype, shape):
    """The ResNet stem's BN + ReLU + max_pool2d(3, 2, 1) as one pass (norm.hip bn_relu_maxpool) and its
    gather-form backward, against the fp32 composition of the three torch ops."""
    from rocket_amd.ops.norm import BatchNormAct2d

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    C = shape[1]
    bn = BatchNormAct2d(C, relu=True, maxpool=True).to(dev)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    x = (torch.randn(shape, device=dev) * 2 + 0.5).to(memory_format=torch.channels_last).to(dtype).requires_grad_(True)
    y = bn(x)
    OH, OW = (shape[2] - 1) // 2 + 1, (shape[3] - 1) // 2 + 1
    assert y.shape == (shape[0], C, OH, OW) and y.dtype == dtype
    gy = torch.randn_like(y)
    y.backward(gy)

    xr = x.detach().float().requires_grad_(True)
    w = bn.weight.detach().clone().requires_grad_(True)
    b = bn.bias.detach().clone().requires_grad_(True)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    ref = F.max_pool2d(F.relu(F.batch_norm(xr, rm, rv, w, b, training=True, momentum=0.1, eps=1e-5)), 3, 2, 1)
    ref.backward(gy.float())
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert _rel(y, ref) < tol
    assert _rel(bn.running_mean, rm) < 1e-5 and _rel(bn.running_var, rv) < 1e-4
    gtol = 1e-4 if dtype == torch.float32 else 3e-2
    assert _rel(x.grad, xr.grad) < gtol
    assert _rel(bn.weight.grad, w.grad) < gtol
    assert _rel(bn.bias.grad, b.grad) < gtol


def _set_grads(params, direct):
    """Fresh gradients: None, or persistent fp32 .grad buffers the kernels accumulate into (the
    engine's direct-gradient mode), pre-filled so accumulation (not overwrite) is checked."""
    for p in params:
        if direct:
            p.grad = torch.full(p.shape, 0.25, dtype=torch.float32, device=p.device)
            p._rocket_direct_grad = True
        else:
            p.grad = None
            p._rocket_direct_grad = False


@pytest.mark.parametrize("direct", [False, True])
@pytest.mark.parametrize("mlp", [False, True])
def test_add_ln_forms_branch_bias_grad(mlp, direct):
    """A linear branch (MLinear / MMlp) feeding a fused add-LayerNorm: the LN backward forms the
    branch's bias gradient (column sums of dr, BiasLink) and the linear skips its own pass; all
    gradients equal the stock-torch composition.  direct: persistent fp32 grads, where the LN
    kernel adds the sums into bias.grad itself."""
    import rocket_amd.ops as ops
    import rocket_amd.ops.mlinear as ml
    from rocket_amd.ops.norm import FusedLayerNorm

    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    C = 128
    branch = (ml.MMlp(C, 4 * C) if mlp else ml.MLinear(C, C)).to(dev)
    ln = FusedLayerNorm(C).to(dev)
    with torch.no_grad():
        for p in list(branch.parameters()) + list(ln.parameters()):
            p.add_(torch.randn_like(p) * 0.1)
    x0 = torch.randn(4, 50, C, device=dev)
    h0 = torch.randn(4, 50, C, device=dev)
    gy = torch.randn(4, 50, C, device=dev)
    gs = torch.randn(4, 50, C, device=dev)
    grads = []
    for fused in (True, False):
        ops.set_fused(fused)
        try:
            _set_grads(list(branch.parameters()) + list(ln.parameters()), direct)
            hits = ml.BIAS_LINK_HITS
            x, h = x0.clone().requires_grad_(), h0.clone().requires_grad_()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                s, y = ln.add_forward(x, branch(h))
            ((y.float() * gy).sum() + (s.float() * gs).sum()).backward()
            torch.cuda.synchronize()
            grads.append(([p.grad.float().clone() for p in branch.parameters()], h.grad.float(), x.grad.float(),
                          ml.BIAS_LINK_HITS - hits))
        finally:
            ops.set_fused(True)
    (gn, hn, xn, hits), (gt, ht, xt, _) = grads
    assert hits == 1
    for a, b in zip(gn, gt):
        assert _rel(a, b) < 3e-2, _rel(a, b)
    assert _rel(hn, ht) < 3e-2 and _rel(xn, xt) < 3e-2


@pytest.mark.parametrize("direct", [False, True])
def test_bias_link_refused_with_second_consumer(direct):
    """The linear's output feeds the add-LayerNorm AND another op: the incoming gradient is dr plus
    that op's gradient, so the LN's column sums of dr are not the bias gradient.  The link must be
    refused (no hit) and the bias gradient must still equal the stock-torch composition (direct:
    the sums the LN kernel already added into bias.grad are backed out)."""
    import rocket_amd.ops as ops
    import rocket_amd.ops.mlinear as ml
    from rocket_amd.ops.norm import FusedLayerNorm

    dev = torch.device("cuda", 0)
    torch.manual_seed(2)
    C = 128
    branch = ml.MLinear(C, C).to(dev)
    ln = FusedLayerNorm(C).to(dev)
    x0 = torch.randn(4, 50, C, device=dev)
    h0 = torch.randn(4, 50, C, device=dev)
    gy = torch.randn(4, 50, C, device=dev)
    gs = torch.randn(4, 50, C, device=dev)
    gz = torch.randn(4, 50, C, device=dev)
    grads = []
    for fused in (True, False):
        ops.set_fused(fused)
        try:
            _set_grads(list(branch.parameters()) + list(ln.parameters()), direct)
            hits = ml.BIAS_LINK_HITS
            x, h = x0.clone().requires_grad_(), h0.clone().requires_grad_()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                r = branch(h)
                s, y = ln.add_forward(x, r)
                z = r.float() * 3.0  # second consumer of the linear's output
            ((y.float() * gy).sum() + (s.float() * gs).sum() + (z * gz).sum()).backward()
            torch.cuda.synchronize()
            grads.append(([p.grad.float().clone() for p in branch.parameters()], ml.BIAS_LINK_HITS - hits))
        finally:
            ops.set_fused(True)
    (gn, hits), (gt, _) = grads
    assert hits == 0
    for a, b in zip(gn, gt):
        assert _rel(a, b) < 3e-2, _rel(a, b)
