"""Native implicit-GEMM convolutions (conv.hip via ops/iconv.py) vs the fp32 PyTorch conv of the
same bf16-rounded operands, at every distinct ResNet-18 (CIFAR) / ResNet-50 conv shape the
native path takes (batch reduced to keep the test short; the kernels' indexing does not depend
on it beyond the pixel count)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

# (N, Cin, H, W, Cout, k, stride)
SHAPES = [
    # ResNet-50 (ImageNet 224): bottleneck 1x1 / 3x3 / 1x1 and the strided 3x3 / 1x1 downsamples
    (4, 64, 56, 56, 64, 1, 1), (4, 64, 56, 56, 64, 3, 1), (4, 64, 56, 56, 256, 1, 1), (4, 256, 56, 56, 64, 1, 1),
    (4, 128, 56, 56, 128, 3, 2), (4, 256, 56, 56, 512, 1, 2), (4, 128, 28, 28, 128, 3, 1),
    (4, 512, 28, 28, 128, 1, 1), (4, 256, 14, 14, 256, 3, 1), (4, 1024, 14, 14, 256, 1, 1),
    (4, 512, 7, 7, 512, 3, 1), (4, 2048, 7, 7, 512, 1, 1), (4, 512, 14, 14, 512, 3, 2),
    # ResNet-18 CIFAR (32x32)
    (8, 64, 32, 32, 64, 3, 1), (8, 64, 32, 32, 128, 3, 2), (8, 128, 16, 16, 128, 3, 1), (8, 256, 8, 8, 256, 3, 1),
    (8, 256, 4, 4, 512, 1, 2), (8, 512, 4, 4, 512, 3, 1),
    # strided input gradients on odd extents / wider kernels (parity classes of unequal size)
    (2, 64, 15, 15, 128, 3, 2), (2, 64, 15, 13, 128, 1, 2), (2, 64, 9, 11, 64, 7, 2), (2, 128, 7, 7, 64, 5, 2),
]


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("N,Cin,H,W,Cout,k,stride", SHAPES)
def test_iconv_fwd_bwd(N, Cin, H, W, Cout, k, stride):
    from rocket_amd.ops.iconv import IConv2d

    torch.manual_seed(0)
    conv = IConv2d(Cin, Cout, k, stride=stride, padding=k // 2, bias=False).cuda()
    conv = conv.to(memory_format=torch.channels_last)
    x = torch.randn(N, Cin, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = conv(x)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_()
    yr = F.conv2d(xr, wr, stride=stride, padding=k // 2)
    yr.backward(g.float())
    assert _rel(y, yr) < 1e-2, _rel(y, yr)
    assert _rel(x.grad, xr.grad) < 1e-2, _rel(x.grad, xr.grad)
    assert _rel(conv.weight.grad, wr.grad) < 2e-3, _rel(conv.weight.grad, wr.grad)


def test_iconv_wgrad_accumulates_into_persistent_grad():
    from rocket_amd.ops.iconv import IConv2d

    torch.manual_seed(1)
    conv = IConv2d(64, 64, 3, padding=1, bias=False).cuda().to(memory_format=torch.channels_last)
    conv.weight.grad = torch.ones_like(conv.weight)
    conv.weight._rocket_direct_grad = True
    x = torch.randn(2, 64, 20, 20, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = conv(x)
    g = torch.randn_like(y)
    y.backward(g)
    wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_()
    F.conv2d(x.float(), wr, padding=1).backward(g.float())
    assert _rel(conv.weight.grad - 1, wr.grad) < 2e-3


@pytest.mark.parametrize("N,Cin,H,W,Cout,k,stride", [(4, 64, 56, 56, 64, 3, 1), (3, 128, 14, 14, 256, 1, 1),
                                                     (8, 256, 7, 7, 512, 3, 2)])
def test_conv_emitted_bn_stats_match_bn(N, Cin, H, W, Cout, k, stride):
    """BatchNorm statistics merged from the conv epilogue's tile partials (rk_bn_finalize) equal
    the BatchNorm of the stored bf16 conv output (fp32 torch batch_norm reference)."""
    from rocket_amd.ops.iconv import IConv2d
    from rocket_amd.ops.norm import BatchNormAct2d

    torch.manual_seed(3)
    conv = IConv2d(Cin, Cout, k, stride=stride, padding=k // 2, bias=False).cuda().to(memory_format=torch.channels_last)
    conv.emit_bn_stats = True
    bn = BatchNormAct2d(Cout, relu=True).cuda()
    ref = torch.nn.BatchNorm2d(Cout).cuda()
    x = (torch.randn(N, Cin, H, W, device="cuda") + 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = conv(x)
        assert getattr(y, "_rocket_bn_partials", None) is not None
        out = bn(y)
    want = torch.relu(ref(y.float()))
    assert _rel(out, want) < 1e-2, _rel(out, want)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(bn.running_var, ref.running_var, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("k,stride", [(3, 1), (3, 2), (1, 2)])
def test_conv_dgrad_accumulate(k, stride):
    """rk_conv_dgrad with accumulate=1 adds the input gradient onto what dX already holds (the
    residual-branch gradient of a ResNet block entry)."""
    from rocket_amd.ops import _lib

    torch.manual_seed(1)
    N, C, H, W, Co = 2, 64, 14, 14, 128
    pad = k // 2
    OH = (H + 2 * pad - k) // stride + 1
    w = torch.randn(Co, C, k, k, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, Co, OH, OH, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    base = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dx = base.clone()
    _lib.check(_lib.kernels().rk_conv_dgrad(1, dy.data_ptr(), w.data_ptr(), dx.data_ptr(), 1, 1, N, H, W, C, Co, k, k,
                                            stride, pad, OH, OH, _lib.stream_ptr(dy.device)), "rk_conv_dgrad")
    want = base.float() + torch.nn.grad.conv2d_input((N, C, H, W), w.float(), dy.float(), stride=stride, padding=pad)
    assert _rel(dx, want) < 1e-2


@pytest.mark.parametrize("kind,cin,width,stride", [("bottleneck", 256, 64, 1), ("bottleneck", 256, 128, 2),
                                                   ("basic", 64, 64, 1), ("basic", 64, 128, 2)])
def test_block_entry_matches_separate(monkeypatch, kind, cin, width, stride):
    """A residual block whose first conv + shortcut form one autograd node (_EntryFn) has the same
    gradients as with separate nodes (autograd's add of the two input gradients)."""
    import rocket_amd.ops.iconv as ic
    from rocket_amd.models.resnet import BasicBlock, Bottleneck

    torch.manual_seed(2)
    blk = (Bottleneck if kind == "bottleneck" else BasicBlock)(cin, width, stride).cuda()
    blk = blk.to(memory_format=torch.channels_last)
    x0 = torch.randn(4, cin, 16, 16, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    for entry in (True, False):
        monkeypatch.setattr(ic, "ENTRY", entry)
        blk.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = blk(x)
        torch.manual_seed(3)
        g = torch.randn(y.shape, device="cuda").to(y.dtype).contiguous(memory_format=torch.channels_last)
        y.backward(g)
        outs.append((y.detach().float(), x.grad.float(), [p.grad.float().clone() for p in blk.parameters()]))
    (y1, dx1, g1), (y2, dx2, g2) = outs
    assert _rel(y1, y2) < 1e-3
    assert _rel(dx1, dx2) < 1e-2, _rel(dx1, dx2)
    for a, b in zip(g1, g2):
        assert _rel(a, b) < 1e-2


def _tail_counts():
    import ctypes

    from rocket_amd.ops import _lib

    out = (ctypes.c_int64 * 2)()
    _lib.kernels().rk_conv_tail_counts(ctypes.cast(out, ctypes.c_void_p))
    return out[0], out[1]


@pytest.mark.parametrize("kind", ["bottleneck", "basic"])
def test_wgrad_combine_in_dgrad_launch(monkeypatch, kind):
    """The weight gradients' split-K combine run by blocks appended to the following dgrad launch
    (conv.hip TailJob, iconv DEFER_REDUCE) gives bit-identical gradients to its own mgemm_reduce
    launch (same per-element summation order), through plain convs and block entries with identity
    and strided shortcuts; every deferred combine is taken by a dgrad launch or flushed."""
    import rocket_amd.ops.iconv as ic
    from rocket_amd.models.resnet import BasicBlock, Bottleneck
    from rocket_amd.ops.norm import BatchNormAct2d

    torch.manual_seed(6)
    if kind == "bottleneck":
        net = torch.nn.Sequential(BatchNormAct2d(256, relu=True), Bottleneck(256, 64, 1), Bottleneck(256, 128, 2))
        cin = 256
    else:
        net = torch.nn.Sequential(BatchNormAct2d(64, relu=True), BasicBlock(64, 64, 1), BasicBlock(64, 128, 2))
        cin = 64
    net = net.cuda().to(memory_format=torch.channels_last)
    x0 = torch.randn(32, cin, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    for defer in (True, False):
        monkeypatch.setattr(ic, "DEFER_REDUCE", defer)
        net.zero_grad(set_to_none=True)
        c0 = _tail_counts()
        x = x0.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = net(x)
        torch.manual_seed(7)
        g = torch.randn(y.shape, device="cuda").to(y.dtype).contiguous(memory_format=torch.channels_last)
        y.backward(g)
        torch.cuda.synchronize()
        c1 = _tail_counts()
        outs.append((x.grad.float(), [p.grad.float().clone() for p in net.parameters()],
                     (c1[0] - c0[0], c1[1] - c0[1])))
    (dx1, g1, (att, fl)), (dx2, g2, (att0, fl0)) = outs
    assert att >= 2 and att0 == 0 and fl0 == 0, (att, fl, att0, fl0)
    assert torch.equal(dx1, dx2)
    for a, b in zip(g1, g2):
        assert torch.equal(a, b)


@pytest.mark.parametrize("kind", ["bottleneck", "basic"])
def test_bn_backward_reduction_in_dgrad_epilogue(monkeypatch, kind):
    """BatchNorm backward reductions done by the consuming stride-1 conv's dgrad epilogue
    (rk_conv_dgrad_bn + rk_bn_bwd_partials) give the gradients of the two-pass BN backward, through
    plain convs, block entries with identity / strided shortcuts, and strided convs (fallback)."""
    import rocket_amd.ops.norm as nm
    from rocket_amd.models.resnet import BasicBlock, Bottleneck
    from rocket_amd.ops.norm import BatchNormAct2d

    torch.manual_seed(4)
    if kind == "bottleneck":
        net = torch.nn.Sequential(BatchNormAct2d(256, relu=True), Bottleneck(256, 64, 1), Bottleneck(256, 128, 2),
                                  Bottleneck(512, 128, 1))
        cin = 256
    else:
        net = torch.nn.Sequential(BatchNormAct2d(64, relu=True), BasicBlock(64, 64, 1), BasicBlock(64, 128, 2),
                                  BasicBlock(128, 128, 1))
        cin = 64
    net = net.cuda().to(memory_format=torch.channels_last)
    for m in net.modules():  # non-trivial affine parameters (the zero-init residual BN too)
        if isinstance(m, BatchNormAct2d):
            with torch.no_grad():
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    state = {k: v.clone() for k, v in net.state_dict().items()}
    x0 = torch.randn(4, cin, 16, 16, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    import rocket_amd.ops.iconv as ic

    monkeypatch.setattr(ic, "BN_FOLD", False)  # the folded pairs need no link (test_bn_fold_matches_unfused)
    for fuse in (True, False):
        net.load_state_dict(state)
        monkeypatch.setattr(nm, "BWD_FUSE", fuse)
        hits0 = nm.LINK_HITS
        net.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = net(x)
        torch.manual_seed(5)
        g = torch.randn(y.shape, device="cuda").to(y.dtype).contiguous(memory_format=torch.channels_last)
        y.backward(g)
        torch.cuda.synchronize()
        outs.append((y.detach().float(), x.grad.float(), [p.grad.float().clone() for p in net.parameters()],
                     nm.LINK_HITS - hits0))
    (y1, dx1, g1, hits), (y2, dx2, g2, nohits) = outs
    assert nohits == 0 and hits >= (7 if kind == "bottleneck" else 4), hits
    assert _rel(y1, y2) < 1e-3
    assert _rel(dx1, dx2) < 2e-2, _rel(dx1, dx2)
    for a, b in zip(g1, g2):
        assert _rel(a, b) < 2e-2, _rel(a, b)


@pytest.mark.parametrize("kind", ["bottleneck", "basic"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_bn_fold_matches_unfused(monkeypatch, kind, dtype):
    """BatchNorm(+ReLU) folded into the consuming conv (conv.hip BatchNorm-apply prologue on the
    forward / wgrad operand, ReLU mask recomputed in the dgrad epilogue) equals the separate
    BatchNorm + conv: outputs, input / parameter gradients and running statistics, through identity
    and strided blocks (the stride-2 consumers stay unfolded)."""
    import rocket_amd.ops.iconv as ic
    from rocket_amd.models.resnet import BasicBlock, Bottleneck
    from rocket_amd.ops.norm import BatchNormAct2d

    torch.manual_seed(6)
    if kind == "bottleneck":
        net = torch.nn.Sequential(BatchNormAct2d(256, relu=True), Bottleneck(256, 64, 1), Bottleneck(256, 128, 2),
                                  Bottleneck(512, 128, 1))
        cin, want_hits = 256, 5
    else:
        net = torch.nn.Sequential(BatchNormAct2d(64, relu=True), BasicBlock(64, 64, 1), BasicBlock(64, 128, 2),
                                  BasicBlock(128, 128, 1))
        cin, want_hits = 64, 3
    net = net.cuda().to(memory_format=torch.channels_last)
    for m in net.modules():
        if isinstance(m, BatchNormAct2d):
            with torch.no_grad():
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    state = {k: v.clone() for k, v in net.state_dict().items()}
    x0 = torch.randn(4, cin, 16, 16, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    outs = []
    for fold in (True, False):
        net.load_state_dict(state)
        monkeypatch.setattr(ic, "BN_FOLD", fold)
        hits0 = ic.FOLD_HITS
        net.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_()
        with torch.autocast("cuda", dtype=dtype):
            y = net(x)
        torch.manual_seed(7)
        g = torch.randn(y.shape, device="cuda").to(y.dtype).contiguous(memory_format=torch.channels_last)
        y.backward(g)
        torch.cuda.synchronize()
        bufs = {k: v.float().clone() for k, v in net.state_dict().items() if "running" in k}
        outs.append((y.detach().float(), x.grad.float(), [p.grad.float().clone() for p in net.parameters()], bufs,
                     ic.FOLD_HITS - hits0))
    (y1, dx1, g1, b1, hits), (y2, dx2, g2, b2, nohits) = outs
    assert nohits == 0 and hits == want_hits, hits
    assert _rel(y1, y2) < 1e-3, _rel(y1, y2)
    assert _rel(dx1, dx2) < 1e-2, _rel(dx1, dx2)
    for a, b in zip(g1, g2):
        assert _rel(a, b) < 1e-2, _rel(a, b)
    for k in b1:
        torch.testing.assert_close(b1[k], b2[k], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("R,stride,pad,H", [(7, 2, 3, 32), (3, 1, 1, 16)])
@pytest.mark.parametrize("layout", ["nchw", "nhwc"])
def test_stem_conv_vs_fp32(R, stride, pad, H, layout):
    """Native stem conv (Cin = 3 padded to 8 channels, rk_conv_fwd_c8 forward with BatchNorm
    partials, wgrad on the padded image) vs fp32 F.conv2d, the ImageNet 7x7/s2 and CIFAR 3x3 stems."""
    from rocket_amd.ops.iconv import IConv2d, TILE_ROWS

    torch.manual_seed(5)
    conv = IConv2d(3, 64, R, stride=stride, padding=pad, bias=False).cuda()
    conv.emit_bn_stats = True
    x = torch.randn(4, 3, H, H, device="cuda").to(torch.bfloat16)
    if layout == "nhwc":
        x = x.contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = conv(x)
    ref = F.conv2d(x.float(), conv.weight.float(), stride=stride, padding=pad)
    assert _rel(y, ref) < 1e-2
    part, ntiles, rows = y._rocket_bn_partials
    assert rows == TILE_ROWS
    s1 = part.view(ntiles, 2, 64)[:, 0].sum(0)
    torch.testing.assert_close(s1, y.float().sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    g = torch.randn(y.shape, device="cuda").to(torch.bfloat16)
    y.backward(g)
    wref = torch.nn.grad.conv2d_weight(x.float(), conv.weight.shape, g.float(), stride=stride, padding=pad)
    assert _rel(conv.weight.grad, wref) < 1e-2
