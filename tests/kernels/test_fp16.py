"""fp16 autocast on the native kernels: implicit-GEMM convs (MFMA f16), the stem conv, the fused
BatchNorm (+ReLU, +residual) passes and the BatchNorm-backward reduction in the conv dgrad epilogue,
each against the fp32 PyTorch op of the same fp16-rounded operands; and a whole ResNet-18 fp16
training step whose kernel trace holds no MIOpen kernels (the reference passes fp16 through
``Accelerator(mixed_precision="fp16")``, ``/root/reference/rocket/core/launcher.py:185-193``)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

H16 = torch.float16


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("N,Cin,H,W,Cout,k,stride", [
    (4, 64, 56, 56, 64, 3, 1), (4, 256, 28, 28, 64, 1, 1), (4, 128, 28, 28, 128, 3, 2), (4, 256, 14, 14, 512, 1, 2),
    (8, 64, 32, 32, 128, 3, 2), (8, 512, 4, 4, 512, 3, 1), (2, 64, 15, 13, 128, 1, 2),
])
def test_iconv_fp16_vs_fp32(N, Cin, H, W, Cout, k, stride):
    from rocket_amd.ops.iconv import IConv2d

    torch.manual_seed(0)
    conv = IConv2d(Cin, Cout, k, stride=stride, padding=k // 2, bias=False).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(N, Cin, H, W, device="cuda").to(H16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    with torch.autocast("cuda", dtype=H16):
        y = conv(x)
    assert y.dtype == H16 and y.is_contiguous(memory_format=torch.channels_last)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    wr = conv.weight.detach().to(H16).float().requires_grad_()
    F.conv2d(xr, wr, stride=stride, padding=k // 2).backward(g.float())
    yr = F.conv2d(xr.detach(), wr.detach(), stride=stride, padding=k // 2)
    # fp16 keeps 10 mantissa bits (bf16: 7): tighter than the bf16 tests' 1e-2
    assert _rel(y, yr) < 3e-3, _rel(y, yr)
    assert _rel(x.grad, xr.grad) < 3e-3, _rel(x.grad, xr.grad)
    assert _rel(conv.weight.grad, wr.grad) < 1e-3, _rel(conv.weight.grad, wr.grad)


def test_stem_fp16_vs_fp32():
    from rocket_amd.ops.iconv import IConv2d

    torch.manual_seed(5)
    conv = IConv2d(3, 64, 7, stride=2, padding=3, bias=False).cuda()
    conv.emit_bn_stats = True
    x = torch.randn(4, 3, 32, 32, device="cuda").to(H16)
    with torch.autocast("cuda", dtype=H16):
        y = conv(x)
    assert y.dtype == H16
    ref = F.conv2d(x.float(), conv.weight.detach().to(H16).float(), stride=2, padding=3)
    assert _rel(y, ref) < 3e-3
    part, ntiles, _ = y._rocket_bn_partials
    torch.testing.assert_close(part.view(ntiles, 2, 64)[:, 0].sum(0), y.float().sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    g = torch.randn(y.shape, device="cuda").to(H16)
    y.backward(g)
    wref = torch.nn.grad.conv2d_weight(x.float(), conv.weight.shape, g.float(), stride=2, padding=3)
    assert _rel(conv.weight.grad, wref) < 3e-3


@pytest.mark.parametrize("residual", [False, True])
def test_batchnorm_act_fp16_vs_fp32(residual):
    from rocket_amd.ops.norm import BatchNormAct2d

    torch.manual_seed(1)
    C = 128
    bn = BatchNormAct2d(C, relu=True).cuda()
    ref = torch.nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
        ref.weight.copy_(bn.weight)
        ref.bias.copy_(bn.bias)
    x = (torch.randn(8, C, 14, 14, device="cuda") * 2 + 0.5).to(H16).contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x) if residual else None
    xa = x.clone().requires_grad_()
    y = bn(xa, r)
    assert y.dtype == H16
    xr = x.float().requires_grad_()
    yr = torch.relu(ref(xr) + (r.float() if residual else 0))
    assert _rel(y, yr) < 3e-3, _rel(y, yr)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g.float())
    assert _rel(xa.grad, xr.grad) < 5e-3, _rel(xa.grad, xr.grad)
    assert _rel(bn.weight.grad, ref.weight.grad) < 3e-3
    assert _rel(bn.bias.grad, ref.bias.grad) < 3e-3
    torch.testing.assert_close(bn.running_mean, ref.running_mean, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(bn.running_var, ref.running_var, rtol=1e-3, atol=1e-4)


def test_bn_backward_in_dgrad_epilogue_fp16(monkeypatch):
    """fp16 BatchNorm -> conv: the conv's dgrad epilogue does the BatchNorm's backward reduction
    (BwdLink) and the gradients equal the unfused fp16 path's."""
    import rocket_amd.ops.norm as nm
    from rocket_amd.models.resnet import BasicBlock
    from rocket_amd.ops.norm import BatchNormAct2d

    torch.manual_seed(4)
    net = torch.nn.Sequential(BatchNormAct2d(64, relu=True), BasicBlock(64, 64, 1), BasicBlock(64, 128, 2))
    net = net.cuda().to(memory_format=torch.channels_last)
    state = {k: v.clone() for k, v in net.state_dict().items()}
    x0 = torch.randn(4, 64, 16, 16, device="cuda").to(H16).contiguous(memory_format=torch.channels_last)
    import rocket_amd.ops.iconv as ic

    monkeypatch.setattr(ic, "BN_FOLD", False)  # folded pairs need no link (test_iconv.py test_bn_fold_matches_unfused)
    outs = []
    for fuse in (True, False):
        net.load_state_dict(state)
        monkeypatch.setattr(nm, "BWD_FUSE", fuse)
        hits0 = nm.LINK_HITS
        net.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_()
        with torch.autocast("cuda", dtype=H16):
            y = net(x)
        assert y.dtype == H16
        torch.manual_seed(5)
        g = torch.randn(y.shape, device="cuda").to(H16).contiguous(memory_format=torch.channels_last)
        y.backward(g)
        torch.cuda.synchronize()
        outs.append((y.detach().float(), x.grad.float(), [p.grad.float().clone() for p in net.parameters()],
                     nm.LINK_HITS - hits0))
    (y1, dx1, g1, hits), (y2, dx2, g2, nohits) = outs
    assert nohits == 0 and hits >= 2, hits
    assert _rel(y1, y2) < 1e-3
    assert _rel(dx1, dx2) < 1e-2, _rel(dx1, dx2)
    for a, b in zip(g1, g2):
        assert _rel(a, b) < 1e-2, _rel(a, b)


def test_resnet18_fp16_step_has_no_miopen_kernels():
    """One ResNet-18 (CIFAR) fp16 training step: every conv and BatchNorm is a native kernel."""
    from torch.profiler import ProfilerActivity, profile

    from rocket_amd.models import resnet18
    from rocket_amd.ops.optim import FusedSGD

    torch.manual_seed(0)
    net = resnet18(10).cuda().to(memory_format=torch.channels_last)
    opt = FusedSGD(net.parameters(), lr=0.01, momentum=0.9)
    x = torch.randn(32, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,), device="cuda")

    def step():
        with torch.autocast("cuda", dtype=H16):
            loss = F.cross_entropy(net.logits(x).float(), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
        return loss

    step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        loss = step()
        torch.cuda.synchronize()
    assert torch.isfinite(loss)
    names = [e.key for e in prof.key_averages() if e.device_type == torch.autograd.DeviceType.CUDA]
    assert any("conv_kernel" in n for n in names), names  # the trace saw the native convs
    bad = [n for n in names if any(t in n.lower() for t in ("miopen", "igemm", "naive_conv", "batchnorm"))]
    assert not bad, bad


def _h(t):
    return t.to(H16).float()


def _ref_lenet_h(x, net):
    """fp32 math on fp16-rounded operands, activations rounded to fp16 between layers (the fp16 AMP
    contract of the fused LeNet's fp16 kernel build)."""
    h = _h(F.max_pool2d(F.relu(F.conv2d(_h(x), _h(net.conv1.weight), net.conv1.bias, padding=2)), 2))
    h = F.max_pool2d(F.relu(F.conv2d(h, _h(net.conv2.weight), net.conv2.bias)), 2)
    a2 = _h(h.flatten(1))
    h1 = _h(F.relu(F.linear(a2, _h(net.fc1.weight), net.fc1.bias)))
    h2 = _h(F.relu(F.linear(h1, _h(net.fc2.weight), net.fc2.bias)))
    return a2, F.linear(h2, _h(net.fc3.weight), net.fc3.bias)


@pytest.mark.parametrize("N", [1024, 64])
def test_lenet_whole_fused_fp16(N):
    """The fp16 build of the whole-network LeNet kernels (selected by fp16 autocast) vs the fp32
    reference of the fp16 contract; activations, fragments and d(activations) are fp16."""
    from rocket_amd.models import LeNet
    from rocket_amd.ops.lenet import lenet_forward

    torch.manual_seed(2)
    net = LeNet(fused=False).cuda()
    ref = LeNet(fused=False).cuda()
    ref.load_state_dict(net.state_dict())
    x = torch.rand(N, 1, 28, 28, device="cuda")
    with torch.autocast("cuda", dtype=H16):
        y = lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3)
    fr = net.conv1._rocket_fragments_h
    assert fr.frag.dtype == H16 and getattr(net.conv1, "_rocket_fragments", None) is None
    _, yr = _ref_lenet_h(x, ref)
    assert y.dtype == torch.float32
    assert _rel(y, yr) < 2e-3, _rel(y, yr)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    for (name, p), pr in zip(net.named_parameters(), ref.parameters()):
        assert _rel(p.grad, pr.grad) < 1e-2, (name, _rel(p.grad, pr.grad))


def test_lenet_blocks_fp16():
    """lenet_features + mlp_head under fp16 autocast: fp16 feature map, fp16 MLP kernel build."""
    from rocket_amd.models import LeNet
    from rocket_amd.ops.lenet import lenet_features, mlp_head

    torch.manual_seed(1)
    net = LeNet(fused=False).cuda()
    ref = LeNet(fused=False).cuda()
    ref.load_state_dict(net.state_dict())
    x = torch.rand(256, 1, 28, 28, device="cuda")
    with torch.autocast("cuda", dtype=H16):
        a2 = lenet_features(x, net.conv1.weight, net.conv1.bias, net.conv2.weight, net.conv2.bias)
        y = mlp_head(a2, [net.fc1, net.fc2, net.fc3])
    assert a2.dtype == H16
    a2r, yr = _ref_lenet_h(x, ref)
    assert _rel(a2, a2r) < 2e-3 and _rel(y, yr) < 2e-3, (_rel(a2, a2r), _rel(y, yr))
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    for (name, p), pr in zip(net.named_parameters(), ref.parameters()):
        assert _rel(p.grad, pr.grad) < 1e-2, (name, _rel(p.grad, pr.grad))


def test_lenet_fp16_training_steps_track_fp32():
    """Engine-free fp16 training loop on the fused LeNet (speculative whole-step path, fused
    cross-entropy, fp16 fragment table re-prepped each forward after in-place weight updates):
    the loss trajectory follows the fp32 PyTorch model's."""
    from rocket_amd.models import LeNet
    from rocket_amd.ops.lenet import fuse_cross_entropy, lenet_forward

    torch.manual_seed(4)
    net = LeNet(fused=False).cuda()
    ref = LeNet(fused=False).cuda()
    ref.load_state_dict(net.state_dict())
    o1 = torch.optim.SGD(net.parameters(), lr=0.05)
    o2 = torch.optim.SGD(ref.parameters(), lr=0.05)
    x = torch.rand(512, 1, 28, 28, device="cuda")
    t = torch.randint(0, 10, (512,), device="cuda")
    l1, l2 = [], []
    for _ in range(8):
        with torch.autocast("cuda", dtype=H16):
            y = lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3, t)
        loss, dummy = fuse_cross_entropy(y, t, 1.0)
        torch.autograd.backward([y], [dummy])
        o1.step()
        o1.zero_grad()
        lr_ = F.cross_entropy(ref.logits(x), t)
        lr_.backward()
        o2.step()
        o2.zero_grad()
        l1.append(float(loss))
        l2.append(float(lr_))
    assert l1[-1] < l1[0]
    for a, b in zip(l1, l2):
        assert abs(a - b) < 1e-2 * abs(b), (l1, l2)


def _lenet_step_grads(net, x, t, dev_scale, spec):
    from rocket_amd.ops.lenet import fuse_cross_entropy, lenet_forward

    for p in net.parameters():
        p.grad = None
    with torch.autocast("cuda", dtype=H16):
        y = lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3, t if spec else None)
    launched = y.grad_fn.spec  # the speculative whole-step launch (None: forward-only launch)
    loss, dummy = fuse_cross_entropy(y, t, 1.0, dev_scale=dev_scale)
    torch.autograd.backward([y], [dummy])
    used_spec = launched is not None and launched[8] is dev_scale
    return float(loss), [p.grad.clone() for p in net.parameters()], used_spec


@pytest.mark.parametrize("spec", [True, False])
def test_lenet_fused_ce_device_loss_scale(spec):
    """The fp16 scaler's loss scale folded into the fused LeNet cross-entropy (device tensor, read
    in-kernel): gradients are S x the unscaled ones, the reported loss is unscaled — in both the
    speculative whole-step launch and the separate backward launch."""
    from rocket_amd.models import LeNet

    torch.manual_seed(5)
    net = LeNet(fused=False).cuda()
    x = torch.rand(256, 1, 28, 28, device="cuda")
    t = torch.randint(0, 10, (256,), device="cuda")
    S = torch.tensor([1024.0], device="cuda")
    l0, g0, _ = _lenet_step_grads(net, x, t, None, spec)
    _lenet_step_grads(net, x, t, S, spec)  # primes the speculative launch with the device scale
    l1, g1, used = _lenet_step_grads(net, x, t, S, spec)
    assert used == spec
    assert abs(l1 - l0) < 1e-5 * abs(l0)
    for (name, _), a, b in zip(net.named_parameters(), g1, g0):
        assert _rel(a / 1024.0, b) < 1e-2, (name, _rel(a / 1024.0, b))


def test_lenet_wgrad_flags_nonfinite_for_scaler():
    """Under the device fp16 scaler the LeNet weight-gradient launch flags non-finite gradients
    into the scaler's found slot itself (armed fold, persistent grads): the scaler skips its check
    launch, a clean step updates, a poisoned (inf input) step is skipped with the weights kept."""
    from rocket_amd.models import LeNet
    from rocket_amd.ops.lenet import fuse_cross_entropy, lenet_forward
    from rocket_amd.ops.optim import FusedAdamW
    from rocket_amd.runtime.amp import FusedGradScaler

    torch.manual_seed(6)
    net = LeNet(fused=False).cuda()
    params = list(net.parameters())
    opt = FusedAdamW(params, lr=1e-3)
    sc = FusedGradScaler("cuda", init_scale=1024.0)
    for p in params:
        p.grad = torch.zeros_like(p)
        p._rocket_direct_grad = True
        p._rocket_optimizer = opt
    opt.prepare()
    x = torch.rand(256, 1, 28, 28, device="cuda")
    t = torch.randint(0, 10, (256,), device="cuda")
    checks = []
    orig = opt.amp_check
    opt.amp_check = lambda amp: (checks.append(1), orig(amp))
    skipped = []
    for poison in (False, True):
        xb = x.clone()
        if poison:
            xb[3, 0, 10, 10] = float("inf")
        before = [p.detach().clone() for p in params]
        opt.amp_fold_armed = True
        with torch.autocast("cuda", dtype=H16):
            y = lenet_forward(xb, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3, t)
        _, dummy = fuse_cross_entropy(y, t, 1.0, dev_scale=sc.scale_tensor)
        torch.autograd.backward([y], [dummy])
        assert opt.amp_checked  # the wgrad launch took the check over
        sc.step(opt, zero_grads=True)
        opt.amp_fold_armed = False
        skipped.append(sc.last_step_skipped())
        changed = any(not torch.equal(a, p.detach()) for a, p in zip(before, params))
        assert changed != poison
    assert skipped == [False, True] and not checks
    assert sc.get_scale() == 512.0
