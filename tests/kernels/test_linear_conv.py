"""Numerics of the MFMA linear and fused conv/ReLU/pool kernels vs PyTorch fp32 references."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).float()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,K,N", [(1024, 400, 120), (1024, 120, 84), (1024, 84, 10), (37, 19, 5), (300, 768, 512)])
@pytest.mark.parametrize("act", [None, "relu", "gelu"])
@pytest.mark.parametrize("xdtype", [torch.float32, torch.bfloat16])
def test_linear_fwd_bwd(M, K, N, act, xdtype):
    from rocket_amd.ops.linear import linear

    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").to(xdtype).requires_grad_()
    w = (torch.randn(N, K, device="cuda") / K**0.5).requires_grad_()
    b = torch.randn(N, device="cuda").requires_grad_()
    y = linear(x, w, b, activation=act, out_dtype=torch.float32)
    # reference: same bf16-rounded operands, fp32 math
    xr = _bf(x.detach()).requires_grad_()
    wr = _bf(w.detach()).requires_grad_()
    br = b.detach().clone().requires_grad_()
    yr = F.linear(xr, wr, br)
    if act == "relu":
        yr = F.relu(yr)
    elif act == "gelu":
        yr = F.gelu(yr)
    assert torch.allclose(y, yr, atol=2e-2, rtol=2e-2), (y - yr).abs().max()
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(_bf(g))
    for a, r in ((x.grad.float(), xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert _rel(a, r) < 2e-2, _rel(a, r)


@pytest.mark.parametrize("cfg", [(1, 6, 28, 5, 2), (6, 16, 14, 5, 0), (3, 8, 17, 3, 1)])
@pytest.mark.parametrize("xdtype", [torch.float32, torch.bfloat16])
def test_conv_relu_pool(cfg, xdtype):
    from rocket_amd.ops.conv import conv_bias_relu_pool

    Ci, Co, H, K, P = cfg
    torch.manual_seed(0)
    N = 64
    x = torch.randn(N, Ci, H, H, device="cuda").to(xdtype).requires_grad_()
    w = (torch.randn(Co, Ci, K, K, device="cuda") / (Ci * K * K) ** 0.5).requires_grad_()
    b = (torch.randn(Co, device="cuda") * 0.1).requires_grad_()
    y = conv_bias_relu_pool(x, w, b, padding=P, out_dtype=torch.float32)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().clone().requires_grad_()
    br = b.detach().clone().requires_grad_()
    yr = F.max_pool2d(F.relu(F.conv2d(xr, wr, br, padding=P)), 2)
    assert torch.allclose(y, yr, atol=1e-4, rtol=1e-4), (y - yr).abs().max()
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    assert _rel(x.grad, xr.grad) < (5e-3 if xdtype == torch.bfloat16 else 1e-5)
    assert _rel(w.grad, wr.grad) < 1e-5
    assert _rel(b.grad, br.grad) < 1e-5


def test_lenet_fused_matches_torch():
    """Fused bf16 LeNet vs the fp32 model: its gradient error must be no worse than torch autocast's."""
    from rocket_amd.models import CrossEntropy, LeNet

    torch.manual_seed(0)
    ref = LeNet(fused=False).cuda()
    amp = LeNet(fused=False).cuda()
    fus = LeNet(fused=True).cuda()
    amp.load_state_dict(ref.state_dict())
    fus.load_state_dict(ref.state_dict())
    x = torch.rand(256, 1, 28, 28, device="cuda")
    y = torch.randint(0, 10, (256,), device="cuda")
    lr = CrossEntropy(fused=False)(ref((x, y)))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        la = CrossEntropy(fused=False)(amp((x, y)))
        lf = CrossEntropy(fused=True)(fus((x, y)))
    assert abs(lr.item() - lf.item()) < 2e-2
    for l in (lr, la, lf):
        l.backward()
    for (n, r), a, f in zip(ref.named_parameters(), amp.parameters(), fus.parameters()):
        err_f, err_a = _rel(f.grad, r.grad), _rel(a.grad, r.grad)
        assert err_f < max(2 * err_a, 2e-2), (n, err_f, err_a)


def _ref_lenet(x, w1, b1, w2, b2, l1, l2, l3):
    """fp32 math on bf16-rounded operands, activations rounded to bf16 between layers (the AMP contract)."""
    h = F.max_pool2d(F.relu(F.conv2d(_bf(x), _bf(w1), b1, padding=2)), 2)
    h = _bf(h)
    h = F.max_pool2d(F.relu(F.conv2d(h, _bf(w2), b2)), 2)
    a2 = _bf(h.flatten(1))
    h1 = _bf(F.relu(F.linear(a2, _bf(l1.weight), l1.bias)))
    h2 = _bf(F.relu(F.linear(h1, _bf(l2.weight), l2.bias)))
    return a2, F.linear(h2, _bf(l3.weight), l3.bias)


@pytest.mark.parametrize("N", [1024, 37])
def test_lenet_fused_blocks(N):
    from rocket_amd.models import LeNet
    from rocket_amd.ops.lenet import lenet_features, mlp_head

    torch.manual_seed(1)
    net = LeNet(fused=False).cuda()
    ref = LeNet(fused=False).cuda()
    ref.load_state_dict(net.state_dict())
    x = torch.rand(N, 1, 28, 28, device="cuda")
    a2 = lenet_features(x, net.conv1.weight, net.conv1.bias, net.conv2.weight, net.conv2.bias)
    y = mlp_head(a2, [net.fc1, net.fc2, net.fc3])
    a2r, yr = _ref_lenet(x, ref.conv1.weight, ref.conv1.bias, ref.conv2.weight, ref.conv2.bias, ref.fc1, ref.fc2, ref.fc3)
    assert _rel(a2, a2r) < 1e-2
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    for (name, p), pr in zip(net.named_parameters(), ref.parameters()):
        assert _rel(p.grad, pr.grad) < 3e-2, (name, _rel(p.grad, pr.grad))


@pytest.mark.parametrize("N", [1024, 64, 4096])
def test_lenet_whole_fused(N):
    """One-launch forward / one-launch backward LeNet vs the fp32 reference (bf16 activation contract)."""
    from rocket_amd.models import LeNet
    from rocket_amd.ops.lenet import lenet_forward

    torch.manual_seed(2)
    net = LeNet(fused=False).cuda()
    ref = LeNet(fused=False).cuda()
    ref.load_state_dict(net.state_dict())
    x = torch.rand(N, 1, 28, 28, device="cuda")
    y = lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3)
    _, yr = _ref_lenet(x, ref.conv1.weight, ref.conv1.bias, ref.conv2.weight, ref.conv2.bias, ref.fc1, ref.fc2, ref.fc3)
    assert y.shape == (N, 10) and y.dtype == torch.float32
    assert _rel(y, yr) < 1e-2, _rel(y, yr)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    for (name, p), pr in zip(net.named_parameters(), ref.parameters()):
        assert _rel(p.grad, pr.grad) < 3e-2, (name, _rel(p.grad, pr.grad))


@pytest.mark.parametrize("N", [1024, 4096])
def test_lenet_fused_cross_entropy(N):
    """Cross-entropy computed inside the LeNet backward launch vs the two-launch path (ce_train's
    d(logits) fed to the same backward): same bf16 contract, so gradients agree to bf16 noise; the loss
    and the Loss-capsule bookkeeping (acc/ring/slot) are checked against F.cross_entropy."""
    from rocket_amd.models import LeNet
    from rocket_amd.ops.cross_entropy import ce_train
    from rocket_amd.ops.lenet import fuse_cross_entropy, lenet_forward

    torch.manual_seed(3)
    net = LeNet(fused=False).cuda()
    ref = LeNet(fused=False).cuda()
    ref.load_state_dict(net.state_dict())
    x = torch.rand(N, 1, 28, 28, device="cuda")
    t = torch.randint(0, 10, (N,), device="cuda")
    t[::7] = -100  # ignored rows
    y = lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3)
    acc = torch.full((1,), 0.5, device="cuda")
    ring = torch.zeros(8, device="cuda")
    slot = torch.full((1,), 3, dtype=torch.int64, device="cuda")
    loss, dummy = fuse_cross_entropy(y, t, 0.5, (acc, ring, slot, 2.0, 1))
    torch.autograd.backward([y], [dummy])
    yr = lenet_forward(x, ref.conv1, ref.conv2, ref.fc1, ref.fc2, ref.fc3)
    lr, dl = ce_train(yr, t, 0.5)
    yr.backward(dl)
    _, y32 = _ref_lenet(x, ref.conv1.weight, ref.conv1.bias, ref.conv2.weight, ref.conv2.bias, ref.fc1, ref.fc2,
                        ref.fc3)
    l32 = F.cross_entropy(y32, t)
    torch.cuda.synchronize()
    assert abs(float(loss) - float(lr)) < 1e-4 * abs(float(lr)), (float(loss), float(lr))
    assert abs(float(loss) - float(l32)) < 1e-2 * abs(float(l32)), (float(loss), float(l32))
    # The fused path keeps d(logits) unnormalised in bf16 (the weight-gradient launch divides by the
    # valid count), ce_train rounds the normalised values: two independent bf16 roundings of d(logits),
    # which heavily cancelling gradient sums (biases: mean of p - onehot) amplify to several %.  So
    # each path is held against the fp32 math of the same AMP contract: the fused one may not be
    # further off than the two-launch one (or than 4 %: the conv biases' sums over N x 784 positions
    # cancel to ~1 % of their terms).
    r32 = LeNet(fused=False).cuda()
    r32.load_state_dict(net.state_dict())
    _, z32 = _ref_lenet(x, r32.conv1.weight, r32.conv1.bias, r32.conv2.weight, r32.conv2.bias, r32.fc1, r32.fc2,
                        r32.fc3)
    (F.cross_entropy(z32, t) * 0.5).backward()
    for (name, p), pr, p32 in zip(net.named_parameters(), ref.parameters(), r32.parameters()):
        e_fused, e_ref = _rel(p.grad, p32.grad), _rel(pr.grad, p32.grad)
        assert e_fused <= max(1.5 * e_ref, 4e-2), (name, e_fused, e_ref)
    assert int(slot) == 4 and float(acc) == 0.0
    assert abs(float(ring[3]) - (0.5 + 2.0 * float(loss))) < 1e-5
    # a second backward without the CE spec consumes dlogits again (spec is one-shot)
    y2 = lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3)
    y2.backward(torch.zeros_like(y2))


@pytest.mark.parametrize("N", [1024, 4096])
def test_lenet_speculative_step_matches(N):
    """Speculative whole step (forward launch also runs the cross-entropy backward,
    rk_lenet_train; the weight-gradient launch applies the loss's gradient scale) vs the
    forward / backward launches: the same bf16 contract and an exact power-of-two scale, so
    loss, gradients and the Loss-capsule bookkeeping agree to fp32 round-off."""
    from rocket_amd.models import LeNet
    from rocket_amd.ops.lenet import fuse_cross_entropy, lenet_forward

    torch.manual_seed(6)
    net = LeNet(fused=False).cuda()
    ref = LeNet(fused=False).cuda()
    ref.load_state_dict(net.state_dict())
    x = torch.rand(N, 1, 28, 28, device="cuda")
    t = torch.randint(0, 10, (N,), device="cuda")
    t[::5] = -100
    outs = []
    for m, target in ((net, t), (ref, None)):
        acc = torch.full((1,), 0.25, device="cuda")
        ring = torch.zeros(4, device="cuda")
        slot = torch.zeros(1, dtype=torch.int64, device="cuda")
        y = lenet_forward(x, m.conv1, m.conv2, m.fc1, m.fc2, m.fc3, target)
        assert (getattr(y.grad_fn, "spec", None) is not None) == (target is not None)
        loss, dummy = fuse_cross_entropy(y, t, 0.5, (acc, ring, slot, 2.0, 1))
        torch.autograd.backward([y], [dummy])
        torch.cuda.synchronize()
        outs.append((y.detach().clone(), float(loss), float(ring[0]), int(slot)))
    (y1, l1, r1, s1), (y2, l2, r2, s2) = outs
    assert torch.equal(y1, y2)
    assert abs(l1 - l2) <= 1e-6 * abs(l2) and abs(r1 - r2) <= 1e-6 * abs(r2) and s1 == s2 == 1
    for (name, p), pr in zip(net.named_parameters(), ref.parameters()):
        assert _rel(p.grad, pr.grad) < 1e-5, (name, _rel(p.grad, pr.grad))


def test_lenet_speculation_dropped_for_other_losses():
    """A forward that speculated but whose backward gets an ordinary d(logits) runs the regular
    backward (same gradients as without speculation); two such misses pause speculation, a fused
    cross-entropy resumes it."""
    from rocket_amd.models import LeNet
    from rocket_amd.ops.lenet import lenet_forward

    torch.manual_seed(7)
    net = LeNet(fused=False).cuda()
    ref = LeNet(fused=False).cuda()
    ref.load_state_dict(net.state_dict())
    x = torch.rand(512, 1, 28, 28, device="cuda")
    t = torch.randint(0, 10, (512,), device="cuda")
    g = torch.randn(512, 10, device="cuda")
    for _ in range(2):
        y = lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3, t)
        assert y.grad_fn.spec is not None
        y.backward(g)
    yr = lenet_forward(x, ref.conv1, ref.conv2, ref.fc1, ref.fc2, ref.fc3)
    yr.backward(g)
    yr = lenet_forward(x, ref.conv1, ref.conv2, ref.fc1, ref.fc2, ref.fc3)
    yr.backward(g)
    for (name, p), pr in zip(net.named_parameters(), ref.parameters()):
        assert torch.equal(p.grad, pr.grad), name
    frags = net.conv1._rocket_fragments
    assert not frags.spec_ok
    y = lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3, t)
    assert y.grad_fn.spec is None
    from rocket_amd.ops.lenet import fuse_cross_entropy

    _, dummy = fuse_cross_entropy(y, t, 1.0)
    torch.autograd.backward([y], [dummy])
    assert frags.spec_ok
    y = lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3, t)
    assert y.grad_fn.spec is not None


@pytest.mark.parametrize("N", [1024, 256])
def test_lenet_fused_backward_deterministic(N):
    """The fused backward has no float atomics (per-block gradient slab rows, reduced in a fixed
    order by the weight-gradient launch): repeated runs give bit-identical gradients."""
    from rocket_amd.models import LeNet
    from rocket_amd.ops.lenet import lenet_forward

    torch.manual_seed(5)
    net = LeNet(fused=False).cuda()
    x = torch.rand(N, 1, 28, 28, device="cuda")
    g = torch.randn(N, 10, device="cuda")
    grads = []
    for _ in range(3):
        net.zero_grad(set_to_none=True)
        y = lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3)
        y.backward(g)
        grads.append([p.grad.clone() for p in net.parameters()])
    for run in grads[1:]:
        for (name, _), a, b in zip(net.named_parameters(), grads[0], run):
            assert torch.equal(a, b), (name, float((a - b).abs().max()))


@pytest.mark.parametrize("M,K,N", [(25216, 768, 2304), (100, 64, 24), (37, 16, 8), (256, 512, 10)])
def test_lib_linear_bias_grad(M, K, N):
    """LibLinear under bf16 autocast: same output / input and weight gradients as nn.Linear, bias
    gradient from the column-sum kernel vs the fp32 row sum of d(out)."""
    from rocket_amd.ops.linear import LibLinear

    torch.manual_seed(1)
    lin = LibLinear(K, N).cuda()
    ref = torch.nn.Linear(K, N).cuda()
    ref.load_state_dict(lin.state_dict())
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    g = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = lin(x)
        yr = ref(x)
    assert type(y.grad_fn).__name__ == "_LibLinearBackward"  # (N = 10: the ResNet-18 CIFAR head)
    y.backward(g)
    yr.backward(g)
    assert y.dtype == torch.bfloat16 and torch.equal(y, yr)
    assert _rel(lin.weight.grad, ref.weight.grad) < 1e-2
    db = g.float().sum(0)
    assert _rel(lin.bias.grad, db) < 1e-4, _rel(lin.bias.grad, db)
