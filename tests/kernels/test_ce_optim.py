"""Numerics of the fused cross-entropy and multi-tensor optimizer kernels vs PyTorch fp32 references."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,C", [(1024, 10), (37, 3), (256, 1000), (5, 64), (9, 65)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("smoothing", [0.0, 0.1])
def test_cross_entropy_matches_torch(N, C, dtype, smoothing):
    from rocket_amd.ops.cross_entropy import cross_entropy

    torch.manual_seed(0)
    x = (torch.randn(N, C, device="cuda") * 3).to(dtype).requires_grad_()
    t = torch.randint(0, C, (N,), device="cuda")
    t[::7] = -100
    xr = x.detach().float().requires_grad_()
    ref = F.cross_entropy(xr, t, label_smoothing=smoothing)
    out = cross_entropy(x, t, label_smoothing=smoothing)
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    assert torch.allclose(out.float(), ref, atol=tol, rtol=tol), (out.item(), ref.item())
    g = torch.tensor(0.37, device="cuda")
    (out * g).backward()
    (ref * g).backward()
    assert torch.allclose(x.grad.float(), xr.grad, atol=tol * 2, rtol=1e-2)


def test_cross_entropy_sum_and_graph_replay():
    from rocket_amd.ops.cross_entropy import cross_entropy

    x = torch.randn(300, 10, device="cuda")
    t = torch.randint(0, 10, (300,), device="cuda")
    assert torch.allclose(cross_entropy(x, t, reduction="sum"), F.cross_entropy(x, t, reduction="sum"), rtol=1e-5)
    # the in-launch ticket counter must reset itself across repeated launches / replays
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            cross_entropy(x, t)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = cross_entropy(x, t)
    for k in range(4):
        x.copy_(torch.randn_like(x))
        g.replay()
        torch.cuda.synchronize()
        assert torch.allclose(y, F.cross_entropy(x, t), rtol=1e-5, atol=1e-6)


def _clone_params(ps):
    return [torch.nn.Parameter(p.detach().clone()) for p in ps]


@pytest.mark.parametrize("kind", ["adamw", "adam", "sgd", "sgd_nesterov", "sgd_big", "sgd_nomom_big", "adamw_big"])
def test_fused_optimizer_matches_torch(kind):
    """Small (LeNet-sized: 1024-element chunks) and big (> 2M parameters: 4096-element chunks, the
    vectorised full-chunk path plus the scalar tail) parameter sets against torch.optim."""
    from rocket_amd.ops.optim import FusedAdam, FusedAdamW, FusedSGD

    torch.manual_seed(0)
    shapes = [(6, 1, 5, 5), (6,), (16, 6, 5, 5), (16,), (120, 400), (120,), (84, 120), (84,), (10, 84), (10,), (5000,)]
    if kind.endswith("_big"):
        shapes = shapes + [(1500, 1501), (512, 2048), (77,)]
        kind = kind[:-4]
    base = [torch.randn(s, device="cuda") for s in shapes]
    a, b = _clone_params(base), _clone_params(base)
    if kind == "adamw":
        oa = FusedAdamW([{"params": a[:4], "lr": 3e-3}, {"params": a[4:], "weight_decay": 0.1}], lr=1e-3)
        ob = torch.optim.AdamW([{"params": b[:4], "lr": 3e-3}, {"params": b[4:], "weight_decay": 0.1}], lr=1e-3)
    elif kind == "adam":
        oa = FusedAdam(a, lr=1e-3, weight_decay=0.01)
        ob = torch.optim.Adam(b, lr=1e-3, weight_decay=0.01)
    elif kind == "sgd":
        oa = FusedSGD(a, lr=0.1, momentum=0.9, weight_decay=1e-4)
        ob = torch.optim.SGD(b, lr=0.1, momentum=0.9, weight_decay=1e-4)
    elif kind == "sgd_nomom":
        oa = FusedSGD(a, lr=0.1, weight_decay=1e-4)
        ob = torch.optim.SGD(b, lr=0.1, weight_decay=1e-4)
    else:
        oa = FusedSGD(a, lr=0.1, momentum=0.9, nesterov=True)
        ob = torch.optim.SGD(b, lr=0.1, momentum=0.9, nesterov=True)
    for step in range(5):
        for pa, pb in zip(a, b):
            g = torch.randn_like(pa)
            pa.grad = g.clone()
            pb.grad = g.clone()
        oa.step()
        ob.step()
        if step == 2:
            for g in oa.param_groups + ob.param_groups:
                g["lr"] *= 0.5
    torch.cuda.synchronize()
    for pa, pb in zip(a, b):
        assert torch.allclose(pa, pb, atol=1e-5, rtol=1e-5), (pa - pb).abs().max()
    sd = oa.state_dict()
    if kind.startswith("adam"):
        assert float(sd["state"][0]["step"]) == 5.0
        assert torch.allclose(sd["state"][4]["exp_avg"], ob.state_dict()["state"][4]["exp_avg"], atol=1e-6)


@pytest.mark.parametrize("C,dtype", [(10, torch.float32), (1000, torch.bfloat16), (1000, torch.float16)])
def test_ce_train_one_launch(C, dtype):
    """ce_train: loss, d(logits) (scaled) and the loss bookkeeping in one launch vs torch."""
    from rocket_amd.ops.cross_entropy import ce_train

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    x = torch.randn(300, C, device=dev).to(dtype)
    t = torch.randint(0, C, (300,), device=dev)
    t[::7] = -100  # ignored rows
    acc = torch.full((1,), 0.5, device=dev)
    ring = torch.zeros(8, device=dev)
    slot = torch.full((1,), 7, dtype=torch.int64, device=dev)
    loss, dx = ce_train(x, t, 0.25, (acc, ring, slot, 2.0, True))
    xr = x.detach().float().requires_grad_(True)
    lr = torch.nn.functional.cross_entropy(xr, t)
    (lr * 0.25).backward()
    torch.testing.assert_close(loss, lr.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dx.float(), xr.grad, rtol=1e-4 if dtype == torch.float32 else 2e-2, atol=1e-5)
    assert abs(float(ring[7]) - (0.5 + 2.0 * float(lr))) < 1e-3  # acc + scale*loss reported
    assert int(slot) == 0 and float(acc) == 0.0  # ring cursor wrapped, window reset


def test_optimizer_maintains_lenet_fragment_table():
    """The fused AdamW writes the bf16 MFMA fragment table of a fused LeNet while updating the
    weights (registered bf16 shadows): after a step the table equals a fresh lenet_prep of the
    new weights bit for bit, and the next forward skips the prep launch."""
    from rocket_amd.models import LeNet
    from rocket_amd.ops import _lib
    from rocket_amd.ops.lenet import lenet_forward
    from rocket_amd.ops.optim import FusedAdamW

    torch.manual_seed(4)
    net = LeNet(fused=True).cuda()
    opt = FusedAdamW(net.parameters(), lr=1e-2)
    x = torch.rand(64, 1, 28, 28, device="cuda")
    for _ in range(3):
        y = lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3)
        y.square().mean().backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
    frags = net.conv1._rocket_fragments
    torch.cuda.synchronize()
    ref = torch.empty_like(frags.frag)
    ws = [p.detach() for p in (net.fc1.weight, net.fc2.weight, net.fc3.weight, net.conv1.weight, net.conv2.weight)]
    _lib.check(_lib.kernels().rk_lenet_prep(*[w.data_ptr() for w in ws], ref.data_ptr(), _lib.stream_ptr(x.device)),
               "rk_lenet_prep")
    torch.cuda.synchronize()
    assert torch.equal(frags.frag.view(torch.int16), ref.view(torch.int16))
    v = frags.versions
    lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3)
    assert frags.versions == v  # live table: no prep
    with torch.no_grad():
        net.fc2.weight.mul_(0.5)  # an outside write bumps the version -> prep on the next forward
    lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3)
    assert frags.versions != v


def test_optimizer_maintains_dense_bf16_weight_copy():
    """LibLinear's bf16 weight copy is a dense bf16 shadow: after fused AdamW steps it equals the
    bf16 rounding of the fp32 master exactly, and forwards stop re-casting (version unchanged)."""
    from rocket_amd.ops.linear import LibLinear
    from rocket_amd.ops.optim import FusedAdamW

    torch.manual_seed(6)
    lin = LibLinear(64, 48).cuda()
    opt = FusedAdamW(lin.parameters(), lr=1e-2)
    x = torch.randn(32, 64, device="cuda")
    for _ in range(3):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = lin(x)
        y.float().square().mean().backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
    torch.cuda.synchronize()
    assert torch.equal(lin._w16, lin.weight.detach().to(torch.bfloat16))
    assert torch.equal(lin._b16, lin.bias.detach().to(torch.bfloat16))
    assert lin._w16_version == lin.weight._version
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ref = torch.nn.functional.linear(x, lin.weight, lin.bias)
        assert torch.equal(lin(x), ref)


@pytest.mark.parametrize("kind", ["adamw", "sgd"])
def test_optimizer_maintains_dense_fp16_weight_copy(kind):
    """fp16 autocast: LibLinear's fp16 weight copy is a dense fp16 shadow (map pointer 2) that the
    fused update writes; switching the autocast dtype re-registers the bf16 one, never a stale copy."""
    from rocket_amd.ops.linear import LibLinear
    from rocket_amd.ops.optim import FusedAdamW, FusedSGD

    torch.manual_seed(7)
    lin = LibLinear(64, 48).cuda()
    opt = FusedAdamW(lin.parameters(), lr=1e-2) if kind == "adamw" else FusedSGD(lin.parameters(), lr=1e-2,
                                                                                 momentum=0.9)
    x = torch.randn(32, 64, device="cuda")
    for dt in (torch.float16, torch.float16, torch.bfloat16, torch.float16):
        with torch.autocast("cuda", dtype=dt):
            y = lin(x)
        y.float().square().mean().backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
    torch.cuda.synchronize()
    assert torch.equal(lin._w16_f16, lin.weight.detach().to(torch.float16))
    assert torch.equal(lin._b16_f16, lin.bias.detach().to(torch.float16))
    assert lin._w16_f16_version == lin.weight._version
    with torch.autocast("cuda", dtype=torch.float16):
        ref = torch.nn.functional.linear(x, lin.weight, lin.bias)
        assert torch.equal(lin(x), ref)
    with torch.autocast("cuda", dtype=torch.bfloat16):  # the bf16 copy was re-cast, not stale
        ref = torch.nn.functional.linear(x, lin.weight, lin.bias)
        assert torch.equal(lin(x), ref)
