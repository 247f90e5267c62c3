"""Data-path kernels vs PyTorch: row gather, loss bookkeeping, optimizer with fused grad clearing."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_gather_rows_multi_tensor():
    from rocket_amd.ops.data import gather_rows

    dev = torch.device("cuda", 0)
    x = torch.randn(1000, 1, 28, 28, device=dev)
    y = torch.randint(0, 10, (1000,), device=dev)
    z = torch.randn(1000, 3, device=dev, dtype=torch.bfloat16)  # 6-byte rows: byte path
    idx = torch.randint(0, 1000, (777,), device=dev)
    outs = [torch.empty((777,) + t.shape[1:], dtype=t.dtype, device=dev) for t in (x, y, z)]
    gather_rows([x, y, z], idx, outs)
    for t, o in zip((x, y, z), outs):
        assert torch.equal(o, t.index_select(0, idx))


def test_gather_rows_long_rows_split_across_waves():
    """Rows longer than one 16 KiB piece are copied by several waves (ViT/ResNet image rows)."""
    from rocket_amd.ops.data import gather_rows

    dev = torch.device("cuda", 0)
    x = torch.randn(64, 3, 224, 224, device=dev, dtype=torch.bfloat16)  # 301,056 B: 18.4 pieces
    y = torch.randn(64, 5000, device=dev)  # 20,000 B: one full piece + a 3,616 B tail
    z = torch.randn(64, 8195, device=dev, dtype=torch.bfloat16)  # 16,390 B, not 16-B aligned: one wave
    lab = torch.randint(0, 1000, (64,), device=dev)
    idx = torch.randint(-64, 64, (45,), device=dev)
    outs = [torch.empty((45,) + t.shape[1:], dtype=t.dtype, device=dev) for t in (x, y, z, lab)]
    gather_rows([x, y, z, lab], idx, outs)
    for t, o in zip((x, y, z, lab), outs):
        assert torch.equal(o, t.index_select(0, idx % 64))


def test_loss_accum_ring():
    from rocket_amd.ops.data import loss_accum

    dev = torch.device("cuda", 0)
    acc = torch.zeros(1, device=dev)
    ring = torch.zeros(4, device=dev)
    slot = torch.zeros(1, dtype=torch.int64, device=dev)
    vals = [1.0, 2.0, 3.0, 4.0, 5.0, 6.0]
    for i, v in enumerate(vals):
        loss_accum(torch.tensor([v], device=dev), acc, ring, slot, 0.5, sync=(i % 2 == 1))
    # windows (1,2) (3,4) (5,6) averaged with scale 0.5 -> 1.5, 3.5, 5.5
    assert ring.tolist()[:3] == [1.5, 3.5, 5.5]
    assert int(slot) == 3 and float(acc) == 0.0


@pytest.mark.parametrize("kind", ["adamw", "sgd"])
def test_fused_step_clears_grads(kind):
    from rocket_amd.ops.optim import FusedAdamW, FusedSGD

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(n, device=dev)) for n in (5000, 37, 4096)]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    if kind == "adamw":
        opt, ropt = FusedAdamW(ps, lr=1e-2), torch.optim.AdamW(ref, lr=1e-2)
    else:
        opt, ropt = FusedSGD(ps, lr=1e-2, momentum=0.9), torch.optim.SGD(ref, lr=1e-2, momentum=0.9)
    for _ in range(3):
        for p, r in zip(ps, ref):
            g = torch.randn_like(p)
            p.grad = g.clone()
            r.grad = g.clone()
        assert opt.prepare()
        opt.launch(zero_grads=True)
        ropt.step()
        for p, r in zip(ps, ref):
            assert torch.count_nonzero(p.grad) == 0
            torch.testing.assert_close(p.detach(), r.detach(), rtol=1e-5, atol=1e-6)


def test_fused_optimizer_channels_last_flat_grads():
    """channels-last weights: flat-gradient views must share the param layout the kernel walks."""
    from rocket_amd.ops.optim import FusedSGD
    from rocket_amd.parallel.flat_grads import FlatGrads

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = torch.nn.Conv2d(8, 16, 3, bias=False).to(dev).to(memory_format=torch.channels_last)
    ref = torch.nn.Conv2d(8, 16, 3, bias=False).to(dev)
    with torch.no_grad():
        ref.weight.copy_(m.weight)
    FlatGrads(list(m.parameters()))
    opt = FusedSGD(m.parameters(), lr=0.1, momentum=0.9)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(4, 8, 10, 10, device=dev)
    for _ in range(3):
        m(x.to(memory_format=torch.channels_last)).square().mean().backward()
        ref(x).square().mean().backward()
        assert m.weight.grad.stride() == m.weight.stride()
        opt.step()
        opt.zero_grad(set_to_none=False)
        ropt.step()
        ropt.zero_grad()
    torch.testing.assert_close(m.weight.detach(), ref.weight.detach(), rtol=1e-5, atol=1e-6)
