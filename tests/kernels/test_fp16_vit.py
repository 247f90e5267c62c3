"""fp16 (autocast fp16) on the transformer kernels: the fused MFMA attention (forward + fused
backward), GELU and LayerNorm (plain and add-fused) against fp32 PyTorch references."""

import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("L", [197, 64])
def test_attention_qkv_16bit(dtype, L):
    from rocket_amd.ops.activation import attention_qkv

    torch.manual_seed(0)
    B, H, D = 3, 4, 64
    qkv0 = torch.randn(B, L, 3 * H * D, device="cuda")
    qkv = qkv0.to(dtype).requires_grad_()
    out = attention_qkv(qkv, H)
    g = torch.randn_like(out)
    out.backward(g)
    ref_in = qkv.detach().float().requires_grad_()
    t = ref_in.view(B, L, 3, H, D).permute(2, 0, 3, 1, 4)
    o = torch.softmax(t[0] @ t[1].transpose(-2, -1) / math.sqrt(D), dim=-1) @ t[2]
    ref = o.transpose(1, 2).reshape(B, L, H * D)
    ref.backward(g.float())
    tol = 1e-2 if dtype == torch.bfloat16 else 3e-3
    assert out.dtype == dtype
    assert _rel(out, ref) < tol, _rel(out, ref)
    assert _rel(qkv.grad, ref_in.grad) < 3 * tol, _rel(qkv.grad, ref_in.grad)


def test_gelu_fp16():
    from rocket_amd.ops.activation import gelu

    x = torch.randn(4096, 768, device="cuda").to(torch.float16).requires_grad_()
    y = gelu(x)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    yr = F.gelu(xr)
    yr.backward(g.float())
    assert y.dtype == torch.float16
    assert _rel(y, yr) < 2e-3 and _rel(x.grad, xr.grad) < 2e-3


@pytest.mark.parametrize("shape", [(1000, 3072), (5, 36), (257, 8)])
def test_gelu_bf16_vector_paths(shape):
    """bf16 GELU forward on the 16-byte / nontemporal kernel (n % 8 == 0, grid-stride tails) and the
    4-element kernel (n % 8 != 0), against fp32 torch."""
    from rocket_amd.ops.activation import gelu

    x = (torch.randn(*shape, device="cuda") * 3).to(torch.bfloat16).requires_grad_()
    y = gelu(x)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    yr = F.gelu(xr)
    yr.backward(g.float())
    assert y.dtype == torch.bfloat16
    assert _rel(y, yr) < 8e-3 and _rel(x.grad, xr.grad) < 8e-3


@pytest.mark.parametrize("add", [False, True])
def test_layernorm_fp16_autocast(add):
    from rocket_amd.ops.norm import FusedLayerNorm

    torch.manual_seed(1)
    C = 768
    ln = FusedLayerNorm(C).cuda()
    with torch.no_grad():
        ln.weight.add_(torch.randn_like(ln.weight) * 0.1)
        ln.bias.add_(torch.randn_like(ln.bias) * 0.1)
    x = torch.randn(8, 197, C, device="cuda", requires_grad=True)
    r = torch.randn(8, 197, C, device="cuda").to(torch.float16).requires_grad_()
    with torch.autocast("cuda", dtype=torch.float16):
        if add:
            s, y = ln.add_forward(x, r)
        else:
            y = ln(x)
    assert y.dtype == torch.float16
    g = torch.randn_like(y)
    loss = (y.float() * g.float()).sum() + ((s.float() * 0.5).sum() if add else 0)
    loss.backward()
    xr = x.detach().clone().requires_grad_()
    rr = r.detach().float().requires_grad_()
    sr = xr + rr if add else xr
    yr = F.layer_norm(sr, (C,), ln.weight, ln.bias, ln.eps)
    lr = (yr * g.float()).sum() + ((sr * 0.5).sum() if add else 0)
    gw = torch.autograd.grad(lr, [xr] + ([rr] if add else []))
    assert _rel(y, yr) < 2e-3
    assert _rel(x.grad, gw[0]) < 5e-3
    if add:
        assert _rel(r.grad, gw[1]) < 5e-3


def test_vit_fp16_step_is_native():
    """A small ViT training step under fp16 autocast on the default (library-GEMM) route: the
    attention, LayerNorm, GELU and GELU-backward/bias-gradient passes are the native fp16 kernels
    (no torch softmax / GELU / fp16 copy kernels in the trace), and the loss is finite."""
    from torch.profiler import ProfilerActivity, profile

    from rocket_amd.models.vit import VisionTransformer
    from rocket_amd.ops.cross_entropy import cross_entropy
    from rocket_amd.ops.optim import FusedAdamW

    torch.manual_seed(0)
    net = VisionTransformer(img_size=64, patch=16, dim=256, depth=2, heads=4, num_classes=10).cuda()
    opt = FusedAdamW(net.parameters(), lr=1e-4)
    x = torch.randn(8, 3, 64, 64, device="cuda")
    y = torch.randint(0, 10, (8,), device="cuda")

    def step():
        with torch.autocast("cuda", dtype=torch.float16):
            loss = cross_entropy(net.logits(x), y)  # the native loss kernel (as the Loss capsule)
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
    assert any("attn_fwd_kernel" in n for n in names) and any("attn_bwd" in n for n in names), names
    assert any("ln_fwd_kernel" in n for n in names) and any("gelu" in n.lower() for n in names), names
    bad = [n for n in names if any(t in n for t in ("softmax_warp", "GeluCUDA", "gelu_kernel", "GeluBackward",
                                                       "igemm", "batched_transpose"))]  # MIOpen patch-embed conv
    assert not bad, bad
