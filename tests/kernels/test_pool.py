"""Native global average pool (ops/pool.py, norm.hip rk_gap_fwd / rk_gap_bwd) vs the PyTorch fp32
reference ``flatten(adaptive_avg_pool2d(x, 1), 1)``: values and input gradients, channels-last
16-bit and fp32 activations, the ResNet-50 (7x7) and CIFAR ResNet-18 (4x4) head shapes."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("shape", [(8, 2048, 7, 7), (16, 512, 4, 4), (3, 24, 5, 3)])
def test_gap_matches_torch(dtype, shape):
    from rocket_amd.ops.pool import global_avg_pool

    torch.manual_seed(0)
    x = torch.randn(*shape, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_()
    y = global_avg_pool(x)
    assert y.grad_fn is not None and type(y.grad_fn).__name__ == "_GapFnBackward"
    xr = x.detach().float().requires_grad_()
    yr = torch.flatten(F.adaptive_avg_pool2d(xr, 1), 1)
    tol = 1e-5 if dtype == torch.float32 else 8e-3
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    assert x.grad.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=tol, atol=tol)


def test_gap_falls_back_for_plain_layout():
    from rocket_amd.ops.pool import global_avg_pool

    x = torch.randn(2, 8, 3, 3, device="cuda", requires_grad=True)  # NCHW contiguous: torch path
    y = global_avg_pool(x)
    assert type(y.grad_fn).__name__ != "_GapFnBackward"
    torch.testing.assert_close(y, x.mean((2, 3)))
