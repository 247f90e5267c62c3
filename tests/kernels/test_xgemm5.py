"""The persistent 256x256 GEMM (rk_xgemm5, native/kernels/xgemm5.hip) against plain PyTorch fp32
references: bias folded into the MFMAs (hi/lo bf16 rank-2 update) or absent, bf16 and fp16 output,
M off the tile grid, N = 128 mod 256 (a wave's half-tile out of range), several tiles per block
(stores of one tile drained under the next), K at the 5-k-tile minimum and long, and a C with a
row stride wider than N; plus the argument checks."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _r(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).to(torch.bfloat16)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _lib():
    from rocket_amd.ops import _lib

    return _lib


def _run(a, b, c, bias, M, N, K, ldc=None):
    L = _lib()
    rc = L.kernels().rk_xgemm5(a.data_ptr(), K, b.data_ptr(), K, c.data_ptr(), ldc or N, L.dtype_code(c),
                               bias.data_ptr() if bias is not None else None, M, N, K, L.stream_ptr(a.device))
    return rc


@pytest.fixture(params=[0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 32 + 7, 32 + 5],
                ids=["auto", "256x256", "128x256", "256x128", "w8-256x256", "w8-128x256", "w8-256x128", "128x128",
                     "256x160", "m16-256x256", "m16-256x160", "m16-128x256", "m16-256x128",
                     "split-128x128", "split-w8-128x256"])
def x5_shape(request):
    """Tile shape of rk_xgemm5 (codes of rk_xgemm5_set_shape): every single-launch shape, and the
    two-launch row split (256x256 rows + a smaller-tile tail) forced onto each problem."""
    lib = _lib().kernels()
    lib.rk_xgemm5_set_shape(request.param)
    yield request.param
    lib.rk_xgemm5_set_shape(0)
    lib.rk_xgemm5_set_shape(32)


@pytest.mark.parametrize("M,N,K", [(300, 256, 320), (777, 384, 448), (2056, 768, 768), (25216, 2304, 768),
                                   (4100, 3072, 768), (1999, 768, 3072), (25216, 768, 768)])
@pytest.mark.parametrize("with_bias", [True, False])
def test_xgemm5_fwd(M, N, K, with_bias, x5_shape):
    torch.manual_seed(M + N + K)
    a, b = _r(M, K), _r(N, K)
    bias = torch.randn(N, device="cuda") if with_bias else None
    c = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device="cuda")
    assert _run(a, b, c, bias, M, N, K) == 0
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t()
    if bias is not None:
        ref = ref + bias
    assert not torch.isnan(c).any()
    assert _rel(c, ref) < 5e-3, _rel(c, ref)


def test_xgemm5_fp16_out_and_wide_ldc(x5_shape):
    torch.manual_seed(5)
    M, N, K, ldc = 1030, 512, 640, 520
    a, b = _r(M, K), _r(N, K)
    bias = torch.randn(N, device="cuda") * 4
    c = torch.full((M, ldc), float("nan"), dtype=torch.float16, device="cuda")
    assert _run(a, b, c, bias, M, N, K, ldc=ldc) == 0
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t() + bias
    assert _rel(c[:, :N], ref) < 2e-3, _rel(c[:, :N], ref)
    assert torch.isnan(c[:, N:]).all()  # the columns past N are never written


def test_xgemm5_bias_exact_to_2e16(x5_shape):
    """A zero product isolates the bias path: C = bf16(b_hi + b_lo) with b_hi + b_lo within 2^-16 of
    b, so C is bf16(b) except where b sits that close to a rounding midpoint (then one ulp off)."""
    M, N, K = 512, 256, 320
    a = torch.zeros(M, K, dtype=torch.bfloat16, device="cuda")
    b = _r(N, K)
    bias = torch.randn(N, device="cuda") * 100
    c = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    assert _run(a, b, c, bias, M, N, K) == 0
    torch.cuda.synchronize()
    want = bias.to(torch.bfloat16).expand(M, N)
    assert (c == want).float().mean().item() > 0.99
    assert ((c.float() - bias).abs() <= bias.abs() * 2.0 ** -8).all()


def test_xgemm5_rejects_unsupported_shapes():
    a, b = _r(256, 256), _r(256, 256)
    c = torch.empty(256, 256, dtype=torch.bfloat16, device="cuda")
    assert _run(a, b, c, None, 256, 256, 256) != 0  # K < 320
    a2, b2 = _r(256, 320), _r(200, 320)
    c2 = torch.empty(256, 200, dtype=torch.bfloat16, device="cuda")
    assert _run(a2, b2, c2, None, 256, 200, 320) != 0  # N % 128
    c3 = torch.empty(256, 256, dtype=torch.float32, device="cuda")
    assert _run(a2, _r(256, 320), c3, None, 256, 256, 320) != 0  # f32 out
