"""The 256x256 one-wave-per-SIMD GEMM (rk_xgemm4, native/kernels/xgemm4.hip) against plain PyTorch
fp32 references: both DMA schedules (burst / spread), the LDS-staged 16-bit epilogue and the direct
one (N % 8 != 0), M / N edges off the tile grid; the fused epilogues of rk_xgemm4_epi (GELU with the
pre-activation, gelu'-multiply with the bias-gradient column sums) and the 16-bit transpose that
feeds the MLP's input-gradient GEMM."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _r(*s, scale=1.0):
    return ((torch.rand(*s, device="cuda") * 2 - 1) * scale).to(torch.bfloat16)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _lib():
    from rocket_amd.ops import _lib

    return _lib


@pytest.mark.parametrize("bits", [0, 32])
@pytest.mark.parametrize("M,N,K", [(300, 264, 128), (777, 516, 192), (2056, 768, 768), (513, 1032, 64)])
def test_xgemm4_fwd(bits, M, N, K):
    L = _lib()
    lib = L.kernels()
    torch.manual_seed(M + N)
    a, b = _r(M, K), _r(N, K)
    bias = torch.randn(N, device="cuda")
    c = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device="cuda")
    lib.rk_xgemm4_set_dbg(bits)
    try:
        L.check(lib.rk_xgemm4(a.data_ptr(), K, b.data_ptr(), K, c.data_ptr(), N, 1, bias.data_ptr(), M, N, K,
                              L.stream_ptr(a.device)), "rk_xgemm4")
        torch.cuda.synchronize()
    finally:
        lib.rk_xgemm4_set_dbg(0)
    ref = a.float() @ b.float().t() + bias
    assert not torch.isnan(c).any()
    assert _rel(c, ref) < 5e-3, _rel(c, ref)


@pytest.mark.parametrize("M,N,K", [(300, 264, 128), (2056, 3072, 768), (257, 520, 64)])
def test_xgemm4_gelu_epilogue(M, N, K):
    L = _lib()
    torch.manual_seed(7)
    a, b = _r(M, K), _r(N, K)
    bias = torch.randn(N, device="cuda")
    z = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    h = torch.empty_like(z)
    L.check(L.kernels().rk_xgemm4_epi(a.data_ptr(), K, b.data_ptr(), K, h.data_ptr(), N, 1, bias.data_ptr(),
                                      z.data_ptr(), None, None, 1, M, N, K, L.stream_ptr(a.device)), "rk_xgemm4_epi")
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t() + bias
    assert _rel(z, ref) < 5e-3
    # h is gelu of the stored (rounded) pre-activation, like the unfused GEMM -> GELU pair
    assert _rel(h, F.gelu(z.float())) < 5e-3


@pytest.mark.parametrize("M,N,K", [(300, 264, 128), (2056, 3072, 768), (777, 1032, 192)])
@pytest.mark.parametrize("colsum", [True, False])
def test_xgemm4_mulgelu_colsum_epilogue(M, N, K, colsum):
    L = _lib()
    lib = L.kernels()
    torch.manual_seed(11)
    dy, w = _r(M, K), _r(K, N)  # dz = (dy @ w) * gelu'(z); w^T is the kernel's B operand
    wt = torch.empty(N, K, dtype=torch.bfloat16, device="cuda")
    L.check(lib.rk_transpose16(w.data_ptr(), K, N, wt.data_ptr(), L.stream_ptr(w.device)), "rk_transpose16")
    z = _r(M, N, scale=3.0)
    dz = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    db = torch.full((N,), 0.5, device="cuda") if colsum else None  # accumulates onto existing values
    L.check(lib.rk_xgemm4_epi(dy.data_ptr(), K, wt.data_ptr(), K, dz.data_ptr(), N, 1, None, None, z.data_ptr(),
                              L.ptr(db), 2, M, N, K, L.stream_ptr(dy.device)), "rk_xgemm4_epi")
    torch.cuda.synchronize()
    assert torch.equal(wt, w.t().contiguous())
    dh = (dy.float() @ w.float()).to(torch.bfloat16).float()  # the unfused path rounds dh to bf16
    zf = z.float().requires_grad_()
    (gz,) = torch.autograd.grad(F.gelu(zf), zf, dh)
    assert _rel(dz, gz) < 5e-3, _rel(dz, gz)
    if colsum:
        assert _rel(db - 0.5, gz.sum(0)) < 2e-3


@pytest.mark.parametrize("rows,cols", [(768, 3072), (770, 264), (64, 8), (130, 72)])
def test_transpose16(rows, cols):
    L = _lib()
    x = _r(rows, cols)
    y = torch.empty(cols, rows, dtype=torch.bfloat16, device="cuda")
    L.check(L.kernels().rk_transpose16(x.data_ptr(), rows, cols, y.data_ptr(), L.stream_ptr(x.device)), "rk_transpose16")
    torch.cuda.synchronize()
    assert torch.equal(y, x.t().contiguous())


def test_mmlp_x4_fusions_match_unfused(monkeypatch):
    """The MLP with the fused x4 epilogues (default) vs the same module with them switched off."""
    from rocket_amd.ops import mlinear
    from rocket_amd.ops.mlinear import MMlp

    torch.manual_seed(5)
    m = MMlp(768, 3072).cuda()
    x = _r(3, 197, 768).requires_grad_()
    g = _r(3, 197, 768)
    outs = []
    for on in (True, False):
        monkeypatch.setattr(mlinear, "X4_MLP", on)
        m.zero_grad(set_to_none=True)
        xx = x.detach().clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(xx)
        y.backward(g)
        outs.append((y.float(), xx.grad.float(), [p.grad.float().clone() for p in m.parameters()]))
    (y1, gx1, gp1), (y0, gx0, gp0) = outs
    assert _rel(y1, y0) < 5e-3
    assert _rel(gx1, gx0) < 5e-3
    for a, b in zip(gp1, gp0):
        assert _rel(a, b) < 5e-3
