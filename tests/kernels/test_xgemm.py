"""Numerics of the macro-tile GEMM (rk_xgemm, native/kernels/xgemm.hip) against plain PyTorch fp32
references (16-bit-rounded operands, fp32 math): the three operand layouts in bf16 and fp16,
M/N edges off the tile grid, several tiles per persistent block (the continuous k-unit stream
across tiles), split-K slabs with the fused bias-gradient row sums, bias / accumulate epilogues;
and the ViT linear / MLP on the xgemm route (ROCKET_VIT_GEMM=x) against nn.Linear."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

XT = [20, 21]  # 256x256 / 256x128 (rocket_amd.ops.mgemm.XTILE + cfg)


def _r(*s, scale=1.0, dtype=torch.bfloat16):
    return ((torch.rand(*s, device="cuda") * 2 - 1) * scale).to(dtype)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _operands(layout, M, N, K, dtype):
    if layout == "fwd":  # A [M,K] row, B [N,K] row
        a, b = _r(M, K, dtype=dtype), _r(N, K, dtype=dtype)
        return a, b, a.float() @ b.float().t(), dict(lda=K, ldb=K)
    if layout == "dgrad":  # A [M,K] row, B stored [K,N] (kmaj)
        a, b = _r(M, K, dtype=dtype), _r(K, N, dtype=dtype)
        return a, b, a.float() @ b.float(), dict(lda=K, ldb=N, b_kmaj=True)
    a, b = _r(K, M, dtype=dtype), _r(K, N, dtype=dtype)  # A stored [K,M], B stored [K,N]
    return a, b, a.float().t() @ b.float(), dict(lda=M, ldb=N, a_kmaj=True, b_kmaj=True)


@pytest.mark.parametrize("tile", XT)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("layout", ["fwd", "dgrad", "wgrad"])
@pytest.mark.parametrize("M,N,K", [(3000, 768, 768), (300, 136, 224), (2056, 2304, 64), (792, 264, 96),
                                   (4096, 4096, 1024)])
def test_xgemm_layouts(tile, dtype, layout, M, N, K):
    """C = A.B^T for the three layouts (asymmetric random operands: a transposed C-write cannot
    pass); (4096, 4096, 1024) puts several tiles on some persistent blocks."""
    from rocket_amd.ops.mgemm import mgemm

    if layout == "wgrad" and M % 8:
        pytest.skip("kmaj A needs M % 8 == 0")
    torch.manual_seed(tile)
    a, b, ref, kw = _operands(layout, M, N, K, dtype)
    c = torch.full((M, N), float("nan"), dtype=torch.float32, device="cuda")
    mgemm(a, b, c, M=M, N=N, K=K, ldc=N, tile=tile + (16 if dtype == torch.float16 else 0), **kw)
    torch.cuda.synchronize()
    assert _rel(c, ref) < 1e-5, _rel(c, ref)


@pytest.mark.parametrize("tile", XT)
def test_xgemm_16bit_out_bias_accumulate(tile):
    from rocket_amd.ops.mgemm import mgemm

    torch.manual_seed(3)
    M, N, K = 777, 512, 256
    a, b = _r(M, K), _r(N, K, scale=0.2)
    bias = torch.randn(N, device="cuda")
    z = a.float() @ b.float().t() + bias
    c = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    mgemm(a, b, c, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, bias=bias, tile=tile)
    assert _rel(c, z) < 5e-3
    c32 = torch.randn(M, N, device="cuda")
    want = c32 + a.float() @ b.float().t()
    mgemm(a, b, c32, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, accumulate=True, tile=tile)
    assert _rel(c32, want) < 1e-5
    ah, bh = a.to(torch.float16), b.to(torch.float16)
    ch = torch.empty(M, N, dtype=torch.float16, device="cuda")
    mgemm(ah, bh, ch, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, bias=bias, tile=tile + 16)
    assert _rel(ch, ah.float() @ bh.float().t() + bias) < 2e-3


@pytest.mark.parametrize("tile", XT)
@pytest.mark.parametrize("split", [1, 3, 9])
def test_xgemm_wgrad_split_rowsum(tile, split):
    """The wgrad form: dW (+)= dY^T X with split-K slabs, db += row sums of dY^T (fused row-sum
    MFMAs of the column-0 tiles) -- including a K not a multiple of the 32-deep unit."""
    from rocket_amd.ops.mgemm import mgemm

    torch.manual_seed(split)
    T, N, K = 4100, 520, 264  # tokens, out, in
    dy, x = _r(T, N), _r(T, K)
    dw = torch.randn(N, K, device="cuda")
    db = torch.randn(N, device="cuda")
    want_w = dw + dy.float().t() @ x.float()
    want_b = db + dy.float().sum(0)
    mgemm(dy, x, dw, M=N, N=K, K=T, lda=N, ldb=K, ldc=K, a_kmaj=True, b_kmaj=True, rowsum=db, accumulate=True,
          splitk=split, tile=tile)
    torch.cuda.synchronize()
    assert _rel(dw, want_w) < 1e-5, _rel(dw, want_w)
    assert _rel(db, want_b) < 1e-5, _rel(db, want_b)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mlp", [False, True])
def test_x_route_matches_linear(monkeypatch, dtype, mlp):
    """MLinear / MMlp on the xgemm route under bf16 or fp16 autocast: forward and every gradient
    equal the stock nn.Linear composition."""
    import rocket_amd.ops as ops
    import rocket_amd.ops.mlinear as ml

    monkeypatch.setattr(ml, "MODE", "x")
    torch.manual_seed(4)
    C = 256
    mod = (ml.MMlp(C, 4 * C) if mlp else ml.MLinear(C, 3 * C)).cuda()
    x0 = torch.randn(4, 197, C, device="cuda")
    grads = []
    for fused in (True, False):
        ops.set_fused(fused)
        try:
            for p in mod.parameters():
                p.grad = None
            x = x0.clone().requires_grad_()
            with torch.autocast("cuda", dtype=dtype):
                y = mod(x)
            assert y.dtype == dtype
            y.float().square().mean().backward()
            torch.cuda.synchronize()
            grads.append((y.float(), x.grad.float(), [p.grad.float().clone() for p in mod.parameters()]))
        finally:
            ops.set_fused(True)
    (yn, xn, gn), (yt, xt, gt) = grads
    assert _rel(yn, yt) < 1e-2 and _rel(xn, xt) < 2e-2
    for a, b in zip(gn, gt):
        assert _rel(a, b) < 2e-2, _rel(a, b)
