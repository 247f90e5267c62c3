"""Numerics of the native MFMA GEMM (rk_mgemm) and the ViT linear/MLP built on it, against
plain PyTorch fp32 references of the same ops (bf16-rounded operands, fp32 math)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

TILES = [0, 4, 5]


def _r(*s, scale=1.0):
    return ((torch.rand(*s, device="cuda") * 2 - 1) * scale).to(torch.bfloat16)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("layout", ["fwd", "dgrad", "wgrad"])
@pytest.mark.parametrize("M,N,K", [(25216, 768, 768), (300, 136, 200), (1000, 2304, 64), (792, 264, 88)])
def test_mgemm_layouts(tile, layout, M, N, K):
    """C = A.B^T for the three operand layouts, including M/N edges that are not tile multiples
    (asymmetric random operands: a transposed C-write cannot pass)."""
    from rocket_amd.ops.mgemm import mgemm

    torch.manual_seed(tile)
    if layout == "fwd":  # A [M,K] row, B [N,K] row
        a, b = _r(M, K), _r(N, K)
        ref = a.float() @ b.float().t()
        kw = dict(lda=K, ldb=K)
    elif layout == "dgrad":  # A [M,K] row, B stored [K,N] (kmaj)
        a, b = _r(M, K), _r(K, N)
        ref = a.float() @ b.float()
        kw = dict(lda=K, ldb=N, b_kmaj=True)
    else:  # A stored [K,M], B stored [K,N]
        if M % 8:
            pytest.skip("kmaj A needs M % 8 == 0")
        a, b = _r(K, M), _r(K, N)
        ref = a.float().t() @ b.float()
        kw = dict(lda=M, ldb=N, a_kmaj=True, b_kmaj=True)
    c = torch.empty(M, N, dtype=torch.float32, device="cuda")
    mgemm(a, b, c, M=M, N=N, K=K, ldc=N, tile=tile, **kw)
    assert _rel(c, ref) < 1e-5, _rel(c, ref)


@pytest.mark.parametrize("tile", [0, 4])
def test_mgemm_epilogues(tile):
    from rocket_amd.ops.mgemm import mgemm

    torch.manual_seed(1)
    M, N, K = 777, 512, 256
    a, b = _r(M, K), _r(N, K, scale=0.2)
    bias = torch.randn(N, device="cuda")
    z = a.float() @ b.float().t() + bias
    # bias + GELU, pre-activation side output, bf16
    c = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    pre = torch.empty_like(c)
    mgemm(a, b, c, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, bias=bias, epi="gelu", c_pre=pre, tile=tile)
    assert _rel(pre, z) < 5e-3 and _rel(c, F.gelu(z)) < 5e-3
    # relu
    mgemm(a, b, c, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, bias=bias, epi="relu", tile=tile)
    assert _rel(c, F.relu(z)) < 5e-3
    # multiply by gelu'(aux): the GELU backward fused into a dgrad
    aux = _r(M, N, scale=3.0)
    zz = aux.float().requires_grad_()
    F.gelu(zz).backward(torch.ones_like(zz))
    mgemm(a, b, c, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, epi="mul_gelu_grad", aux=aux, tile=tile)
    assert _rel(c, (a.float() @ b.float().t()) * zz.grad) < 5e-3
    # accumulate into f32
    c32 = torch.randn(M, N, device="cuda")
    want = c32 + a.float() @ b.float().t()
    mgemm(a, b, c32, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, accumulate=True, tile=tile)
    assert _rel(c32, want) < 1e-5


@pytest.mark.parametrize("split", [1, 3, 7])
def test_mgemm_splitk_rowsum(split):
    """wgrad shape: split-K slabs + combine (accumulating into an existing grad) and the fused
    bias gradient (row sums of the K-major A operand)."""
    from rocket_amd.ops.mgemm import mgemm

    torch.manual_seed(2)
    T, N, K = 4096 + 197, 384, 256  # tokens (not a k-tile multiple, odd), out features, in features
    dy, x = _r(T, N), _r(T, K)
    dw = torch.randn(N, K, device="cuda")
    db = torch.randn(N, device="cuda")
    want_w = dw + dy.float().t() @ x.float()
    want_b = db + dy.float().sum(0)
    mgemm(dy, x, dw, M=N, N=K, K=T, lda=N, ldb=K, ldc=K, a_kmaj=True, b_kmaj=True, rowsum=db, accumulate=True,
          splitk=split, tile=0)
    assert _rel(dw, want_w) < 1e-5
    assert _rel(db, want_b) < 1e-5


def test_mgemm_rejects_bad_shapes():
    from rocket_amd.ops._lib import NativeError
    from rocket_amd.ops.mgemm import mgemm

    a, b = _r(64, 100), _r(64, 100)  # K % 8 != 0
    c = torch.empty(64, 64, device="cuda")
    with pytest.raises(NativeError):
        mgemm(a, b, c, M=64, N=64, K=100, lda=100, ldb=100, ldc=64)


def _ref_linear_grads(mod_ref, x, g):
    xr = x.detach().float().requires_grad_()
    y = mod_ref(xr)
    y.backward(g.float())
    return y, xr.grad


@pytest.fixture(params=["native", "hybrid", "lib", "libw", "libd", "x5", "mixed"])
def gemm_mode(request, monkeypatch):
    import rocket_amd.ops.mlinear as ml

    monkeypatch.setattr(ml, "MODE", request.param)
    return request.param


def test_mlinear_matches_linear(gemm_mode):
    from rocket_amd.ops.mlinear import MLinear

    torch.manual_seed(3)
    m = MLinear(768, 2304).cuda()
    ref = torch.nn.Linear(768, 2304).cuda()
    ref.load_state_dict(m.state_dict())
    with torch.no_grad():  # reference on the same bf16-rounded weights
        ref.weight.copy_(ref.weight.to(torch.bfloat16).float())
    x = _r(4, 197, 768).requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    assert y.dtype == torch.bfloat16 and y.shape == (4, 197, 2304)
    g = _r(4, 197, 2304)
    y.backward(g)
    yr, dxr = _ref_linear_grads(ref, x, g)
    assert _rel(y, yr) < 5e-3
    assert _rel(x.grad, dxr) < 5e-3
    tol = 1e-3 if gemm_mode not in ("lib", "libd", "x5", "mixed") else 5e-3  # the library wgrad rounds dW to bf16
    assert _rel(m.weight.grad, ref.weight.grad) < tol
    assert _rel(m.bias.grad, ref.bias.grad) < tol


def test_mmlp_matches_unfused(gemm_mode):
    from rocket_amd.ops.mlinear import MMlp

    torch.manual_seed(4)
    m = MMlp(768, 3072).cuda()
    fc1, fc2 = torch.nn.Linear(768, 3072).cuda(), torch.nn.Linear(3072, 768).cuda()
    fc1.load_state_dict(m.fc1.state_dict())
    fc2.load_state_dict(m.fc2.state_dict())
    with torch.no_grad():
        for lin in (fc1, fc2):
            lin.weight.copy_(lin.weight.to(torch.bfloat16).float())
    x = _r(2, 197, 768).requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    g = _r(2, 197, 768)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    yr = fc2(F.gelu(fc1(xr)))
    yr.backward(g.float())
    assert _rel(y, yr) < 1e-2
    assert _rel(x.grad, xr.grad) < 1e-2
    for a, b in ((m.fc1.weight, fc1.weight), (m.fc1.bias, fc1.bias), (m.fc2.weight, fc2.weight),
                 (m.fc2.bias, fc2.bias)):
        assert _rel(a.grad, b.grad) < 1e-2


def test_mlinear_direct_grad_accumulates(monkeypatch):
    """With a persistent grad (engine flat buckets / graph capture) the native wgrad accumulates in place."""
    import rocket_amd.ops.mlinear as ml
    from rocket_amd.ops.mlinear import MLinear

    monkeypatch.setattr(ml, "MODE", "native")
    torch.manual_seed(5)
    m = MLinear(256, 512).cuda()
    for p in m.parameters():
        p.grad = torch.ones_like(p)
        p._rocket_direct_grad = True
    seen = []
    for p in m.parameters():
        p._rocket_grad_hook = lambda q: seen.append(q)
    x = _r(1024, 256)
    g = _r(1024, 512)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    y.backward(g)
    assert len(seen) == 2
    want_w = 1 + g.float().t() @ x.float()
    want_b = 1 + g.float().sum(0)
    assert _rel(m.weight.grad, want_w) < 1e-4 and _rel(m.bias.grad, want_b) < 1e-4


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("direct", [False, True])
def test_lib_direct_grads_split(monkeypatch, f32, direct):
    """Library routing: split-K partial products combined by rk_slab_acc straight into the persistent
    weight.grad (bf16 or fp32 partials), bias gradient by column sums - against fp32 math."""
    import rocket_amd.ops.linear as lin
    import rocket_amd.ops.mlinear as ml
    from rocket_amd.ops.mlinear import MLinear

    monkeypatch.setattr(ml, "MODE", "lib")
    monkeypatch.setattr(lin, "_WGRAD_F32", f32)
    torch.manual_seed(6)
    m = MLinear(384, 768).cuda()
    if direct:
        for p in m.parameters():
            p.grad = torch.full_like(p, 0.5)
            p._rocket_direct_grad = True
    x = _r(8192, 384)
    g = _r(8192, 768)
    assert lin._wgrad_splits(8192, 768, 384) > 1
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    y.backward(g)
    base = 0.5 if direct else 0.0
    want_w = base + g.float().t() @ x.float()
    want_b = base + g.float().sum(0)
    assert _rel(m.weight.grad, want_w) < (1e-4 if f32 else 5e-3)
    assert _rel(m.bias.grad, want_b) < 1e-4


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("splits", [1, 3, 4, 9])
def test_slab_acc(dt, splits):
    from rocket_amd.ops import _lib

    part = (torch.randn(splits, 1000, 24, device="cuda")).to(dt)
    dst = torch.randn(1000, 24, device="cuda")
    want = dst + part.float().sum(0)
    _lib.check(_lib.kernels().rk_slab_acc(part.data_ptr(), _lib.dtype_code(part), splits, dst.numel(),
                                          dst.data_ptr(), 1, _lib.stream_ptr(dst.device)), "rk_slab_acc")
    torch.testing.assert_close(dst, want, rtol=1e-5, atol=1e-5)
    _lib.check(_lib.kernels().rk_slab_acc(part.data_ptr(), _lib.dtype_code(part), splits, dst.numel(),
                                          dst.data_ptr(), 0, _lib.stream_ptr(dst.device)), "rk_slab_acc")
    torch.testing.assert_close(dst, part.float().sum(0), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("direct", [False, True])
def test_lib_linear_fp16_split(direct):
    """LibLinear (ViT head / patch-embed path) under fp16 autocast with a split-K weight gradient:
    the fp16 partial products are combined by rk_slab_acc's fp16 path (it used to read them as
    fp32 - an out-of-bounds read that faulted the fp16 ViT bench)."""
    from rocket_amd.ops.linear import LibLinear, _wgrad_splits

    torch.manual_seed(7)
    m = LibLinear(384, 768).cuda()
    if direct:
        for p in m.parameters():
            p.grad = torch.full_like(p, 0.5)
            p._rocket_direct_grad = True
    x = _r(8192, 384)
    g = _r(8192, 768)
    assert _wgrad_splits(8192, 768, 384) > 1
    with torch.autocast("cuda", dtype=torch.float16):
        y = m(x)
    assert y.dtype == torch.float16
    y.backward(g)
    base = 0.5 if direct else 0.0
    assert _rel(m.weight.grad, base + g.float().t() @ x.float()) < 5e-3
    assert _rel(m.bias.grad, base + g.float().sum(0)) < 1e-3


@pytest.mark.parametrize("M,N", [(25216, 3072), (300, 136)])
def test_gelu_bwd_colsum(M, N):
    from rocket_amd.ops.mlinear import _gelu_bwd_bias

    torch.manual_seed(7)
    z = _r(M, N, scale=3.0)
    dh = _r(M, N)
    b = torch.nn.Parameter(torch.zeros(N, device="cuda"))
    dz, db = _gelu_bwd_bias(dh, z, b)
    zr = z.float().requires_grad_()
    F.gelu(zr).backward(dh.float())
    assert _rel(dz, zr.grad) < 5e-3
    assert _rel(db, zr.grad.sum(0)) < 1e-4


@pytest.mark.parametrize("src,dst", [(torch.float32, torch.bfloat16), (torch.float32, torch.float16),
                                     (torch.bfloat16, torch.bfloat16), (torch.float16, torch.float16)])
def test_patchify_kernel_is_the_im2col_permutation(src, dst):
    """rk_patchify (cast + stride-k / kernel-k im2col in one pass) equals the torch permutation
    bit for bit (same round-to-nearest-even cast)."""
    from rocket_amd.ops import _lib

    torch.manual_seed(9)
    x = torch.randn(3, 3, 64, 48, device="cuda").to(src)
    B, C, H, W = x.shape
    k = 16
    ref = x.to(dst).reshape(B, C, H // k, k, W // k, k).permute(0, 2, 4, 1, 3, 5).reshape(-1, C * k * k)
    out = torch.empty_like(ref)
    _lib.check(_lib.kernels().rk_patchify(_lib.dtype_code(x), _lib.dtype_code(out), x.data_ptr(), out.data_ptr(),
                                          B, C, H, W, k, _lib.stream_ptr(x.device)), "rk_patchify")
    assert torch.equal(out, ref)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("direct", [False, True])
def test_patch_embed_matches_conv(direct, dtype):
    """ViT patch embedding as patchify + library GEMM vs an fp32 nn.Conv2d on the same 16-bit
    weights (bf16 and fp16 autocast)."""
    from rocket_amd.ops.linear import PatchEmbed

    torch.manual_seed(8)
    pe = PatchEmbed(3, 768, 16).cuda()
    ref = torch.nn.Conv2d(3, 768, 16, stride=16).cuda()
    ref.load_state_dict(pe.state_dict())
    with torch.no_grad():
        ref.weight.copy_(ref.weight.to(dtype).float())
    if direct:
        for p in pe.parameters():
            p.grad = torch.full_like(p, 0.25)
            p._rocket_direct_grad = True
    x = torch.randn(4, 3, 224, 224, device="cuda").to(dtype)
    with torch.autocast("cuda", dtype=dtype):
        y = pe(x)
    assert y.shape == (4, 196, 768) and y.dtype == dtype
    assert type(y.grad_fn).__name__ == "_PatchEmbedFnBackward"
    g = _r(4, 196, 768)
    y.backward(g)
    yr = ref(x.float()).flatten(2).transpose(1, 2)
    yr.backward(g.float())
    base = 0.25 if direct else 0.0
    assert _rel(y, yr) < 1e-2
    assert _rel(pe.weight.grad - base, ref.weight.grad) < 1e-2
    assert _rel(pe.bias.grad - base, ref.bias.grad) < 1e-3


@pytest.mark.parametrize("layout", ["fwd", "dgrad"])
@pytest.mark.parametrize("M,N,K", [(25216, 768, 768), (4096, 2304, 3072), (300, 136, 200), (1000, 2304, 64),
                                   (792, 264, 88), (512, 512, 128), (257, 520, 192), (4196, 4096, 64),
                                   (9000, 3000, 136)])
def test_mgemm_pingpong(layout, M, N, K):
    """Tile 10 (two staggered wave groups, half-tile DMA schedule): edges, partial k-tiles, 1-3
    k-tile loops; repeated launches must agree bitwise (a mis-ordered LDS hand-off shows up as
    run-to-run differences before it shows up as a large error)."""
    from rocket_amd.ops.mgemm import mgemm

    torch.manual_seed(K)
    if layout == "fwd":
        a, b = _r(M, K), _r(N, K)
        ref = a.float() @ b.float().t()
        kw = dict(lda=K, ldb=K)
    else:
        a, b = _r(M, K), _r(K, N)
        ref = a.float() @ b.float()
        kw = dict(lda=K, ldb=N, b_kmaj=True)
    # persistent blocks: > 256 tiles puts several tiles (and their k-tile streams) on one block
    bias = torch.randn(N, device="cuda") if N % 3 == 0 else None
    if bias is not None:
        ref = ref + bias
        kw["bias"] = bias
    c = torch.empty(M, N, dtype=torch.float32, device="cuda")
    mgemm(a, b, c, M=M, N=N, K=K, ldc=N, tile=10, **kw)
    assert _rel(c, ref) < 1e-5, _rel(c, ref)
    first = c.clone()
    for _ in range(4):
        c.zero_()
        mgemm(a, b, c, M=M, N=N, K=K, ldc=N, tile=10, **kw)
        assert torch.equal(c, first)


def test_mgemm_pingpong_epilogue():
    from rocket_amd.ops.mgemm import mgemm

    torch.manual_seed(3)
    M, N, K = 1000, 768, 320
    a, b = _r(M, K), _r(N, K, scale=0.2)
    bias = torch.randn(N, device="cuda")
    z = a.float() @ b.float().t() + bias
    c = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    pre = torch.empty_like(c)
    mgemm(a, b, c, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, bias=bias, epi="gelu", c_pre=pre, tile=10)
    assert _rel(pre, z) < 5e-3 and _rel(c, F.gelu(z)) < 5e-3


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(128, 1000, 768), (256, 1000, 2048)])
def test_mlinear_small_head_native(M, N, K, monkeypatch):
    """The default route's small products (classifier heads) run on mgemm: forward, input and
    parameter gradients against fp32 torch on bf16-rounded operands."""
    from rocket_amd.ops import mlinear

    monkeypatch.setattr(mlinear, "MODE", "mixed")
    assert mlinear._small(M, N, K, torch.bfloat16)
    torch.manual_seed(0)
    m = mlinear.MLinear(K, N).cuda()
    x = (torch.randn(M, K, device="cuda") * 0.5).requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    g = torch.randn_like(y.float())
    y.float().backward(g)
    xr = x.detach().bfloat16().float().requires_grad_()
    wr = m.weight.detach().bfloat16().float().requires_grad_()
    br = m.bias.detach().float().requires_grad_()
    yr = xr @ wr.t() + br
    yr.backward(g)
    scale = yr.abs().max().item()
    assert (y.float() - yr).abs().max().item() <= 2e-2 * scale
    assert (x.grad - xr.grad).abs().max().item() <= 2e-2 * xr.grad.abs().max().item()
    assert (m.weight.grad - wr.grad).abs().max().item() <= 2e-2 * wr.grad.abs().max().item()
    assert (m.bias.grad - br.grad).abs().max().item() <= 2e-2 * br.grad.abs().max().item()



@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,dtype", [(256, 10, 512, torch.bfloat16), (100, 100, 768, torch.bfloat16),
                                         (37, 10, 2048, torch.float16), (64, 3, 96, torch.float32),
                                         (1000, 10, 520, torch.bfloat16)])
def test_head_kernels_vs_fp32(M, N, K, dtype):
    """Class counts off the MFMA routes' N % 8 rule run on head.hip (one forward, one backward
    launch, fp32 logits): forward, input / weight / bias gradients against fp32 torch on the same
    (16-bit) input."""
    from rocket_amd.ops import mlinear

    torch.manual_seed(1)
    m = mlinear.MLinear(K, N).cuda()
    x = (torch.randn(M, K, device="cuda") * 0.5).to(dtype).requires_grad_()
    ctx = torch.autocast("cuda", dtype=torch.bfloat16) if dtype != torch.float16 else \
        torch.autocast("cuda", dtype=torch.float16)
    with ctx:
        assert mlinear._head_ok(m, x)
        y = m(x)
    assert y.dtype == torch.float32 and y.shape == (M, N)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    wr = m.weight.detach().clone().requires_grad_()
    br = m.bias.detach().clone().requires_grad_()
    yr = xr @ wr.t() + br
    yr.backward(g)
    assert (y - yr).abs().max().item() <= 1e-4 * yr.abs().max().item() + 1e-5
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert (x.grad.float() - xr.grad).abs().max().item() <= tol * xr.grad.abs().max().item()
    assert (m.weight.grad - wr.grad).abs().max().item() <= 1e-4 * wr.grad.abs().max().item()
    assert (m.bias.grad - br.grad).abs().max().item() <= 1e-4 * br.grad.abs().max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_pooled_head_matches_pool_then_head(dtype):
    """The global average pool fused into the head's launches (_PooledHeadFn) gives the outputs and
    gradients of ops.pool.global_avg_pool followed by the head kernels (same rounding points)."""
    from rocket_amd.ops import mlinear
    from rocket_amd.ops.pool import global_avg_pool

    torch.manual_seed(2)
    m = mlinear.MLinear(512, 10).cuda()
    x0 = torch.randn(64, 512, 4, 4, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    outs = []
    for fused in (True, False):
        m.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_()
        with torch.autocast("cuda", dtype=dtype):
            assert mlinear.pooled_head_ok(m, x)
            y = mlinear.pooled_head(m, x) if fused else m(global_avg_pool(x))
        torch.manual_seed(3)
        g = torch.randn_like(y)
        y.backward(g)
        outs.append((y.detach(), x.grad.float(), m.weight.grad.clone(), m.bias.grad.clone()))
    (y1, dx1, w1, b1), (y2, dx2, w2, b2) = outs
    assert x.grad.is_contiguous(memory_format=torch.channels_last)
    assert torch.allclose(y1, y2, rtol=1e-5, atol=1e-5)
    assert torch.allclose(dx1, dx2, rtol=1e-2, atol=1e-6)
    assert torch.allclose(w1, w2, rtol=1e-4, atol=1e-6) and torch.allclose(b1, b2, rtol=1e-5, atol=1e-6)
