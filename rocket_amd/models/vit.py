"""ViT-Base/16 (Dosovitskiy et al.) for the BASELINE "ViT-B/16 bf16 DDP" config.

Pre-norm encoder, 12 layers × (MHSA 12 heads + MLP 3072), 224×224 input → 196
patches + [CLS] = 197 tokens, width 768.

MI355X path: LayerNorm is the one-wave-per-row HIP kernel emitting bf16 straight
into the next GEMM (:class:`~rocket_amd.ops.norm.FusedLayerNorm`), with the residual add fused in;
attention is one fused MFMA kernel reading the packed QKV projection, forward and one fused
backward kernel (``native/kernels/attn.hip``); GELU forward and backward (with fc1's bias
gradient) are single streaming kernels.  The projections (:class:`~rocket_amd.ops.mlinear.MLinear`,
:class:`~rocket_amd.ops.mlinear.MMlp`) are routed by ``ROCKET_VIT_GEMM``: ``lib`` (default:
hipBLASLt with the shipped TunableOp table and a bf16 weight copy kept by the fused optimizer,
K-split wgrads), ``native`` (every product on ``native/kernels/mgemm.hip``: bias / GELU epilogues,
gelu' in fc2's dgrad epilogue, split-K wgrad with the bias gradient from the same launch) or
``hybrid``; the default is the faster one measured in-model (``profiles/r2_vit_gemm_routing.md``).
The residual stream stays fp32 (standard AMP numerics); everything feeding a GEMM is bf16.

Forward contract: ``(img, label) -> (img, label, logits)``.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from rocket_amd.ops.activation import attention_qkv
from rocket_amd.ops.linear import PatchEmbed
from rocket_amd.ops.mlinear import MLinear, MMlp
from rocket_amd.ops.norm import FusedLayerNorm


class Attention(nn.Module):
    def __init__(self, dim: int, heads: int):
        super().__init__()
        self.heads = heads
        self.qkv = MLinear(dim, 3 * dim)
        self.proj = MLinear(dim, dim)

    def forward(self, x):
        # fused MFMA attention straight from the packed projection (no head permutes)
        return self.proj(attention_qkv(self.qkv(x), self.heads))


class Block(nn.Module):
    def __init__(self, dim: int, heads: int, mlp_ratio: float = 4.0):
        super().__init__()
        self.norm1 = FusedLayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, heads)
        self.norm2 = FusedLayerNorm(dim, eps=1e-6)
        self.mlp = MMlp(dim, int(dim * mlp_ratio))

    def forward(self, x, pending=None):
        """x: fp32 residual stream; pending: the previous sub-layer's output, not yet added.
        Each residual add is fused into the LayerNorm that follows it."""
        x, h = self.norm1.add_forward(x, pending)
        x, h = self.norm2.add_forward(x, self.attn(h))
        return x, self.mlp(h)


class _Embed(torch.autograd.Function):
    """``cat([cls, patches]).float() + pos`` -> the fp32 residual stream, with a backward that reads
    d(stream) once for the position gradient (a contiguous reduction over the batch) and takes the
    [CLS] gradient from its first row (sum over the batch of d(stream)[:, 0] is exactly that row), so
    no concatenation and no separate bf16 reduction over the expanded [CLS] token."""

    @staticmethod
    def forward(ctx, patches, cls, pos):
        B, P, D = patches.shape
        x = torch.empty(B, P + 1, D, dtype=torch.float32, device=patches.device)
        x[:, 1:] = patches.float() + pos[:, 1:]
        x[:, :1] = (cls.float() + pos[:, :1]).expand(B, 1, D)
        ctx.pdtype = patches.dtype
        return x

    @staticmethod
    def backward(ctx, dx):
        dpos = dx.sum(0, keepdim=True)
        return dx[:, 1:].to(ctx.pdtype), dpos[:, :1].clone(), dpos


class VisionTransformer(nn.Module):
    def __init__(self, img_size=224, patch=16, in_chans=3, num_classes=1000, dim=768, depth=12, heads=12,
                 mlp_ratio=4.0):
        super().__init__()
        self.patch = patch
        self.patch_embed = PatchEmbed(in_chans, dim, patch)  # conv k=16/s=16 as patchify + one GEMM
        n = (img_size // patch) ** 2
        self.cls_token = nn.Parameter(torch.zeros(1, 1, dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, n + 1, dim))
        self.blocks = nn.ModuleList([Block(dim, heads, mlp_ratio) for _ in range(depth)])
        self.norm = FusedLayerNorm(dim, eps=1e-6)
        self.head = MLinear(dim, num_classes)  # nn.Linear; the ViT GEMM route (ROCKET_VIT_GEMM) runs it too
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        nn.init.trunc_normal_(self.cls_token, std=0.02)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                nn.init.zeros_(m.bias)

    def logits(self, x):
        if not torch.is_autocast_enabled(x.device.type):
            x = x.to(self.fc.weight.dtype if hasattr(self, "fc") else self.head.weight.dtype)  # bf16-stored images
        x = self.patch_embed(x)  # [B, 196, D]
        x = _Embed.apply(x, self.cls_token, self.pos_embed)  # fp32 residual stream
        pending = None
        for blk in self.blocks:
            x, pending = blk(x, pending)
        _, h = self.norm.add_forward(x, pending)
        return self.head(h[:, 0])

    def forward(self, batch):
        if isinstance(batch, torch.Tensor):
            return self.logits(batch)
        img, label = batch[0], batch[1]
        return (img, label, self.logits(img))


def vit_b16(num_classes: int = 1000, img_size: int = 224) -> VisionTransformer:
    return VisionTransformer(img_size=img_size, num_classes=num_classes)
