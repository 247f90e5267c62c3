import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from rocket_amd.ops.activation import attention_qkv

dev = torch.device("cuda", 0)
torch.manual_seed(0)
B, L, H, D = 1, 16, 1, 64


def ref_attn(qkv, H):
    B, L, C3 = qkv.shape
    D = C3 // (3 * H)
    t = qkv.float().view(B, L, 3, H, D).permute(2, 0, 3, 1, 4)
    p = torch.softmax(t[0] @ t[1].transpose(-2, -1) / D ** 0.5, dim=-1)
    return (p @ t[2]).transpose(1, 2).reshape(B, L, H * D), p


for lo_d, hi_d in [(0, 8), (8, 16), (16, 32), (32, 64), (0, 64)]:
    qkv = torch.zeros(B, L, 3 * D, device=dev)
    qkv[0, :, lo_d:hi_d] = torch.randn(L, hi_d - lo_d, device=dev) * 2
    qkv[0, :, D + lo_d:D + hi_d] = torch.randn(L, hi_d - lo_d, device=dev) * 2
    qkv[0, :, 2 * D:2 * D + L] = torch.eye(L, device=dev)  # V = identity -> O[:, :L] = P
    qkv = qkv.to(torch.bfloat16)
    o = attention_qkv(qkv, H).float()
    r, p = ref_attn(qkv, H)
    print(f"dims [{lo_d},{hi_d}) rel err {((o - r).norm() / r.norm()).item():.4f}")
    if lo_d == 0 and hi_d == 64:
        torch.set_printoptions(precision=2, linewidth=200)
        print("kernel P row0", o[0, 0, :L])
        print("ref    P row0", p[0, 0, 0])
        print("kernel P row1", o[0, 1, :L])
        print("ref    P row1", p[0, 0, 1])
