import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from rocket_amd.ops.activation import attention_qkv

dev = torch.device("cuda", 0)
torch.manual_seed(0)
B, L, H, D = 1, 16, 1, 64
qkv = torch.zeros(B, L, 3 * H * D, device=dev)
v = torch.arange(L, dtype=torch.float32, device=dev)[:, None].repeat(1, D)  # V row j = j
qkv[0, :, 2 * D:] = v
o = attention_qkv(qkv.to(torch.bfloat16), H)
print("uniform attention -> expected all 7.5; got row0", o[0, 0, :8].tolist(), "row5", o[0, 5, :8].tolist())
# identity-ish: q = k = one-hot scaled -> each query attends to itself
qkv = torch.zeros(B, L, 3 * H * D, device=dev)
for j in range(L):
    qkv[0, j, j] = 8.0          # q
    qkv[0, j, D + j] = 8.0      # k
qkv[0, :, 2 * D:] = v
o = attention_qkv(qkv.to(torch.bfloat16), H)
print("self attention -> expected o[j]=j; got", [round(x, 2) for x in o[0, :, 0].tolist()])

def ref_attn(qkv, H):
    B, L, C3 = qkv.shape
    D = C3 // (3 * H)
    t = qkv.float().view(B, L, 3, H, D).permute(2, 0, 3, 1, 4)
    p = torch.softmax(t[0] @ t[1].transpose(-2, -1) / D ** 0.5, dim=-1)
    return (p @ t[2]).transpose(1, 2).reshape(B, L, H * D)

for (B, L, H) in [(1, 16, 1), (1, 16, 2), (2, 16, 1), (1, 64, 1), (1, 65, 1), (1, 197, 1), (2, 197, 12)]:
    qkv = (torch.randn(B, L, 3 * H * D, device=dev) * 1.5).to(torch.bfloat16)
    o = attention_qkv(qkv, H).float()
    r = ref_attn(qkv, H)
    err = ((o - r).norm() / r.norm()).item()
    per_head = [round(((o - r).view(B, L, H, D)[:, :, h].norm() / r.view(B, L, H, D)[:, :, h].norm()).item(), 3) for h in range(min(H, 4))]
    rows_bad = ((o - r).abs().amax(-1) > 0.1).nonzero()[:5].tolist()
    print(B, L, H, "rel", round(err, 4), "per-head", per_head, "bad rows", rows_bad)
