"""Diagnostics for rk_xgemm5: per 256x256 tile (and per 32x32 block of a bad tile) relative error
against fp32, for a shape / bias choice, plus the block -> tile assignment of the persistent walk."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rocket_amd.ops import _lib  # noqa: E402


def run(M, N, K, with_bias, fill=0.0):
    lib = _lib.kernels()
    torch.manual_seed(1)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda") if with_bias else None
    c = torch.full((M, N), fill, dtype=torch.bfloat16, device="cuda")
    rc = lib.rk_xgemm5(a.data_ptr(), K, b.data_ptr(), K, c.data_ptr(), N, 1, bias.data_ptr() if with_bias else None,
                       M, N, K, _lib.stream_ptr(a.device))
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t() + (bias if with_bias else 0)
    err = (c.float() - ref).abs()
    tm, tn = (M + 255) // 256, (N + 255) // 256
    bad = []
    for i in range(tm):
        for j in range(tn):
            e = err[i * 256:(i + 1) * 256, j * 256:(j + 1) * 256]
            r = ref[i * 256:(i + 1) * 256, j * 256:(j + 1) * 256].abs().max().item()
            if e.max().item() > 0.02 * r or not torch.isfinite(e).all():
                sub = []
                for bi in range(0, e.shape[0], 32):
                    for bj in range(0, e.shape[1], 32):
                        s = e[bi:bi + 32, bj:bj + 32]
                        if s.max().item() > 0.02 * r or not torch.isfinite(s).all():
                            sub.append((bi // 32, bj // 32))
                bad.append({"tile": (i, j), "lin": i * tn + j, "nsub": len(sub), "sub": sub[:12]})
    return {"M": M, "N": N, "K": K, "bias": with_bias, "rc": rc, "tiles": tm * tn, "nbad": len(bad), "bad": bad[:20]}


if __name__ == "__main__":
    lib = _lib.kernels()
    for M, N, K in ((300, 256, 320), (777, 384, 448), (2056, 768, 768), (4100, 3072, 768)):
        for shape in (1, 4, 7, 8, 9, 10, 11, 12, 32 + 7):
            lib.rk_xgemm5_set_shape(0)
            lib.rk_xgemm5_set_shape(32)
            lib.rk_xgemm5_set_shape(shape)
            for wb in (False, True):
                r = run(M, N, K, wb)
                r["shape"] = shape
                ref_err = None
                print(json.dumps(r)[:400], flush=True)
    lib.rk_xgemm5_set_shape(0)
    lib.rk_xgemm5_set_shape(32)
