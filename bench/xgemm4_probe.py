"""The one-wave-per-SIMD 256x256 GEMM (rk_xgemm4, native/kernels/xgemm4.hip) against hipBLASLt
(torch matmul) and rk_mgemm tile 0 on the forward layout: 4096^3, 8192^3 and the ViT-B/16
projection forwards (M = 128*197 tokens).  Numerics vs an fp32 reference, then the median of 20
CUDA-event timings per engine, interleaved per shape.  Uniform [-1, 1) operands.

    python bench/xgemm4_probe.py [--out gpurun_out/xgemm4_probe.jsonl]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bench.xgemm_probe import timeit  # noqa: E402
from rocket_amd.ops import _lib  # noqa: E402
from rocket_amd.ops.mgemm import mgemm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/xgemm4_probe.jsonl")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    dev = torch.device("cuda")
    lib = _lib.kernels()
    torch.manual_seed(0)
    r = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    M = 128 * 197
    shapes = [("sq4096", 4096, 4096, 4096), ("sq8192", 8192, 8192, 8192), ("qkv", M, 2304, 768),
              ("proj", M, 768, 768), ("fc1", M, 3072, 768), ("fc2", M, 768, 3072), ("odd", 1000, 520, 192)]
    out = open(a.out, "w")
    for name, m, n, k in shapes:
        x, w = r(m, k), r(n, k)
        bias = torch.randn(n, device=dev)
        y = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
        ref = x.float() @ w.float().t() + bias

        def x4():
            _lib.check(lib.rk_xgemm4(x.data_ptr(), k, w.data_ptr(), k, y.data_ptr(), n, 1, bias.data_ptr(), m, n, k,
                                     _lib.stream_ptr(dev)), "rk_xgemm4")

        x4()
        torch.cuda.synchronize()
        err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
        flop = 2.0 * m * n * k
        rec = {"case": name, "M": m, "N": n, "K": k, "rel_err": round(err, 5)}
        y0 = torch.empty_like(y)
        for tag, fn in (("x4", x4), ("lib", lambda: torch.addmm(bias.to(torch.bfloat16), x, w.t())),
                        ("t0", lambda: mgemm(x, w, y0, M=m, N=n, K=k, lda=k, ldb=k, ldc=n, bias=bias, tile=0))):
            ms = timeit(fn)
            rec[tag] = {"ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 1)}
        rec["x4_vs_lib"] = round(rec["lib"]["ms"] / rec["x4"]["ms"], 3)
        for bits in (8, 4, 12, 16, 17, 1):  # variant R (4) / no in-loop DMA (1) / + no barrier (2): garbage results
            if bits in (4, 16):
                lib.rk_xgemm4_set_dbg(bits)
                x4()
                torch.cuda.synchronize()
                rec[f"x4_{bits}_rel_err"] = round(((y.float() - ref).abs().max() / ref.abs().max()).item(), 5)
            lib.rk_xgemm4_set_dbg(bits)
            rec[f"x4_dbg{bits}"] = round(flop / timeit(x4) / 1e9, 1)
        lib.rk_xgemm4_set_dbg(0)
        print(json.dumps(rec), flush=True)
        out.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
