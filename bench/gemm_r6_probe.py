"""Round-6 GEMM probe: the persistent 256x256 kernel with the tile drained under the next one
(rk_xgemm5, native/kernels/xgemm5.hip) against hipBLASLt (torch.addmm, the ViT default) and the
round-5 one-wave-per-SIMD kernel (rk_xgemm4, spread DMA + LDS-staged stores) on the ViT-B/16
projection shapes (forward layout C = A B^T + bias, bf16).  Numerics vs an fp32 reference for every
native variant; rounds interleaved per shape (median of 20 CUDA-event timings each).

    python bench/gemm_r6_probe.py [--out gpurun_out/gemm_r6_probe.jsonl] [--rounds 3]
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

M = 128 * 197
SHAPES = {"sq4096": (4096, 4096, 4096), "sq8192": (8192, 8192, 8192), "qkv": (M, 2304, 768),
          "proj": (M, 768, 768), "fc1": (M, 3072, 768), "fc2": (M, 768, 3072),
          # input gradients (dx = dy W, as dy [M, N_out] x W^T [K_in, N_out]^T)
          "qkv_dg": (M, 768, 2304), "fc1_dg": (M, 768, 3072), "fc2_dg": (M, 3072, 768)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/gemm_r6_probe.jsonl")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default="qkv,proj,fc1,fc2,fc2_dg,qkv_dg,sq8192")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    dev = torch.device("cuda")
    lib = _lib.kernels()
    torch.manual_seed(0)
    r = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    out = open(a.out, "w")
    for name in a.shapes.split(","):
        m, n, k = SHAPES[name]
        x, w = r(m, k), r(n, k)
        bias = torch.randn(n, device=dev)
        b16 = bias.to(torch.bfloat16)
        y = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
        ref = x.float() @ w.float().t() + bias
        stream = _lib.stream_ptr(dev)

        def x5(with_bias=True):
            def f():
                _lib.check(lib.rk_xgemm5(x.data_ptr(), k, w.data_ptr(), k, y.data_ptr(), n, 1,
                                         bias.data_ptr() if with_bias else None, m, n, k, stream), "rk_xgemm5")
            return f

        def x4():
            lib.rk_xgemm4_set_dbg(32)
            _lib.check(lib.rk_xgemm4(x.data_ptr(), k, w.data_ptr(), k, y.data_ptr(), n, 1, bias.data_ptr(), m, n, k,
                                     stream), "rk_xgemm4")

        rec = {"case": name, "M": m, "N": n, "K": k}
        for tag, fn, rf in (("x5", x5(True), ref), ("x5_nobias", x5(False), ref - bias)):
            y.fill_(float("nan"))
            fn()
            torch.cuda.synchronize()
            err = ((y.float() - rf).abs().max() / rf.abs().max()).item()
            rec[f"{tag}_rel_err"] = round(err, 5) if err == err else "nan"
        flop = 2.0 * m * n * k
        def shaped(sh):
            def f():
                lib.rk_xgemm5_set_shape(sh)
                x5(True)()
                lib.rk_xgemm5_set_shape(0)
            return f

        def fam(f):
            def g():
                lib.rk_xgemm5_set_shape(16 + f)
                x5(True)()
                lib.rk_xgemm5_set_shape(16 + 2)
            return g

        engines = {"lib": lambda: torch.addmm(b16, x, w.t()), "x5": x5(True), "x5_nobias": x5(False),
                   "f0": fam(0), "f1": fam(1), "s1": shaped(1), "s8": shaped(8), "s9": shaped(9), "s10": shaped(10)}
        times = {t: [] for t in engines}
        for _ in range(a.rounds):
            for tag, fn in engines.items():
                times[tag].append(timeit(fn))
        lib.rk_xgemm4_set_dbg(0)
        for tag, ts in times.items():
            ms = sorted(ts)[len(ts) // 2]
            rec[tag] = {"ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 1)}
        print(json.dumps(rec), flush=True)
        out.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
