"""Round-5 GEMM probe: the one-wave-per-SIMD 256x256 kernel (rk_xgemm4) with the library's DMA
schedule (dbg bit 5: tile t+2's LDS-DMA spread one instruction per 4 MFMAs instead of a burst at
the barrier) against the burst schedule, the DMA-free loop (timing only) and hipBLASLt, on the
forward layout at 4096^3 / 8192^3 and the ViT-B/16 projection shapes.  Numerics vs an fp32
reference for every variant that produces results; rounds interleaved per shape (median of 20).

    python bench/gemm_r5_probe.py [--out gpurun_out/gemm_r5_probe.jsonl] [--rounds 3]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/gemm_r5_probe.jsonl")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default="sq4096,sq8192,qkv,proj,fc1,fc2")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    dev = torch.device("cuda")
    lib = _lib.kernels()
    torch.manual_seed(0)
    r = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    M = 128 * 197
    allshapes = {"sq4096": (4096, 4096, 4096), "sq8192": (8192, 8192, 8192), "qkv": (M, 2304, 768),
                 "proj": (M, 768, 768), "fc1": (M, 3072, 768), "fc2": (M, 768, 3072)}
    out = open(a.out, "w")
    for name in a.shapes.split(","):
        m, n, k = allshapes[name]
        x, w = r(m, k), r(n, k)
        bias = torch.randn(n, device=dev)
        b16 = bias.to(torch.bfloat16)
        y = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
        ref = x.float() @ w.float().t() + bias

        def x4(bits):
            def f():
                lib.rk_xgemm4_set_dbg(bits)
                _lib.check(lib.rk_xgemm4(x.data_ptr(), k, w.data_ptr(), k, y.data_ptr(), n, 1, bias.data_ptr(), m, n, k,
                                         _lib.stream_ptr(dev)), "rk_xgemm4")
            return f

        rec = {"case": name, "M": m, "N": n, "K": k}
        for tag, bits in (("x4", 0), ("x4_spread", 32)):
            y.zero_()
            x4(bits)()
            torch.cuda.synchronize()
            rec[f"{tag}_rel_err"] = round(((y.float() - ref).abs().max() / ref.abs().max()).item(), 5)
        flop = 2.0 * m * n * k
        engines = {"lib": lambda: torch.addmm(b16, x, w.t()), "x4": x4(0), "x4_spread": x4(32), "x4_nodma": x4(1)}
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
