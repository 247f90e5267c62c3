"""Per-block phase stamps of the 256x256 one-wave-per-SIMD GEMM (rk_xgemm4, spread-DMA schedule):
prologue (first two k-tiles landed + first fragment reads), main loop, epilogue, per block, and how
the blocks' start times fall into rounds.  Says where a short-K (ViT, K = 768) tile's time goes.

    python bench/x4_trace.py [--out gpurun_out/x4_trace.json]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rocket_amd.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/x4_trace.json")
    a = ap.parse_args()
    dev = torch.device("cuda")
    lib = _lib.kernels()
    torch.manual_seed(0)
    r = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    M = 128 * 197
    res = {}
    for name, (m, n, k) in {"qkv": (M, 2304, 768), "proj": (M, 768, 768), "sq8192": (8192, 8192, 8192)}.items():
        x, w = r(m, k), r(n, k)
        bias = torch.randn(n, device=dev)
        y = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
        tiles = -(-m // 256) * -(-n // 256)
        tr = torch.zeros(tiles * 8, dtype=torch.int64, device=dev)
        out = {}
        for bits in (32, 33):  # spread / spread without in-loop DMA
            lib.rk_xgemm4_set_dbg(bits)
            for it in range(4):
                lib.rk_xgemm4_set_trace(tr.data_ptr() if it == 3 else None)
                _lib.check(lib.rk_xgemm4(x.data_ptr(), k, w.data_ptr(), k, y.data_ptr(), n, 1, bias.data_ptr(), m, n, k,
                                         _lib.stream_ptr(dev)), "rk_xgemm4")
            torch.cuda.synchronize()
            t = tr.view(tiles, 8).cpu().tolist()
            t0 = min(b[0] for b in t)
            us = lambda v: (v) / 100.0  # noqa: E731  (100 MHz)
            pro = [us(b[1] - b[0]) for b in t]
            loop = [us(b[2] - b[1]) for b in t]
            epi = [us(b[3] - b[2]) for b in t]
            starts = sorted(us(b[0] - t0) for b in t)
            ends = sorted(us(b[3] - t0) for b in t)
            # rounds: block start times cluster; report the start of every 256th block
            out[f"dbg{bits}"] = {
                "span_us": round(ends[-1], 2), "prologue_us_p50": round(statistics.median(pro), 2),
                "loop_us_p50": round(statistics.median(loop), 2), "loop_us_max": round(max(loop), 2),
                "epilogue_us_p50": round(statistics.median(epi), 2), "epilogue_us_max": round(max(epi), 2),
                "start_of_block_rank": {i: round(starts[i], 2) for i in range(0, tiles, 128)},
                "end_rank": {i: round(ends[i], 2) for i in range(0, tiles, 128)},
            }
        lib.rk_xgemm4_set_trace(None)
        lib.rk_xgemm4_set_dbg(0)
        res[name] = out
        print(name, json.dumps(out), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
