"""Where the macro-tile GEMM's main loop spends its time: rk_xgemm at 4096^3 (and a ViT shape) with
parts of the loop switched off (rk_xgemm_set_dbg bits: 1 no LDS-DMA, 2 no barrier, 4 no fragment
reads, 8 no MFMAs; outputs are garbage then).  Median of 20 CUDA-event timings per variant.

    python bench/xgemm_dbg.py [--tiles 20,21] [--bits 0,1,2,4,8,3,5,6,7]
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
    ap.add_argument("--tiles", default="20,21")
    ap.add_argument("--bits", default="0,1,2,4,8,3,5,6,9,10,12,7,14")
    a = ap.parse_args()
    dev = torch.device("cuda")
    lib = _lib.kernels()
    r = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    shapes = [("sq4096", 4096, 4096, 4096), ("fc1fwd", 25216, 3072, 768)]
    for name, M, N, K in shapes:
        x, w = r(M, K), r(N, K)
        c = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        for t in [int(v) for v in a.tiles.split(",")]:
            row = {"shape": name, "tile": t}
            for bits in [int(v) for v in a.bits.split(",")]:
                lib.rk_xgemm_set_dbg(bits)
                ms = timeit(lambda: mgemm(x, w, c, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, tile=t))
                row[str(bits)] = round(2.0 * M * N * K / ms / 1e9, 1)
            lib.rk_xgemm_set_dbg(0)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
