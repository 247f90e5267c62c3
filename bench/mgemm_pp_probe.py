"""Tile 10 (ping-pong 256x256) against tile 0 and hipBLASLt at the ViT-B/16 forward / dgrad shapes
and two square sizes: max error vs fp32, median time of 20 (CUDA events), TFLOP/s.  Uniform
[-1, 1) operands.

    python bench/mgemm_pp_probe.py [--tiles 0,10] [--out gpurun_out/mgemm_pp.jsonl]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rocket_amd.ops.mgemm import mgemm  # noqa: E402
from bench.mgemm_probe import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="0,10")
    ap.add_argument("--out", default="gpurun_out/mgemm_pp.jsonl")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    tiles = [int(t) for t in args.tiles.split(",")]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    T = 128 * 197
    shapes = [("qkv", "fwd", T, 2304, 768), ("qkv", "dgrad", T, 768, 2304), ("proj", "fwd", T, 768, 768),
              ("proj", "dgrad", T, 768, 768), ("fc1", "fwd", T, 3072, 768), ("fc1", "dgrad", T, 768, 3072),
              ("fc2", "fwd", T, 768, 3072), ("fc2", "dgrad", T, 3072, 768), ("sq4k", "fwd", 4096, 4096, 4096),
              ("sq8k", "fwd", 8192, 8192, 8192)]
    r = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    out = open(args.out, "w")
    for name, d, M, N, K in shapes:
        a = r(M, K)
        if d == "fwd":
            b = r(N, K)
            kw = dict(lda=K, ldb=K)
            tfn = lambda: a @ b.t()  # noqa: E731
        else:
            b = r(K, N)
            kw = dict(lda=K, ldb=N, b_kmaj=True)
            tfn = lambda: a @ b  # noqa: E731
        ref = tfn().float() if M * N * K > 2 ** 34 else (a.float() @ (b.float().t() if d == "fwd" else b.float()))
        scale = ref.abs().max().item()
        flop = 2.0 * M * N * K
        tl = timeit(tfn, args.iters)
        rec = {"layer": name, "dir": d, "M": M, "N": N, "K": K, "lib_tflops": round(flop / tl / 1e9, 1)}
        c = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        for t in tiles:
            run = lambda t=t: mgemm(a, b, c, M=M, N=N, K=K, ldc=N, tile=t, **kw)  # noqa: E731
            run()
            torch.cuda.synchronize()
            err = (c.float() - ref).abs().max().item() / scale
            tm = timeit(run, args.iters)
            rec[f"t{t}"] = {"tflops": round(flop / tm / 1e9, 1), "err": round(err, 5)}
        print(json.dumps(rec), flush=True)
        out.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
