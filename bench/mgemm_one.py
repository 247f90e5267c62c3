"""Run a few rk_mgemm configurations back to back (for rocprofv3 --pmc passes).

    python bench/mgemm_one.py qkv:fwd:0 qkv:fwd:4 fc1:dgrad:0 ... [--iters 10]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rocket_amd.ops.mgemm import mgemm  # noqa: E402

LAYERS = {"qkv": (768, 2304), "proj": (768, 768), "fc1": (768, 3072), "fc2": (3072, 768), "sq": (4096, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cases", nargs="+")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--M", type=int, default=128 * 197)
    a = ap.parse_args()
    dev = torch.device("cuda")
    M = a.M
    for case in a.cases:
        name, d, tile = case.split(":")[:3]
        split = int(case.split(":")[3]) if case.count(":") >= 3 else 1
        kin, nout = LAYERS[name]
        r = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731
        x, w, dy = r(M, kin), r(nout, kin), r(M, nout)
        if d == "fwd":
            args = (x, w, torch.empty(M, nout, dtype=torch.bfloat16, device=dev))
            kw = dict(M=M, N=nout, K=kin, lda=kin, ldb=kin, ldc=nout)
        elif d == "dgrad":
            args = (dy, w, torch.empty(M, kin, dtype=torch.bfloat16, device=dev))
            kw = dict(M=M, N=kin, K=nout, lda=nout, ldb=kin, ldc=kin, b_kmaj=True)
        else:
            args = (dy, x, torch.zeros(nout, kin, dtype=torch.float32, device=dev))
            kw = dict(M=nout, N=kin, K=M, lda=nout, ldb=kin, ldc=kin, a_kmaj=True, b_kmaj=True, splitk=split)
        for _ in range(a.iters):
            mgemm(*args, tile=int(tile), **kw)
        torch.cuda.synchronize()
        print(case, "ok", flush=True)


if __name__ == "__main__":
    main()
