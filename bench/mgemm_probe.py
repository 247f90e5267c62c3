"""Numerics + speed of the native MFMA GEMM (rk_mgemm) against hipBLASLt at the ViT-B/16 shapes.

For every projection (qkv 768->2304, proj 768->768, fc1 768->3072, fc2 3072->768) at
M = 128*197 tokens and each direction (fwd / dgrad / wgrad), every tile config is checked
against an fp32 torch reference and timed (CUDA events, median of 20) next to torch's bf16
matmul of the same product.  Uniform [-1, 1) operands (zero-filled data inflates MFMA clocks).

    python bench/mgemm_probe.py [--out gpurun_out/mgemm_probe.jsonl] [--quick]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rocket_amd.ops.mgemm import TILES, mgemm, pick_split, pick_tile  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    t = sorted(s.elapsed_time(e) for s, e in ev)
    return t[len(t) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/mgemm_probe.jsonl")
    ap.add_argument("--M", type=int, default=128 * 197)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default="", help="comma list of directions (fwd,dgrad,wgrad)")
    ap.add_argument("--epi", action="store_true", help="also time the fused GELU epilogues (fc1 fwd, fc2 dgrad)")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M = args.M
    layers = {"qkv": (768, 2304), "proj": (768, 768), "fc1": (768, 3072), "fc2": (3072, 768)}
    out = open(args.out, "w")
    if args.epi:
        epi_cases(M, out)
        if args.only == "none":
            return

    def r(*s):
        return (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)

    for name, (kin, nout) in layers.items():
        x, w, dy = r(M, kin), r(nout, kin) * 0.05, r(M, nout)
        cases = {
            # direction: (a, b, a_kmaj, b_kmaj, gM, gN, gK, lda, ldb, torch fn, fp32 ref fn)
            "fwd": (x, w, False, False, M, nout, kin, kin, kin, lambda: x @ w.t(), lambda: x.float() @ w.float().t()),
            "dgrad": (dy, w, False, True, M, kin, nout, nout, kin, lambda: dy @ w, lambda: dy.float() @ w.float()),
            "wgrad": (dy, x, True, True, nout, kin, M, nout, kin, lambda: dy.t() @ x, lambda: dy.float().t() @ x.float()),
        }
        if args.only:
            cases = {k: v for k, v in cases.items() if k in args.only.split(",")}
        for d, (a, b, ak, bk, gM, gN, gK, lda, ldb, tfn, rfn) in cases.items():
            ref = rfn()
            scale = ref.abs().max().item()
            flop = 2.0 * gM * gN * gK
            t_lib = timeit(tfn)
            rec = {"layer": name, "dir": d, "M": gM, "N": gN, "K": gK, "hipblaslt_ms": round(t_lib, 4),
                   "hipblaslt_tflops": round(flop / t_lib / 1e9, 1)}
            if d == "wgrad":
                configs = [(t, s) for t in TILES for s in (1, 2, 3, 4, 6, 8) if t < 6]
                if args.quick:
                    configs = [pick_split(gM, gN, gK)]
                rec["auto"] = list(pick_split(gM, gN, gK))
            else:
                configs = [(t, 1) for t in TILES] if not args.quick else [(pick_tile(gM, gN, gK), 1)]
                configs = [(t, s) for t, s in configs if not (t >= 6 and ak and bk) and t in (0, 4, 7, 8, 9)]
                rec["auto"] = [pick_tile(gM, gN, gK), 1]
            for t, s in configs:
                odt = torch.float32 if d == "wgrad" else torch.bfloat16
                c = torch.zeros(gM, gN, dtype=odt, device=dev)

                def run(c=c, t=t, s=s):
                    mgemm(a, b, c, M=gM, N=gN, K=gK, lda=lda, ldb=ldb, ldc=gN, a_kmaj=ak, b_kmaj=bk, splitk=s, tile=t)

                run()
                torch.cuda.synchronize()
                err = (c.float() - ref).abs().max().item() / scale
                tm = timeit(run)
                rec[f"t{t}s{s}"] = {"ms": round(tm, 4), "tflops": round(flop / tm / 1e9, 1), "rel_err": err}
            best = min((v["ms"], k) for k, v in rec.items() if isinstance(v, dict))
            rec["best"] = best[1]
            rec["best_vs_lib"] = round(t_lib / best[0], 3)
            print(json.dumps(rec), flush=True)
            out.write(json.dumps(rec) + "\n")
            out.flush()


def epi_cases(M, out):
    dev = torch.device("cuda")
    r = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    x, w1, w2 = r(M, 768), r(3072, 768) * 0.05, r(768, 3072) * 0.05
    b1 = torch.randn(3072, device=dev)
    dy = r(M, 768)
    h = torch.empty(M, 3072, dtype=torch.bfloat16, device=dev)
    pre = torch.empty_like(h)
    for t in TILES:
        rec = {"case": "fc1_fwd_gelu", "tile": t}
        rec["ms_gelu"] = timeit(lambda: mgemm(x, w1, h, M=M, N=3072, K=768, lda=768, ldb=768, ldc=3072, bias=b1,
                                              epi="gelu", c_pre=pre, tile=t))
        rec["ms_plain"] = timeit(lambda: mgemm(x, w1, h, M=M, N=3072, K=768, lda=768, ldb=768, ldc=3072, bias=b1,
                                               tile=t))
        rec["ms_dgrad_gelu"] = timeit(lambda: mgemm(dy, w2, h, M=M, N=3072, K=768, lda=768, ldb=3072, ldc=3072,
                                                    b_kmaj=True, epi="mul_gelu_grad", aux=pre, tile=t))
        rec["ms_dgrad_plain"] = timeit(lambda: mgemm(dy, w2, h, M=M, N=3072, K=768, lda=768, ldb=3072, ldc=3072,
                                                     b_kmaj=True, tile=t))
        z = (x.float() @ w1.float().t() + b1)
        mgemm(x, w1, h, M=M, N=3072, K=768, lda=768, ldb=768, ldc=3072, bias=b1, epi="gelu", c_pre=pre, tile=t)
        rec["gelu_rel_err"] = ((h.float() - torch.nn.functional.gelu(z)).norm() / torch.nn.functional.gelu(z).norm()).item()
        print(json.dumps(rec), flush=True)
        out.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
