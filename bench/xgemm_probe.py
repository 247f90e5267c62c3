"""Numerics + speed of the macro-tile GEMM (rk_xgemm, native/kernels/xgemm.hip) against hipBLASLt
and the older rk_mgemm tile 0, at 4096^3 / 8192^3 and the ViT-B/16 shapes (M = 128*197 tokens).

Every product is checked against an fp32 torch reference (max |err| / max |ref|), then timed with
CUDA events (median of 20), interleaved per shape in one process.  Uniform [-1, 1) operands.

    python bench/xgemm_probe.py [--out gpurun_out/xgemm_probe.jsonl] [--cfgs 20,21,23] [--shapes sq,vit]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rocket_amd.ops.mgemm import mgemm  # noqa: E402


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
    ap.add_argument("--out", default="gpurun_out/xgemm_probe.jsonl")
    ap.add_argument("--cfgs", default="0,20,21,22,23")
    ap.add_argument("--shapes", default="sq,vit")
    ap.add_argument("--dirs", default="fwd,dgrad,wgrad")
    ap.add_argument("--splits", default="1,2,4,6,8")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    cfgs = [int(c) for c in args.cfgs.split(",")]
    out = open(args.out, "w")

    def r(*s):
        return (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)

    cases = []
    if "sq" in args.shapes:
        for n in (4096, 8192):
            cases.append((f"sq{n}", "fwd", n, n, n))
    if "vit" in args.shapes:
        M = 128 * 197
        for name, (kin, nout) in {"qkv": (768, 2304), "proj": (768, 768), "fc1": (768, 3072),
                                  "fc2": (3072, 768)}.items():
            for d in args.dirs.split(","):
                cases.append((name, d, M, kin, nout))
    for name, d, M, kin, nout in cases:
        if name.startswith("sq"):
            a, b = r(M, kin), r(nout, kin)
            spec = (a, b, False, False, M, nout, kin, kin, kin, lambda: a @ b.t(), lambda: a.float() @ b.float().t())
        else:
            x, w, dy = r(M, kin), r(nout, kin) * 0.05, r(M, nout)
            spec = {
                "fwd": (x, w, False, False, M, nout, kin, kin, kin, lambda: x @ w.t(), lambda: x.float() @ w.float().t()),
                "dgrad": (dy, w, False, True, M, kin, nout, nout, kin, lambda: dy @ w, lambda: dy.float() @ w.float()),
                "wgrad": (dy, x, True, True, nout, kin, M, nout, kin, lambda: dy.t() @ x,
                          lambda: dy.float().t() @ x.float()),
            }[d]
        a, b, ak, bk, gM, gN, gK, lda, ldb, tfn, rfn = spec
        ref = rfn()
        scale = ref.abs().max().item()
        flop = 2.0 * gM * gN * gK
        rec = {"case": name, "dir": d, "M": gM, "N": gN, "K": gK}
        runs = {"lib": tfn}
        splits = [int(s) for s in args.splits.split(",")] if d == "wgrad" else [1]
        for t in cfgs:
            if t == 22 and ak:
                continue
            for s in splits:
                odt = torch.float32 if d == "wgrad" else torch.bfloat16
                c = torch.zeros(gM, gN, dtype=odt, device=dev)

                def run(c=c, t=t, s=s):
                    mgemm(a, b, c, M=gM, N=gN, K=gK, lda=lda, ldb=ldb, ldc=gN, a_kmaj=ak, b_kmaj=bk, splitk=s, tile=t)

                try:
                    run()
                    torch.cuda.synchronize()
                except Exception as e:  # unsupported config for this shape
                    rec[f"t{t}s{s}"] = {"error": str(e)[:160]}
                    continue
                err = (c.float() - ref).abs().max().item() / scale
                rec[f"t{t}s{s}"] = {"rel_err": float(f"{err:.3g}")}
                runs[f"t{t}s{s}"] = run
        # interleaved timing rounds
        times = {k: [] for k in runs}
        for _ in range(3):
            for k, fn in runs.items():
                times[k].append(timeit(fn, 10))
        for k, ts in times.items():
            tm = sorted(ts)[len(ts) // 2]
            entry = rec.setdefault(k, {})
            entry.update(ms=round(tm, 4), tflops=round(flop / tm / 1e9, 1))
        ok = [(v["ms"], k) for k, v in rec.items() if isinstance(v, dict) and "ms" in v and k != "lib"]
        best = min(ok) if ok else (float("nan"), None)
        rec["best"] = best[1]
        rec["best_vs_lib"] = round(rec["lib"]["ms"] / best[0], 3) if ok else None
        print(json.dumps(rec), flush=True)
        out.write(json.dumps(rec) + "\n")
        out.flush()


if __name__ == "__main__":
    main()
