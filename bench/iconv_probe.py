"""Per-layer-shape timing of the native implicit-GEMM convs (forward, dgrad, wgrad) of a ResNet.

Every distinct conv geometry of the model (with its multiplicity in one step) is timed in
isolation with HIP events on random bf16 NHWC operands, so the step's conv time can be attributed
to shapes and directions (which tiles / shapes to optimise first).

    python bench/iconv_probe.py [--model resnet50] [--batch 256]  ->  one JSON line per shape + a total
"""

import argparse
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    from rocket_amd import models
    from rocket_amd.ops import iconv

    dev = torch.device("cuda", 0)
    res = 32 if a.model == "resnet18" else 224
    net = {"resnet18": lambda: models.resnet18(10), "resnet50": lambda: models.resnet50(1000)}[a.model]()
    net = net.to(dev).to(memory_format=torch.channels_last)
    shapes = collections.Counter()

    def hook(mod, inp, out):
        x = inp[0]
        if iconv.native_ok(mod, x):
            shapes[(tuple(x.shape), mod.out_channels, mod.kernel_size[0], mod.stride[0], mod.padding[0])] += 1

    for m in net.modules():
        if isinstance(m, iconv.IConv2d):
            m.register_forward_hook(hook)
    x = torch.randn(a.batch, 3, res, res, device=dev, dtype=torch.bfloat16)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        net.logits(x)
    total = collections.Counter()
    for (xs, co, r, st, pad), cnt in sorted(shapes.items(), key=lambda kv: -kv[1]):
        N, C, H, W = xs
        xc = torch.randn(xs, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(co, C, r, r, device=dev).contiguous(memory_format=torch.channels_last)
        w16 = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        geo = iconv._geo(xc, w16, st, pad)
        OH, OW = geo[-2], geo[-1]
        dy = torch.randn(N, co, OH, OW, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        flops = 2.0 * N * OH * OW * co * C * r * r
        t = {
            "fwd": timed(lambda: iconv._conv_fwd(xc, w16, st, pad, None)),
            "dgrad": timed(lambda: iconv._conv_dgrad(dy, w16, geo, None)),
            "wgrad": timed(lambda: iconv._conv_wgrad(dy, xc, w, geo)),
        }
        rec = dict(x=list(xs), cout=co, k=r, stride=st, count=cnt)
        for d, ms in t.items():
            rec[f"{d}_us"] = round(ms * 1e3, 1)
            rec[f"{d}_tf"] = round(flops / (ms * 1e-3) / 1e12, 1)
            total[d] += ms * cnt
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_ms_per_step": {d: round(v, 3) for d, v in total.items()},
                      "sum_ms": round(sum(total.values()), 3)}), flush=True)


if __name__ == "__main__":
    main()
