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
    ap.add_argument("--cfgs", default="0", help="conv pipelines to A/B (rk_conv_set_cfg), e.g. 0,1,2,3")
    ap.add_argument("--check", action="store_true", help="compare every pipeline's outputs with pipeline 0's")
    ap.add_argument("--only", default="", help="shapes to run, e.g. 'c128h16k3s1,c64h32k3s1' (Cin, H, kernel, stride)")
    ap.add_argument("--dirs", default="fwd,dgrad,wgrad")
    a = ap.parse_args()
    cfgs = [int(c) for c in a.cfgs.split(",")]
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
        if a.only and f"c{C}h{H}k{r}s{st}" not in a.only.split(","):
            continue
        xc = torch.randn(xs, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(co, C, r, r, device=dev).contiguous(memory_format=torch.channels_last)
        w16 = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        geo = iconv._geo(xc, w16, st, pad)
        OH, OW = geo[-2], geo[-1]
        dy = torch.randn(N, co, OH, OW, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        flops = 2.0 * N * OH * OW * co * C * r * r
        lib = iconv._kernels()
        fns = {
            "fwd": lambda: iconv._conv_fwd(xc, w16, st, pad, None),
            "dgrad": lambda: iconv._conv_dgrad(dy, w16, geo, None),
            "wgrad": lambda: iconv._conv_wgrad(dy, xc, w, geo),
        }
        fns = {d: f for d, f in fns.items() if d in a.dirs.split(",")}
        rec = dict(x=list(xs), cout=co, k=r, stride=st, count=cnt)
        ref = {}
        for rep in range(2):  # interleaved rounds (one process): the second round is reported
            for c in cfgs:
                lib.rk_conv_set_cfg(c)
                for d, fn in fns.items():
                    ms = timed(fn)
                    if rep == 1:
                        rec[f"{d}_us_c{c}"] = round(ms * 1e3, 1)
                        rec[f"{d}_tf_c{c}"] = round(flops / (ms * 1e-3) / 1e12, 1)
                        total[(c, d)] += ms * cnt
                    if a.check and rep == 0:
                        out = fn()
                        out = out[0] if isinstance(out, tuple) else out
                        if c == cfgs[0]:
                            ref[d] = out.float().clone()
                        else:
                            err = (out.float() - ref[d]).abs().max().item() / (ref[d].abs().max().item() + 1e-6)
                            rec[f"{d}_relerr_c{c}"] = err
        lib.rk_conv_set_cfg(cfgs[0])
        print(json.dumps(rec), flush=True)
    for c in cfgs:
        print(json.dumps({"cfg": c, "total_ms_per_step": {d: round(total[(c, d)], 3) for d in ("fwd", "dgrad", "wgrad") if d in a.dirs.split(",")},
                          "sum_ms": round(sum(total[(c, d)] for d in a.dirs.split(",")), 3)}), flush=True)


if __name__ == "__main__":
    main()
