"""Fused BatchNorm(+residual+ReLU) HIP kernels vs PyTorch/MIOpen BN + add + relu, ResNet-50 shapes (bf16, NHWC).

Prints one JSON line per shape: fused and torch fwd+bwd ms, and the effective HBM GB/s of the fused path.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from rocket_amd.ops.norm import BatchNormAct2d


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    dev = torch.device("cuda", 0)
    for (n, c, h, res) in [(256, 256, 56, True), (256, 64, 56, False), (256, 512, 28, True), (256, 128, 28, False),
                           (256, 1024, 14, True), (256, 2048, 7, True)]:
        x = torch.randn(n, c, h, h, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        r = torch.randn_like(x) if res else None
        x.requires_grad_(True)
        bn = BatchNormAct2d(c, relu=True).to(dev)
        ref = torch.nn.BatchNorm2d(c).to(dev)
        gy = torch.randn_like(x)

        def fused():
            y = bn(x, residual=r)
            y.backward(gy)

        def torch_path():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = ref(x)
                if r is not None:
                    y = y + r
                y = F.relu(y)
            y.backward(gy)

        tf = bench(fused)
        tt = bench(torch_path)
        elems = x.numel()
        # fwd: stats read x; apply read x (+r) write y + 1-bit ReLU mask.  bwd: reduce read dy,x,mask;
        # apply read dy,x,mask write dx (+dres)
        nbytes = 2 * elems * (1 + 2 + (1 if res else 0) + 2 + 3 + (1 if res else 0) + 3 / 16)
        print(json.dumps(dict(shape=[n, c, h, h], residual=res, fused_ms=round(tf, 3), torch_ms=round(tt, 3),
                              fused_GBps=round(nbytes / tf / 1e6, 1))), flush=True)


if __name__ == "__main__":
    main()
