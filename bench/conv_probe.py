"""Probe MIOpen conv throughput for ResNet layer shapes: layout x dtype, fwd+bwd (for choosing the conv path)."""
import json
import sys
import time

import torch
import torch.nn.functional as F


def run(n, c, h, k, r, stride, fmt, dtype, iters=10):
    dev = torch.device("cuda", 0)
    x = torch.randn(n, c, h, h, device=dev, dtype=dtype).to(memory_format=fmt).requires_grad_(True)
    w = torch.randn(k, c, r, r, device=dev, dtype=dtype).to(memory_format=fmt).requires_grad_(True)
    for _ in range(3):
        y = F.conv2d(x, w, stride=stride, padding=r // 2)
        y.backward(torch.ones_like(y))
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        y = F.conv2d(x, w, stride=stride, padding=r // 2)
        y.backward(torch.ones_like(y))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / iters
    ho = (h + 2 * (r // 2) - r) // stride + 1
    flops = 3 * 2 * n * k * c * r * r * ho * ho
    return dt * 1e3, flops / dt / 1e12


shapes = [(256, 64, 32, 64, 3, 1), (256, 128, 16, 128, 3, 1), (256, 64, 56, 64, 3, 1), (256, 256, 56, 64, 1, 1),
          (256, 512, 7, 512, 3, 1)]
for s in shapes:
    for fmt, fn in ((torch.channels_last, "nhwc"), (torch.contiguous_format, "nchw")):
        ms, tf = run(*s, fmt, torch.bfloat16)
        print(json.dumps(dict(shape=s, fmt=fn, ms=round(ms, 3), tflops=round(tf, 1))), flush=True)
