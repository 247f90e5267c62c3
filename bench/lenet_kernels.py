"""Per-kernel timing of the LeNet hot path (HIP events, median of repeated launches).

    python bench/lenet_kernels.py [--batch 1024] [--reps 50]

Each native kernel of one fused LeNet training step is launched in isolation on
realistic inputs (one real step is run first to produce them) and timed with
``torch.cuda.Event``; one JSON line per kernel plus a summary line.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, reps, inner=20):
    """Median per-launch device time of `inner` back-to-back launches (host gaps amortised)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(max(3, reps // 5)):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(inner):
            fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / inner)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    from rocket_amd.models import CrossEntropy, LeNet
    from rocket_amd.ops import _lib
    from rocket_amd.ops.lenet import _LeNetFeatures, _MLPHead  # noqa: F401
    from rocket_amd.ops.optim import FusedAdamW

    lib = _lib.kernels()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    N = args.batch
    net = LeNet(fused=True).to(dev)
    x = torch.rand(N, 1, 28, 28, device=dev)
    y = torch.randint(0, 10, (N,), device=dev)
    opt = FusedAdamW(net.parameters())
    out = net((x, y))
    loss = CrossEntropy(fused=True)(out)
    loss.backward()
    opt.step()
    torch.cuda.synchronize()

    s = _lib.stream_ptr(dev)
    w1, b1, w2, b2 = (p.detach() for p in (net.conv1.weight, net.conv1.bias, net.conv2.weight, net.conv2.bias))
    a1 = torch.empty(N, 1176, dtype=torch.bfloat16, device=dev)
    c1 = torch.empty(N, 1176, dtype=torch.uint8, device=dev)
    a2 = torch.empty(N, 400, dtype=torch.bfloat16, device=dev)
    c2 = torch.empty(N, 400, dtype=torch.uint8, device=dev)
    gbuf = torch.zeros(10000, device=dev)
    res = {}
    res["lenet_conv_fwd"] = timeit(lambda: lib.rk_lenet_conv_fwd(x.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(), a1.data_ptr(), c1.data_ptr(), a2.data_ptr(), c2.data_ptr(), N, s), args.reps)
    da2 = (torch.randn(N, 400, device=dev) * 1e-3).to(torch.bfloat16)
    for rounds in (1, 2):
        res[f"lenet_conv_bwd_r{rounds}"] = timeit(lambda: lib.rk_lenet_conv_bwd(x.data_ptr(), a1.data_ptr(), c1.data_ptr(), da2.data_ptr(), c2.data_ptr(), w2.data_ptr(), gbuf.data_ptr(), gbuf[200:].data_ptr(), gbuf[400:].data_ptr(), gbuf[3000:].data_ptr(), N, rounds, s), args.reps)
    fc = [net.fc1, net.fc2, net.fc3]
    W = [l.weight.detach() for l in fc]
    B = [l.bias.detach() for l in fc]
    bf = dict(dtype=torch.bfloat16, device=dev)
    xT, h1T, h2T = torch.empty(400, N, **bf), torch.empty(120, N, **bf), torch.empty(84, N, **bf)
    logits = torch.empty(N, 10, device=dev)
    res["mlp3_fwd"] = timeit(lambda: lib.rk_mlp3_fwd(a2.data_ptr(), 400, W[0].data_ptr(), B[0].data_ptr(), 120, W[1].data_ptr(), B[1].data_ptr(), 84, W[2].data_ptr(), B[2].data_ptr(), 10, xT.data_ptr(), h1T.data_ptr(), h2T.data_ptr(), logits.data_ptr(), N, s), args.reps)
    dy = torch.randn(N, 10, device=dev) * 1e-3
    dyT, d2T, d1T, dx = torch.empty(10, N, **bf), torch.empty(84, N, **bf), torch.empty(120, N, **bf), torch.empty(N, 400, **bf)
    res["mlp3_dgrad"] = timeit(lambda: lib.rk_mlp3_dgrad(dy.data_ptr(), 10, W[2].data_ptr(), 84, h2T.data_ptr(), W[1].data_ptr(), 120, h1T.data_ptr(), W[0].data_ptr(), 400, dyT.data_ptr(), d2T.data_ptr(), d1T.data_ptr(), dx.data_ptr(), N, s), args.reps)
    import ctypes

    P, I = ctypes.c_void_p * 3, ctypes.c_int * 3
    gw = [torch.zeros_like(w) for w in W]
    gb = [torch.zeros_like(b) for b in B]
    probs = ((dyT, h2T, gw[2], gb[2], 10, 84), (d2T, h1T, gw[1], gb[1], 84, 120), (d1T, xT, gw[0], gb[0], 120, 400))
    args_w = (P(*[p[0].data_ptr() for p in probs]), P(*[p[1].data_ptr() for p in probs]), P(*[p[2].data_ptr() for p in probs]), P(*[p[3].data_ptr() for p in probs]), I(*[p[4] for p in probs]), I(*[p[5] for p in probs]))
    res["mlp3_wgrad"] = timeit(lambda: lib.rk_mlp3_wgrad(3, *args_w, N, None, 0, 0, None, None, s), args.reps)
    from rocket_amd.ops.cross_entropy import cross_entropy

    lg = logits.clone().requires_grad_()
    res["ce_fwd"] = timeit(lambda: cross_entropy(lg, y), args.reps)
    l = cross_entropy(lg, y)
    res["ce_fwd+bwd"] = timeit(lambda: torch.autograd.grad(cross_entropy(lg, y), lg), args.reps)
    res["adamw_step"] = timeit(lambda: opt.launch(), args.reps)
    res["index_select_x"] = timeit(lambda: x.index_select(0, y.sort().indices), args.reps)
    for k, v in res.items():
        print(json.dumps({"kernel": k, "us_median": round(v, 2)}))
    print(json.dumps({"sum_us": round(sum(v for k, v in res.items() if k not in ("lenet_conv_bwd_r2", "ce_fwd")), 1)}))


if __name__ == "__main__":
    main()
