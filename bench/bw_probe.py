"""HBM streaming ceiling on this box: torch copy / add / fill on a 411 MB bf16 tensor (ResNet-50's
largest BatchNorm shape), effective TB/s (bytes moved / time), for comparison with the fused
BatchNorm passes (bench/bn_probe.py)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=20):
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
    dev = torch.device("cuda", 0)
    n = 256 * 256 * 56 * 56
    x = torch.randn(n, device=dev, dtype=torch.bfloat16)
    r = torch.randn_like(x)
    y = torch.empty_like(x)
    b = 2 * n
    rec = {}
    for name, fn, nb in [("copy", lambda: y.copy_(x), 2 * b), ("add", lambda: torch.add(x, r, out=y), 3 * b),
                         ("fill", lambda: y.fill_(1.0), b), ("sum", lambda: x.sum(), b)]:
        ms = timed(fn)
        rec[name] = {"ms": round(ms, 3), "TBps": round(nb / ms / 1e9, 2)}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
