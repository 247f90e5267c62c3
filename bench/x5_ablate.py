"""xgemm5 main-loop ablation (timing only): each bit removes one part of the k-loop (bench/gemm_r6_probe
shapes).  bit 0: in-loop DMA, 1: the per-k-tile barrier, 2: the fragment reads, 3: the lgkm waits."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench.gemm_r6_probe import SHAPES  # noqa: E402
from bench.xgemm_probe import timeit  # noqa: E402
from rocket_amd.ops import _lib  # noqa: E402

lib = _lib.kernels()
dev = torch.device("cuda")
for name in (sys.argv[1] if len(sys.argv) > 1 else "sq8192,qkv").split(","):
    m, n, k = SHAPES[name]
    x = (torch.rand(m, k, device=dev) * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(n, k, device=dev) * 2 - 1).to(torch.bfloat16)
    bias = torch.randn(n, device=dev)
    y = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
    rec = {"case": name}
    for tag, bits in (("full", 0), ("noDMA", 1), ("noBar", 2), ("noRead", 4), ("noWait", 8), ("noDMA_noBar", 3),
                      ("noDMA_noRead", 5), ("noAll", 15)):
        def f():
            lib.rk_xgemm5_set_shape(1 | (bits << 8))
            lib.rk_xgemm5(x.data_ptr(), k, w.data_ptr(), k, y.data_ptr(), n, 1, bias.data_ptr(), m, n, k,
                          _lib.stream_ptr(dev))
        ts = sorted(timeit(f) for _ in range(3))
        rec[tag] = round(2.0 * m * n * k / ts[1] / 1e9, 1)
    lib.rk_xgemm5_set_shape(0)
    print(json.dumps(rec), flush=True)
