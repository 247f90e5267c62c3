"""LayerNorm backward (rk_ln_bwd) on the ViT-B/16 residual-stream shape (25216 x 768, fp32 x / dx /
dsum, bf16 dy / dres, + dgamma / dbeta / dres column sums) over its grid and prefetch settings
(rk_ln_set_bwd_cfg), with the effective bandwidth of the streamed tensors.  Median of 20.

    python bench/ln_probe.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bench.xgemm_probe import timeit  # noqa: E402
from rocket_amd.ops import _lib  # noqa: E402


def main():
    dev = torch.device("cuda")
    lib = _lib.kernels()
    R, C = 128 * 197, 768
    x = torch.randn(R, C, device=dev)
    dsum = torch.randn(R, C, device=dev)
    dy = torch.randn(R, C, device=dev).to(torch.bfloat16)
    g = torch.randn(C, device=dev)
    mean = x.mean(1)
    rstd = torch.rsqrt(x.var(1, unbiased=False) + 1e-6)
    dx = torch.empty_like(x)
    dres = torch.empty_like(dy)
    dgam, dbet, dsb = (torch.zeros(C, device=dev) for _ in range(3))
    ctr = _lib.Workspace.get(dev).counter("ln_probe")
    nbytes = (3 * 4 + 2 * 2) * R * C
    for rpb, pf in ((16, 1), (16, 0), (32, 1), (64, 1), (0, 1)):
        _lib.check(lib.rk_ln_set_bwd_cfg(rpb, pf), "cfg")
        ws = torch.empty(int(lib.rk_ln_workspace(R, C)), device=dev)

        def run():
            _lib.check(lib.rk_ln_bwd(0, 1, dy.data_ptr(), x.data_ptr(), g.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                     dx.data_ptr(), dsum.data_ptr(), dres.data_ptr(), dgam.data_ptr(), dbet.data_ptr(),
                                     dsb.data_ptr(), None, R, C, ws.data_ptr(), ctr, _lib.stream_ptr(dev)), "rk_ln_bwd")

        ms = timeit(run)
        print(json.dumps({"rpb": rpb, "prefetch": pf, "us": round(ms * 1e3, 1), "TB/s": round(nbytes / ms / 1e9, 2)}),
              flush=True)
    _lib.check(lib.rk_ln_set_bwd_cfg(16, 1), "cfg")


if __name__ == "__main__":
    main()
