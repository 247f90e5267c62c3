"""Isolated timing of rk_conv_dgrad (stride 1 vs the stride-2 parity-class launch) against the
library's conv2d_input at ResNet-50 shapes.  Prints one JSON line per case."""
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from rocket_amd.ops import _lib


def t_ms(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def case(N, C, H, Co, k, stride):
    pad = k // 2
    OH = (H + 2 * pad - k) // stride + 1
    cl = torch.channels_last
    w = torch.randn(Co, C, k, k, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    dy = torch.randn(N, Co, OH, OH, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    dx = torch.empty(N, C, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
    lib = _lib.kernels()
    st = _lib.stream_ptr(dy.device)

    def nat():
        _lib.check(lib.rk_conv_dgrad(1, dy.data_ptr(), w.data_ptr(), dx.data_ptr(), 1, 0, N, H, H, C, Co, k, k, stride,
                                     pad, OH, OH, st), "dgrad")

    def ref():
        torch.nn.grad.conv2d_input((N, C, H, H), w, dy, stride=stride, padding=pad)

    flops = 2.0 * N * OH * OH * Co * C * k * k
    tn, tl = t_ms(nat), t_ms(ref)
    print(json.dumps({"N": N, "C": C, "H": H, "Co": Co, "k": k, "stride": stride, "native_us": round(tn * 1e3, 1),
                      "lib_us": round(tl * 1e3, 1), "native_TF": round(flops / tn / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    for args in [(256, 1024, 14, 2048, 1, 2), (256, 1024, 7, 2048, 1, 1), (256, 256, 56, 512, 1, 2),
                 (256, 256, 28, 512, 1, 1), (256, 128, 56, 128, 3, 2), (256, 128, 28, 128, 3, 1),
                 (256, 512, 14, 512, 3, 2), (256, 512, 7, 512, 3, 1)]:
        case(*args)
