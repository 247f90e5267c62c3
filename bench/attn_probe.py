"""Attention kernels at the ViT-B/16 shape (B=128, L=197, H=12, D=64): forward, fused backward,
split backward (median of HIP-event timings) -> one JSON line."""

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
    return ts[len(ts) // 2] * 1e3


def main():
    from rocket_amd.ops import _lib
    from rocket_amd.ops.activation import _attn_lib

    B, L, H, D = 128, 197, 12, 64
    lib = _attn_lib()
    dev = torch.device("cuda", 0)
    qkv = torch.randn(B, L, 3 * H * D, device=dev).to(torch.bfloat16)
    out = torch.empty(B, L, H * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H, L, device=dev)
    dout = torch.randn_like(out)
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(B * H, L, device=dev)
    C3, HD, es = 3 * H * D, H * D, 2
    base, gbase = qkv.data_ptr(), dqkv.data_ptr()
    s = _lib.stream_ptr(dev)

    def fwd():
        lib.rk_attn_fwd(base, base + HD * es, base + 2 * HD * es, C3, out.data_ptr(), HD, lse.data_ptr(), B, L, H,
                        0.125, s)

    def bwd():
        lib.rk_attn_bwd(base, base + HD * es, base + 2 * HD * es, C3, out.data_ptr(), dout.data_ptr(), HD,
                        lse.data_ptr(), delta.data_ptr(), gbase, gbase + HD * es, gbase + 2 * HD * es, C3, B, L, H,
                        0.125, s)

    fwd()
    rec = {"fwd_us": round(timed(fwd), 1)}
    lib.rk_attn_set_bwd_fused(1)
    rec["bwd_fused_us"] = round(timed(bwd), 1)
    # phase stamps of the fused kernel (delta doubles as the stamp buffer: 4 floats per block)
    stamps = torch.zeros(B * H * 4, device=dev)
    lib.rk_attn_set_stamps(stamps.data_ptr())
    bwd()
    torch.cuda.synchronize()
    lib.rk_attn_set_stamps(None)
    st = stamps.view(-1, 4).median(0).values / 100.0  # 100 MHz ticks -> us
    rec["fused_phase_us"] = {"staged": round(float(st[1]), 2), "loop_done": round(float(st[2]), 2),
                             "end": round(float(st[3]), 2)}
    lib.rk_attn_set_bwd_fused(2)
    rec["bwd_stream_us"] = round(timed(bwd), 1)
    stamps.zero_()
    lib.rk_attn_set_stamps(stamps.data_ptr())
    bwd()
    torch.cuda.synchronize()
    lib.rk_attn_set_stamps(None)
    st = stamps.view(-1, 4).median(0).values / 100.0
    rec["stream_phase_us"] = {"staged": round(float(st[1]), 2), "loop_done": round(float(st[2]), 2),
                              "end": round(float(st[3]), 2)}
    lib.rk_attn_set_bwd_fused(0)
    rec["bwd_split_us"] = round(timed(bwd), 1)
    lib.rk_attn_set_bwd_fused(1)
    flops = 4.0 * B * H * L * L * D
    rec["fwd_tf"] = round(flops / rec["fwd_us"] / 1e6, 1)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
