"""Dispatch gap between two dependent kernels vs the bytes the first one wrote (diagnostics).

A 1-block spin kernel first fills the queue; then a writer kernel (256 blocks, each writing
bytes/256, plain or nontemporal stores) and a 256-block stamper are enqueued back to back.  The gap
= stamper's first block start - writer's last block end (s_memrealtime, 100 MHz), median of 20.
If it grows with the bytes written, the kernel-boundary release (dirty L2 written back so the
other XCDs see the data) is on the critical path of dependent launch chains like the LeNet step.

    python bench/gap_probe.py  ->  one JSON line per (bytes, store kind)
"""

import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from rocket_amd.ops import _lib

    lib = _lib.kernels()
    dev = torch.device("cuda", 0)
    s = _lib.stream_ptr(dev)
    blocks = 256
    buf = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    sink = torch.zeros(64, device=dev)
    wtr = torch.zeros(blocks, 2, dtype=torch.int64, device=dev)
    rtr = torch.zeros(blocks, dtype=torch.int64, device=dev)
    for total in (0, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20):
        for nt in (0, 1):
            gaps, spans = [], []
            for _ in range(20):
                lib.rk_spin(30.0, 1, sink.data_ptr(), s)
                _lib.check(lib.rk_gap_write(buf.data_ptr(), total // blocks, blocks, nt, wtr.data_ptr(), s), "gap_write")
                _lib.check(lib.rk_gap_stamp(blocks, rtr.data_ptr(), 0, s), "gap_stamp")
                torch.cuda.synchronize()
                w, r = wtr.cpu(), rtr.cpu()
                gaps.append(float(r.min() - w[:, 1].max()) * 0.01)
                spans.append(float(w[:, 1].max() - w[:, 0].min()) * 0.01)
            print(json.dumps({"bytes": total, "nontemporal": nt, "gap_us_median": round(statistics.median(gaps), 2),
                              "gap_us_min": round(min(gaps), 2), "writer_span_us": round(statistics.median(spans), 2)}),
                  flush=True)


def any_order():
    """Does hipExtAnyOrderLaunch let a kernel start before the previous one on the stream ends?
    A 1-block 40 us spin, then a stamper launched with / without the flag."""
    from rocket_amd.ops import _lib

    lib = _lib.kernels()
    dev = torch.device("cuda", 0)
    s = _lib.stream_ptr(dev)
    sink = torch.zeros(64, device=dev)
    rtr = torch.zeros(4, dtype=torch.int64, device=dev)
    base = torch.zeros(1, dtype=torch.int64, device=dev)
    import time

    for spin_blocks in (1, 109, 256, 1024):
        for flag in (0, 1):
            for host_delay in (0.0, 20e-6):
                ds = []
                for _ in range(10):
                    _lib.check(lib.rk_gap_stamp(1, base.data_ptr(), 0, s), "gap_stamp")
                    lib.rk_spin(40.0, spin_blocks, sink.data_ptr(), s)
                    t = time.perf_counter()
                    while time.perf_counter() - t < host_delay:  # the stamper's packet arrives later
                        pass
                    _lib.check(lib.rk_gap_stamp(4, rtr.data_ptr(), flag, s), "gap_stamp")
                    torch.cuda.synchronize()
                    ds.append(float(rtr.min() - base[0]) * 0.01)
                print(json.dumps({"spin_blocks": spin_blocks, "any_order": flag, "host_delay_us": host_delay * 1e6,
                                  "stamper_start_after_spin_start_us": round(statistics.median(ds), 2),
                                  "note": "< 40 us: the stamper overlapped the spin"}), flush=True)


def big_blocks():
    """Gap after a 4 MB writer for a stamper of 64-thread blocks vs 1024-thread blocks with 0 / 64 /
    137 KB of LDS (the LeNet step kernel's shape)."""
    from rocket_amd.ops import _lib

    lib = _lib.kernels()
    dev = torch.device("cuda", 0)
    s = _lib.stream_ptr(dev)
    buf = torch.empty(4 << 20, dtype=torch.uint8, device=dev)
    sink = torch.zeros(64, device=dev)
    wtr = torch.zeros(256, 2, dtype=torch.int64, device=dev)
    rtr = torch.zeros(256, dtype=torch.int64, device=dev)
    for lds in (-1, 0, 65536, 137936):
        gaps = []
        for _ in range(20):
            lib.rk_spin(30.0, 1, sink.data_ptr(), s)
            _lib.check(lib.rk_gap_write(buf.data_ptr(), (4 << 20) // 256, 256, 0, wtr.data_ptr(), s), "gap_write")
            if lds < 0:
                _lib.check(lib.rk_gap_stamp(256, rtr.data_ptr(), 0, s), "gap_stamp")
            else:
                _lib.check(lib.rk_gap_stamp_big(256, rtr.data_ptr(), lds, s), "gap_stamp_big")
            torch.cuda.synchronize()
            gaps.append(float(rtr.min() - wtr[:, 1].max()) * 0.01)
        print(json.dumps({"stamper": "64 threads" if lds < 0 else f"1024 threads, {lds} B LDS",
                          "gap_us_median": round(statistics.median(gaps), 2)}), flush=True)


if __name__ == "__main__":
    any_order()
    main()
