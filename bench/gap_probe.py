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
                _lib.check(lib.rk_gap_stamp(blocks, rtr.data_ptr(), s), "gap_stamp")
                torch.cuda.synchronize()
                w, r = wtr.cpu(), rtr.cpu()
                gaps.append(float(r.min() - w[:, 1].max()) * 0.01)
                spans.append(float(w[:, 1].max() - w[:, 0].min()) * 0.01)
            print(json.dumps({"bytes": total, "nontemporal": nt, "gap_us_median": round(statistics.median(gaps), 2),
                              "gap_us_min": round(min(gaps), 2), "writer_span_us": round(statistics.median(spans), 2)}),
                  flush=True)


if __name__ == "__main__":
    main()
