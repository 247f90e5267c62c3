"""Do parallel branches of a replayed HIP graph run concurrently on MI355X?

The overlapped data-parallel step (``runtime/graphs.py``, capture mode ``overlap``) relies on it:
each bucket all-reduce is a branch forked off backward.  Two chains of small latency-bound
spin kernels (each holds one CU for a fixed time) are captured (a) on one stream, (b) on two
streams forked from the capture stream and joined at the end; if hipGraphLaunch executes the
branches concurrently, (b) takes about half of (a).  Reported for the current
DEBUG_CLR_GRAPH_PACKET_CAPTURE setting (run it with both).

    python bench/graph_branch_probe.py   ->  one JSON line
"""

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


SPIN_US, N_SPIN = 100.0, 4


def chain(x, n):
    """n spin kernels of SPIN_US each on one CU (known duration, tiny footprint)."""
    from rocket_amd.ops import _lib

    lib = _lib.kernels()
    for _ in range(N_SPIN):
        lib.rk_spin(SPIN_US, 1, x.data_ptr(), _lib.stream_ptr(x.device))
    return x


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    import rocket_amd  # noqa: F401  (HIP env defaults, as in training)

    dev = torch.device("cuda", 0)
    a = torch.zeros(64 * 1024, device=dev)  # 256 KB: a few workgroups per kernel
    b = torch.zeros(64 * 1024, device=dev)
    n = 200
    side = torch.cuda.Stream()

    def serial():
        chain(a, n)
        chain(b, n)

    def forked():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            chain(b, n)
        chain(a, n)
        cur.wait_stream(side)

    out = {"packet_capture": os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE"), "spin_us": SPIN_US, "spins": N_SPIN}
    for name, fn in (("serial", serial), ("forked", forked)):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        out[f"graph_{name}_ms"] = round(timed(g.replay), 4)
        out[f"eager_{name}_ms"] = round(timed(fn), 4)
    out["graph_branch_speedup"] = round(out["graph_serial_ms"] / out["graph_forked_ms"], 3)
    out["eager_branch_speedup"] = round(out["eager_serial_ms"] / out["eager_forked_ms"], 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
