"""Back-to-back HIP-graph replay cost on this box (what a launch-bound step pays per replay).

    python bench/graph_launch_probe.py

Captures a graph of K tiny kernels and times 2000 replays in a row: (a) replay only, (b) an eager
kernel launch before every replay (the loader's gather), (c) plus a timing-event record per step
(StepTimer), (d) the same K kernels launched eagerly, (e) one graph holding 4 steps (4K kernels),
(f) the graph replayed as a native launch list (rocket_amd.runtime.native.LaunchList), (g) an eager
kernel plus the launch list.
Prints one JSON line with microseconds per step for each variant.
"""

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


def main():
    dev = torch.device("cuda", 0)
    K = 6
    xs = [torch.zeros(256 * 1024, device=dev) for _ in range(K)]  # 1 MB each: ~1-2 us kernels

    def work(k=K):
        for i in range(k):
            xs[i % K].add_(1.0)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        work()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        work()
    gk = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(gk):
        work()
    from rocket_amd.runtime.native import LaunchList
    from rocket_amd.ops import _lib

    ll, why = LaunchList.build(gk)
    assert ll is not None, why
    sp = _lib.stream_ptr(dev)
    g4 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g4):
        work(4 * K)
    y = torch.zeros(1024 * 1024, device=dev)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(4096)]
    pos = [0]

    def with_event():
        y.add_(1.0)
        g.replay()
        evs[pos[0] % len(evs)].record()
        pos[0] += 1

    res = {
        "graph_replay_us": timed(g.replay),
        "kernel_plus_replay_us": timed(lambda: (y.add_(1.0), g.replay())),
        "kernel_replay_event_us": timed(with_event),
        "eager_K_kernels_us": timed(work),
        "graph_4_steps_per_replay_us": timed(g4.replay) / 4,
        "single_kernel_us": timed(lambda: y.add_(1.0)),
        "launch_list_us": timed(lambda: ll.launch(sp)),
        "kernel_plus_launch_list_us": timed(lambda: (y.add_(1.0), ll.launch(sp))),
    }
    print(json.dumps({k: round(v, 2) for k, v in res.items()}))


if __name__ == "__main__":
    main()
