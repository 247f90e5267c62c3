"""Native launch-list replay of captured HIP graphs (``native/runtime/launchlist.cpp``).

The list walks the captured graph once and re-issues its kernel nodes as plain stream launches;
replaying it must produce exactly what ``graph.replay()`` produces.  Graphs with copy/memset nodes
are refused (their parameters cannot be read back reliably) and keep graph replay.
"""

import pytest
import torch

from rocket_amd.ops import _lib
from rocket_amd.runtime.native import LaunchList

pytestmark = pytest.mark.gpu


def _capture(fn, warm=True):
    g = torch.cuda.CUDAGraph(keep_graph=True)
    if warm:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()  # warm-up outside the capture (allocator, lazy init)
        torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        fn()
    return g


def test_launch_list_matches_graph_replay():
    dev = torch.device("cuda", 0)
    a = torch.randn(4096, device=dev)
    b = torch.empty_like(a)
    c = torch.empty_like(a)
    acc = torch.zeros(4096, device=dev)
    raw = torch.zeros(1 << 16, dtype=torch.uint8, device=dev)

    def step():
        torch.add(a, 1.0, out=b)    # PyTorch kernels only
        torch.mul(b, 2.0, out=c)
        acc.add_(c)                 # accumulates across replays: replay count and order matter
        raw.fill_(7)

    g = _capture(step)
    ll, why = LaunchList.build(g)
    assert ll is not None, why
    assert ll.size == 4 and ll.kinds == [0, 0, 0, 0]
    acc.zero_()
    stream = _lib.stream_ptr(dev)
    for _ in range(5):
        ll.launch(stream)
    torch.cuda.synchronize()
    ref = torch.zeros_like(acc)
    for _ in range(5):
        ref.add_((a + 1.0) * 2.0)
    assert torch.equal(acc, ref)  # same kernels in the same order: bit-exact
    assert int(raw.min()) == 7 and int(raw.max()) == 7
    acc.zero_()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(acc, ref)


def test_launch_list_refuses_copy_nodes():
    dev = torch.device("cuda", 0)
    a = torch.randn(4096, device=dev)
    b = torch.empty_like(a)
    g = _capture(lambda: b.copy_(a))  # a device-to-device copy node
    ll, why = LaunchList.build(g)
    if ll is None:
        assert "memcpy" in why or "memset" in why, why
    g.replay()  # the caller's fallback still works
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_launch_list_runs_native_kernels():
    """A graph of this framework's own HIP kernels (the fused optimizer) replays identically."""
    from rocket_amd.ops.optim import FusedAdamW

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(n, device=dev)) for n in (1000, 37, 4096)]
    for p in ps:
        p.grad = torch.randn_like(p)
    ref = [p.detach().clone() for p in ps]
    opt = FusedAdamW(ps, lr=1e-2)
    opt.prepare()
    grads = [p.grad.detach().clone() for p in ps]
    g = _capture(lambda: opt.launch(zero_grads=False), warm=False)  # captured, not run
    ll, why = LaunchList.build(g)
    assert ll is not None, why
    opt2 = torch.optim.AdamW([torch.nn.Parameter(r.clone()) for r in ref], lr=1e-2)
    stream = _lib.stream_ptr(dev)
    for _ in range(3):
        for p, gr in zip(ps, grads):
            p.grad.copy_(gr)
        ll.launch(stream)
        for q, gr in zip(opt2.param_groups[0]["params"], grads):
            q.grad = gr.clone()
        opt2.step()
    torch.cuda.synchronize()
    for p, q in zip(ps, opt2.param_groups[0]["params"]):
        assert torch.allclose(p, q, atol=1e-5, rtol=1e-5), float((p - q).abs().max())
