"""The overlapped, captured data-parallel step (``DataParallel.capture_mode == "overlap"``).

On the single-GPU box a stand-in transport reduces every bucket with a recognisable kernel
(``nan_to_num_``) on the reducer's side stream, forked from the gradient hook with an event and joined
before the optimizer — exactly the stream/event pattern of the native RCCL reducer
(``native/runtime/comm.cpp``).  The captured graph is then inspected node by node
(``runtime/native.py`` ``describe_graph``): every bucket's reduction is its own branch that
depends on the backward kernel producing the bucket's last gradient, runs concurrently with the
backward kernels of earlier layers, and precedes the optimizer update.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu


class _FakeReducer:
    def __init__(self, flats):
        self.flats = list(flats)
        self.stream = torch.cuda.Stream(priority=-1)
        self.done = [torch.cuda.Event() for _ in self.flats]
        self.pending = set()
        self.order = []

    def launch(self, i):
        cur = torch.cuda.current_stream()
        ready = torch.cuda.Event()
        ready.record(cur)
        self.stream.wait_event(ready)
        with torch.cuda.stream(self.stream):
            self.flats[i].nan_to_num_()  # identity "all-reduce" of a world-1 group (distinct kernel)
            self.done[i].record(self.stream)
        self.pending.add(i)
        self.order.append(i)

    def join(self):
        cur = torch.cuda.current_stream()
        for i in sorted(self.pending):
            cur.wait_event(self.done[i])
        self.pending.clear()


class _FakeComm:
    native = False
    world, rank, avg_native = 1, 0, True

    def broadcast(self, t, src=0):
        return None

    def make_reducer(self, flats):
        self.reducer = _FakeReducer(flats)
        return self.reducer


def _ancestors(n, edges):
    pred = [[] for _ in range(n)]
    for a, b in edges:
        pred[b].append(a)
    memo = {}

    def anc(i):
        if i not in memo:
            s = set()
            for p in pred[i]:
                s.add(p)
                s |= anc(p)
            memo[i] = s
        return memo[i]

    return [anc(i) for i in range(n)]


def test_overlapped_bucket_reduce_is_a_parallel_branch(monkeypatch):
    monkeypatch.setenv("ROCKET_P2P", "0")
    from rocket_amd.ops.optim import FusedSGD
    from rocket_amd.parallel.ddp import DataParallel
    from rocket_amd.runtime.native import LaunchList, describe_graph

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    layers = []
    for _ in range(6):
        layers += [torch.nn.Linear(256, 256), torch.nn.ReLU()]
    net = torch.nn.Sequential(*layers, torch.nn.Linear(256, 10)).to(dev)
    comm = _FakeComm()
    dp = DataParallel(net, comm=comm, first_bucket_mb=0.2, bucket_cap_mb=0.5)
    assert dp.capture_mode == "overlap" and len(dp.buckets) >= 4
    opt = FusedSGD(net.parameters(), lr=0.01, momentum=0.9)
    x = torch.randn(64, 256, device=dev)

    def step():
        dp(x).square().mean().backward()
        opt.launch(zero_grads=True)

    dp(x).square().mean().backward()  # eager: creates .grad views, primes the optimizer tables
    assert opt.prepare()
    opt.launch(zero_grads=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()

    g = torch.cuda.CUDAGraph(keep_graph=True)
    comm.reducer.order.clear()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        step()
    assert sorted(comm.reducer.order) == list(range(len(dp.buckets)))  # each bucket launched once

    nodes, edges = describe_graph(g)
    anc = _ancestors(len(nodes), edges)
    red = [i for i, (t, name) in enumerate(nodes) if "nan_to_num" in name]
    opt_nodes = [i for i, (t, name) in enumerate(nodes) if "sgd_mt" in name]
    assert len(red) == len(dp.buckets), nodes
    assert len(opt_nodes) == 1
    o = opt_nodes[0]
    kern = [i for i, (t, _) in enumerate(nodes) if t == 0 and i not in red and i != o]
    for r in red:
        assert r in anc[o], "optimizer must wait for every bucket's reduction"
        assert any(k in anc[r] for k in kern), "a reduction must follow the backward kernel that completes its bucket"
    # the first bucket's reduction overlaps backward work of earlier layers: some backward kernel
    # is neither its ancestor nor its descendant (a parallel branch of the graph)
    first = min(red, key=lambda r: len(anc[r]))
    concurrent = [k for k in kern if k not in anc[first] and first not in anc[k]]
    assert concurrent, "bucket all-reduce is serialised with the rest of backward"
    ll, why = LaunchList.build(g)
    assert ll is None and "parallel" in why

    # replaying the graph gives the eager step's result from the same state
    params = list(net.parameters())
    snap = [(p.detach().clone(), opt.state[p]["momentum_buffer"].clone()) for p in params]

    def restore():
        with torch.no_grad():
            for p, (w, m) in zip(params, snap):
                p.copy_(w)
                opt.state[p]["momentum_buffer"].copy_(m)

    step()
    torch.cuda.synchronize()
    eager = [p.detach().clone() for p in params]
    restore()
    g.replay()
    torch.cuda.synchronize()
    for p, e in zip(params, eager):
        torch.testing.assert_close(p.detach(), e, rtol=1e-5, atol=1e-6)


def test_native_rccl_reducer_graph_structure(monkeypatch):
    """The REAL native reducer (``parallel/rccl.py`` NativeReducer over an RcclComm, world 1 on the
    single-GPU box) captured with forward/backward and the optimizer: the RCCL nodes it leaves in
    the graph sit on branches parallel to backward work and precede the optimizer."""
    monkeypatch.setenv("ROCKET_P2P", "0")
    from rocket_amd.ops.optim import FusedSGD
    from rocket_amd.parallel.ddp import DataParallel
    from rocket_amd.parallel.rccl import RcclComm
    from rocket_amd.runtime import comm as rcomm
    from rocket_amd.runtime.native import describe_graph

    rcomm.init()
    dev = torch.device("cuda", 0)
    comm = RcclComm(dev)
    try:
        torch.manual_seed(0)
        layers = []
        for _ in range(6):
            layers += [torch.nn.Linear(256, 256), torch.nn.ReLU()]
        net = torch.nn.Sequential(*layers, torch.nn.Linear(256, 10)).to(dev)
        dp = DataParallel(net, comm=comm, first_bucket_mb=0.2, bucket_cap_mb=0.5)
        assert dp.capture_mode == "overlap" and dp._native is not None and len(dp.buckets) >= 4
        opt = FusedSGD(net.parameters(), lr=0.01, momentum=0.9)
        x = torch.randn(64, 256, device=dev)

        def step():
            dp(x).square().mean().backward()
            opt.launch(zero_grads=True)

        dp(x).square().mean().backward()
        assert opt.prepare()
        opt.launch(zero_grads=True)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            step()
        nodes, edges = describe_graph(g)
        anc = _ancestors(len(nodes), edges)
        opt_nodes = [i for i, (t, name) in enumerate(nodes) if "sgd_mt" in name]
        assert len(opt_nodes) == 1, nodes
        o = opt_nodes[0]
        red = [i for i, (t, name) in enumerate(nodes) if "nccl" in name.lower() or "rccl" in name.lower()]
        print(f"captured graph: {len(nodes)} nodes, {len(red)} RCCL nodes: {[nodes[i] for i in red][:4]}")
        if not red:
            pytest.skip("RCCL emits no graph node for a world-1 all-reduce (nothing to place)")
        kern = [i for i, (t, _) in enumerate(nodes) if t == 0 and i not in red and i != o]
        for r in red:
            assert r in anc[o], "optimizer must wait for every bucket's RCCL all-reduce"
        first = min(red, key=lambda r: len(anc[r]))
        concurrent = [k for k in kern if k not in anc[first] and first not in anc[k]]
        assert concurrent, "RCCL all-reduce is serialised with the rest of backward"
        g.replay()
        torch.cuda.synchronize()
    finally:
        comm.close()
