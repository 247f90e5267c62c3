"""Native runtime on the GPU: own RCCL communicator (world 1 on the single-GPU box), the side-stream
bucket reducer inside a captured HIP graph, and the host loader's pinned staging + copy stream."""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl():
    from rocket_amd.parallel.rccl import RcclComm
    from rocket_amd.runtime import comm

    comm.init()
    c = RcclComm(torch.device("cuda", 0))
    yield c
    c.close()


def test_rccl_collectives_world1(rccl):
    dev = torch.device("cuda", 0)
    t = torch.arange(10, dtype=torch.float32, device=dev)
    rccl.all_reduce_avg(t).wait()
    assert torch.equal(t, torch.arange(10, dtype=torch.float32, device=dev))
    b = torch.arange(6, dtype=torch.bfloat16, device=dev)
    rccl.broadcast(b, 0)
    out = torch.empty(6, dtype=torch.bfloat16, device=dev)
    rccl.all_gather(out, b)
    rs = torch.empty(6, dtype=torch.bfloat16, device=dev)
    rccl.reduce_scatter(rs, b)
    torch.cuda.synchronize()
    assert torch.equal(out, b) and torch.equal(rs, b)


def test_native_reducer_in_graph(rccl):
    """DataParallel on the native transport: bucket launches on the side stream and the join are
    captured into one HIP graph together with forward/backward; replays match eager grads."""
    from rocket_amd.parallel.ddp import DataParallel

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.ReLU(), torch.nn.Linear(256, 10)).to(dev)
    dp = DataParallel(net, comm=rccl, first_bucket_mb=0.01, bucket_cap_mb=0.05)
    assert len(dp.buckets) > 1 and dp._native is not None
    x = torch.randn(32, 64, device=dev)

    def step():
        dp.zero_()
        dp(x).square().mean().backward()

    step()
    ref = [p.grad.clone() for p in net.parameters()]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        step()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    for p, r in zip(net.parameters(), ref):
        torch.testing.assert_close(p.grad, r)


def test_host_loader_cuda():
    from rocket_amd.runtime.host_data import HostLoader, HostTensorDataset

    x = torch.randn(1000, 3, 16, 16)
    y = torch.arange(1000)
    loader = HostLoader(HostTensorDataset(x, y), batch_size=100, shuffle=True, seed=2,
                        device=torch.device("cuda", 0))
    seen = []
    for bx, by in loader:
        assert bx.is_cuda and bx._rocket_persistent
        torch.testing.assert_close(bx.cpu(), x[by.cpu()])
        seen += by.tolist()
    assert sorted(seen) == list(range(1000))
