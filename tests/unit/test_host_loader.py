"""Native host batch assembler (C++ thread pool) + HostLoader semantics on CPU."""

import pytest
import torch

import rocket_amd as rocket
from rocket_amd.runtime.data import DeviceLoader, DeviceTensorDataset
from rocket_amd.runtime.host_data import HostLoader, HostTensorDataset


def _data(n=1000):
    g = torch.Generator().manual_seed(0)
    return torch.randn(n, 3, 8, 8, generator=g), torch.arange(n), torch.randint(0, 255, (n, 5), generator=g).to(torch.uint8)


@pytest.mark.parametrize("shuffle", [False, True])
def test_host_loader_rows_and_order_match_device_loader(shuffle):
    x, y, z = _data()
    h = HostLoader(HostTensorDataset(x, y, z), batch_size=64, shuffle=shuffle, seed=5, num_threads=4)
    d = DeviceLoader(DeviceTensorDataset(x, y, z), batch_size=64, shuffle=shuffle, seed=5)
    hb, db = list(h), list(d)
    assert len(hb) == len(db) == 16
    for (hx, hy, hz), (dx, dy, dz) in zip(hb, db):
        assert torch.equal(hy, dy) and torch.equal(hx, x[hy]) and torch.equal(hz, z[hy])


def test_host_loader_sharding_skip_and_epochs():
    x, y, _ = _data(100)
    ds = HostTensorDataset(x, y)
    r0 = [b[1].tolist() for b in HostLoader(ds, batch_size=8, num_replicas=2, rank=0)]
    r1 = [b[1].tolist() for b in HostLoader(ds, batch_size=8, num_replicas=2, rank=1)]
    assert len(r0) == len(r1) == 7  # 13 batches -> even_batches pads to 14
    assert {i for b in r0 + r1 for i in b} == set(range(100))
    sk = HostLoader(ds, batch_size=8, num_replicas=2, rank=0).with_skip(3)
    assert [b[1].tolist() for b in sk] == r0[3:]
    loader = HostLoader(ds, batch_size=10, shuffle=True, seed=1)
    e0 = [b[1].tolist() for b in loader]
    e1 = [b[1].tolist() for b in loader]
    assert e0 != e1 and sorted(sum(e0, [])) == sorted(sum(e1, [])) == list(range(100))


def test_host_loader_early_break_and_reuse():
    x, y, _ = _data(500)
    loader = HostLoader(HostTensorDataset(x, y), batch_size=16, num_threads=3)
    for i, _ in enumerate(loader):
        if i == 2:
            break
    full = [b[1] for b in loader]
    assert torch.equal(torch.cat(full), torch.arange(500))


def test_launcher_with_host_dataset(tmp_path):
    x = torch.randn(64, 4)
    y = torch.randint(0, 3, (64,))
    net = torch.nn.Linear(4, 3)

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = net

        def forward(self, b):
            return (self.lin(b[0]), b[1])

    class Obj(torch.nn.Module):
        def forward(self, b):
            return torch.nn.functional.cross_entropy(b[0], b[1])

    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    w0 = net.weight.detach().clone()
    rocket.Launcher([rocket.Looper([rocket.Dataset(rocket.HostTensorDataset(x, y), batch_size=8),
                                    rocket.Module(Net(), [rocket.Loss(Obj()), rocket.Optimizer(opt)])],
                                   progress=False)],
                    cpu=True, num_epochs=2, destroy_process_group_after_launch=False).launch()
    assert not torch.equal(w0, net.weight.detach())
