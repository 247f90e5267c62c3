"""Device loader on the GPU: batches gathered one ahead with the AQL barrier bit clear
(``rk_gather_rows_any_order``) hold exactly the sampled rows, across epochs, while the queue is
kept busy by long kernels that read the previous batch (a gather that overtook a reader of its ring
slot, or the index-table upload it depends on, would show up as a mismatch)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("any_order", [True, False])
def test_any_order_gather_batches_exact(monkeypatch, any_order):
    from rocket_amd.ops import _lib
    from rocket_amd.runtime.data import DeviceLoader, DeviceTensorDataset

    monkeypatch.setattr(DeviceLoader, "ANY_ORDER", any_order)
    dev = torch.device("cuda", 0)
    n, bs = 4096, 256
    x = torch.randn(n, 1, 28, 28, device=dev)
    y = torch.arange(n, device=dev)
    dl = DeviceLoader(DeviceTensorDataset(x, y), batch_size=bs, shuffle=True, drop_last=True, seed=3)
    lib = _lib.kernels()
    sink = torch.zeros(64, device=dev)
    for epoch in range(2):
        dl.set_epoch(epoch)
        order = [i for b in dl.batch_sampler.local_batches() for i in b]
        got = []
        for j, (xb, yb) in enumerate(dl):
            lib.rk_spin(20.0, 4, sink.data_ptr(), _lib.stream_ptr(dev))  # keep the queue ahead of the GPU
            got.append((xb.sum((1, 2, 3)).clone(), yb.clone()))  # read the slot before it is reused
        idx = torch.tensor(order, device=dev)
        ys = torch.cat([g[1] for g in got])
        xs = torch.cat([g[0] for g in got])
        torch.cuda.synchronize()
        assert torch.equal(ys, y[idx]), epoch
        torch.testing.assert_close(xs, x[idx].sum((1, 2, 3)))


def test_deferred_batches_materialize_exact():
    """Deferred mode without a claiming consumer: every batch gathered through the device-side
    cursor (``rk_gather_rows_cursor``) on first read holds the sampled rows, across epochs; a batch
    nobody read is gathered before the next one, so the cursor stays in step."""
    from rocket_amd.runtime.data import DeviceLoader, DeviceTensorDataset, materialize_batch, pending_rows

    dev = torch.device("cuda", 0)
    n, bs = 2048, 128
    x = torch.randn(n, 1, 28, 28, device=dev)
    y = torch.arange(n, device=dev)
    dl = DeviceLoader(DeviceTensorDataset(x, y), batch_size=bs, shuffle=True, drop_last=True, seed=9)
    dl.defer = True
    for epoch in range(2):
        dl.set_epoch(epoch)
        order = torch.tensor([i for b in dl.batch_sampler.local_batches() for i in b], device=dev)
        for j, batch in enumerate(dl):
            assert pending_rows(batch) is not None
            if j % 3 == 2:
                continue  # skipped: the loader gathers it before handing out the next batch
            materialize_batch(batch)
            xb, yb = batch
            torch.cuda.synchronize()
            assert torch.equal(yb, y[order[j * bs:(j + 1) * bs]]), (epoch, j)
            assert torch.equal(xb, x[order[j * bs:(j + 1) * bs]])


@pytest.mark.parametrize("capture", [True, False])
def test_lenet_gathers_its_deferred_batches(monkeypatch, capture, tmp_path):
    """The fused LeNet step kernel gathering its own batches (deferred loader, device cursor, graph
    replays) trains exactly like the loader-gathered run: identical losses and weights."""
    import rocket_amd as rocket
    from rocket_amd.models import CrossEntropy, LeNet
    from rocket_amd.ops.optim import FusedAdamW
    from rocket_amd.runtime.data import DeviceLoader

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    data = (torch.rand(2048, 1, 28, 28, generator=g, device=dev), torch.randint(0, 10, (2048,), generator=g, device=dev))
    runs = []
    for defer in (True, False):
        monkeypatch.setattr(DeviceLoader, "DEFER", defer)
        torch.manual_seed(0)
        net = LeNet()
        losses = []

        class Rec(rocket.Capsule):
            def launch(self, attrs=None):
                if attrs is not None and attrs.looper is not None and "loss" in attrs.looper.state:
                    losses.append(attrs.looper.state.loss)

        caps = [rocket.Dataset(rocket.DeviceTensorDataset(*data), batch_size=256, shuffle=True),
                rocket.Module(net, [rocket.Loss(CrossEntropy()), rocket.Optimizer(FusedAdamW(net.parameters(), lr=1e-3))],
                              capture=capture, warmup=1), Rec(priority=10)]
        rocket.Launcher([rocket.Looper(caps, progress=False)], tag="gpu", logging_dir=str(tmp_path / str(defer)),
                        num_epochs=2, mixed_precision="bf16", destroy_process_group_after_launch=False).launch()
        torch.cuda.synchronize()
        runs.append(([float(v) for v in losses], [p.detach().clone() for p in net.parameters()]))
    (l1, p1), (l2, p2) = runs
    assert len(l1) == len(l2) == 16 and l1 == l2, (l1, l2)
    for a, b in zip(p1, p2):
        assert torch.equal(a, b)
