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
