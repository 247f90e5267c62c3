"""Engine + data-path semantics on CPU: GA state machine, scheduler stepping, sharding oracles, collate/move."""

import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

import rocket_amd as rocket
from rocket_amd.core.capsule import Capsule
from rocket_amd.runtime.data import EpochSampler, num_batches, shard_batches
from rocket_amd.runtime.engine import Engine
from rocket_amd.utils.torch import torch_collate, torch_move


# ------------------------------------------------------------------ sharding
def _batches(n, bs):
    idx = list(range(n))
    return [idx[i : i + bs] for i in range(0, n, bs)]


def test_shard_oracle_wraparound():
    # verified on the reference (accelerate BatchSamplerShard): 40 samples, bs 6, W 2
    b = _batches(40, 6)
    r0 = shard_batches(b, 6, 2, 0, drop_last=False)
    r1 = shard_batches(b, 6, 2, 1, drop_last=False)
    assert len(r0) == len(r1) == 4
    assert r0[-1] == [36, 37, 38, 39, 0, 1]
    assert r1[-1] == [2, 3, 4, 5, 6, 7]


def test_shard_uneven_and_drop_last():
    b = _batches(10, 2)  # 5 batches
    assert shard_batches(b, 2, 2, 0, drop_last=False, even_batches=False) == [[0, 1], [4, 5], [8, 9]]
    assert shard_batches(b, 2, 2, 1, drop_last=False, even_batches=False) == [[2, 3], [6, 7]]
    assert shard_batches(b, 2, 2, 1, drop_last=True) == [[2, 3], [6, 7]]


@settings(max_examples=60, deadline=None)
@given(n=st.integers(1, 200), bs=st.integers(1, 17), W=st.integers(1, 8))
def test_shard_properties(n, bs, W):
    b = _batches(n, bs)
    shards = [shard_batches(b, bs, W, r, drop_last=False) for r in range(W)]
    lens = {len(s) for s in shards}
    assert len(lens) == 1  # even_batches: every rank the same number of batches
    assert lens.pop() == num_batches(n, bs, False, W)
    seen = {i for s in shards for batch in s for i in batch}
    assert seen == set(range(n))  # every sample is consumed
    if W > 1 and n >= bs * W:
        assert all(len(batch) == bs for s in shards for batch in s)  # padding makes full batches


def test_epoch_sampler_deterministic():
    a, b = EpochSampler(50, shuffle=True, seed=3), EpochSampler(50, shuffle=True, seed=3)
    a.set_epoch(2)
    b.set_epoch(2)
    assert list(a) == list(b)
    b.set_epoch(3)
    assert list(a) != list(b)
    assert sorted(a) == list(range(50))


# ------------------------------------------------------------ GA / scheduler
class _Probe(Capsule):
    def __init__(self, engine_box):
        super().__init__(priority=10)
        self.box = engine_box
        self.sync = []
        self.lrs = []

    def launch(self, attrs=None):
        self.sync.append(self._accelerator.sync_gradients)


def _ga_tree(n_batches, ga, epochs=1, lr=1.0):
    torch.manual_seed(0)
    data = [(torch.randn(3), torch.tensor(0)) for _ in range(n_batches)]
    net = torch.nn.Linear(3, 2)
    opt = torch.optim.SGD(net.parameters(), lr=lr)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: 1.0 / (1 + s))
    steps = []
    orig = opt.step

    def counting_step(*a, **k):
        steps.append(1)
        return orig(*a, **k)

    opt.step = counting_step

    class Obj(torch.nn.Module):
        def forward(self, batch):
            return torch.nn.functional.cross_entropy(batch[2], batch[1])

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = net

        def forward(self, batch):
            return (batch[0], batch[1], self.lin(batch[0]))

    probe = _Probe(None)
    tree = rocket.Launcher(
        [rocket.Looper([rocket.Dataset(data, batch_size=1),
                        rocket.Module(Net(), [rocket.Loss(Obj()), rocket.Optimizer(opt), rocket.Scheduler(sched)]),
                        probe], progress=False)],
        gradient_accumulation_steps=ga, num_epochs=epochs, cpu=True, destroy_process_group_after_launch=False,
    )
    return tree, probe, steps, sched


def test_ga_sync_pattern_and_forced_sync_at_epoch_end():
    tree, probe, steps, sched = _ga_tree(n_batches=7, ga=3)
    tree.launch()
    # sync on micro-steps 3, 6 and the last batch of the epoch (end_of_dataloader forces it)
    assert probe.sync == [False, False, True, False, False, True, True]
    assert len(steps) == 3
    # scheduler: one real step per sync, _step_count advanced on every micro-step
    assert sched.last_epoch == 3
    assert sched._step_count == 1 + 7


def test_ga_step_counter_resets_each_epoch():
    tree, probe, steps, _ = _ga_tree(n_batches=4, ga=3, epochs=2)
    tree.launch()
    assert probe.sync == [False, False, True, True] * 2


def test_loss_reports_ga_window_mean():
    vals = []

    class Rec(Capsule):
        def __init__(self):
            super().__init__(priority=10)

        def launch(self, attrs=None):
            if self._accelerator.sync_gradients:
                vals.append(float(attrs.looper.state.loss))

    losses = [1.0, 3.0, 5.0, 7.0]

    class Obj(torch.nn.Module):
        def forward(self, batch):
            return batch[1] * batch[0].sum() * 0 + batch[1]  # loss == the label value

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.ones(1))

        def forward(self, batch):
            x, y = batch
            return (x * self.w, y.float().sum())

    data = [(torch.ones(1), torch.tensor(v)) for v in losses]
    opt = torch.optim.SGD(Net().parameters(), lr=0.0)
    net = Net()
    opt = torch.optim.SGD(net.parameters(), lr=0.0)
    rocket.Launcher(
        [rocket.Looper([rocket.Dataset(data, batch_size=1), rocket.Module(net, [rocket.Loss(Obj()), rocket.Optimizer(opt)]),
                        Rec()], progress=False)],
        gradient_accumulation_steps=2, cpu=True, destroy_process_group_after_launch=False,
    ).launch()
    assert vals == [2.0, 6.0]


def test_engine_gather_for_metrics_single_process():
    e = Engine(cpu=True)
    t = torch.arange(5)
    assert torch.equal(e.gather_for_metrics(t), t)
    assert e.gather_for_metrics([1, 2]) == [1, 2]


def test_engine_flat_grads_zeroing():
    e = Engine(cpu=True, flat_grads=True)
    net = e.prepare_model(torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Linear(4, 2)))
    opt = e.prepare_optimizer(torch.optim.SGD(net.parameters(), lr=0.1))
    ptrs = [p.grad.data_ptr() for p in net.parameters()]
    net(torch.randn(3, 4)).sum().backward()
    assert all(p.grad.abs().sum() > 0 for p in net.parameters())
    assert [p.grad.data_ptr() for p in net.parameters()] == ptrs  # accumulated in place
    opt.step()
    opt.zero_grad()
    assert all(float(p.grad.abs().sum()) == 0 for p in net.parameters())
    assert [p.grad.data_ptr() for p in net.parameters()] == ptrs


# ------------------------------------------------------------- collate/move
def test_collate_keeps_builtin_leaves():
    batch = torch_collate([{"x": torch.ones(2), "name": "a", "n": 1}, {"x": torch.zeros(2), "name": "b", "n": 2}])
    assert batch["x"].shape == (2, 2)
    assert batch["name"] == ["a", "b"]
    assert batch["n"] == [1, 2]


def test_move_nested():
    out = torch_move({"a": [torch.ones(1), "s"], "b": (torch.zeros(1),)}, torch.device("cpu"))
    assert out["a"][1] == "s" and isinstance(out["b"], tuple)


def test_ga_oracle_from_survey():
    """SURVEY §2.4 verified oracle: 7 batches/epoch, GA=2, 2 epochs -> [0,1,0,1,0,1,1]*2, 8 updates."""
    tree, probe, steps, _ = _ga_tree(n_batches=7, ga=2, epochs=2)
    tree.launch()
    assert [int(s) for s in probe.sync] == [0, 1, 0, 1, 0, 1, 1] * 2
    assert len(steps) == 8


def test_pre_sharded_device_dataset_batches_all_local_samples():
    """A pre-sharded DeviceTensorDataset (this rank's samples only) is batched whole on every rank,
    not split again by rank."""
    from rocket_amd.runtime.data import DeviceLoader, DeviceTensorDataset

    x = torch.arange(40).float().reshape(40, 1)
    ds = DeviceTensorDataset(x, torch.arange(40), pre_sharded=True)
    for rank in (0, 1):
        dl = DeviceLoader(ds, batch_size=8, num_replicas=2, rank=rank, drop_last=True)
        seen = sorted(int(v) for b in dl for v in b[1])
        assert seen == list(range(40))
    glob = DeviceLoader(DeviceTensorDataset(x, torch.arange(40)), batch_size=8, num_replicas=2, rank=1)
    assert sum(len(b[1]) for b in glob) < 40
