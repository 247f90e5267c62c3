"""Tracker buffering/flush to the JSONL backend; Meter + Metric on CPU; Looper termination."""

import json
import os

import torch

import rocket_amd as rocket


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(4, 3)

    def forward(self, b):
        return (b[0], b[1], self.lin(b[0]))


class _Obj(torch.nn.Module):
    def forward(self, b):
        return torch.nn.functional.cross_entropy(b[2], b[1])


class _Acc(rocket.Metric):
    def __init__(self):
        super().__init__()
        self.hits = self.total = 0
        self.history = []

    def launch(self, attrs=None):
        self.hits += int((attrs.batch[2].argmax(1) == attrs.batch[1]).sum())
        self.total += attrs.batch[1].numel()
        attrs.looper.state.acc = self.hits / self.total
        attrs.tracker.scalars.append(rocket.Attributes(step=self._step, data={"acc": attrs.looper.state.acc}))

    def reset(self, attrs=None):
        self.history.append(self.total)
        self.hits = self.total = 0


def test_tracker_jsonl_and_meter(tmp_path):
    torch.manual_seed(0)
    data = [(torch.randn(4), torch.tensor(i % 3)) for i in range(24)]
    net = _Net()
    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    acc = _Acc()
    rocket.Launcher(
        [
            rocket.Looper([rocket.Dataset(data, batch_size=4),
                           rocket.Module(net, [rocket.Loss(_Obj()), rocket.Optimizer(opt)]),
                           rocket.Tracker(backend="jsonl", flush_every=2)], tag="train", progress=False),
            # a distinct dataset object: the same object would resolve to the train loader (reference dedupe)
            rocket.Looper([rocket.Dataset(list(data), batch_size=6), rocket.Module(net), rocket.Meter([acc], keys=[1, 2]),
                           rocket.Tracker(backend="jsonl")], tag="eval", grad_enabled=False, progress=False),
        ],
        tag="exp", logging_dir=str(tmp_path), num_epochs=2, cpu=True, destroy_process_group_after_launch=False,
    ).launch()
    recs = [json.loads(l) for l in open(tmp_path / "exp" / "v0" / "metrics.jsonl")]
    losses = [r for r in recs if "train_loss" in r]
    lrs = [r for r in recs if "opt.lr.0" in r]
    accs = [r for r in recs if "acc" in r]
    assert [r["step"] for r in losses] == list(range(12))  # 6 steps x 2 epochs, in order
    assert len(lrs) == 12 and all(abs(r["opt.lr.0"] - 0.1) < 1e-9 for r in lrs)
    assert len(accs) == 8 and {r["step"] for r in accs} == {0, 1}  # Metric._step = epoch
    assert acc.history == [24, 24]  # every sample seen once per eval epoch
    assert all(isinstance(r["train_loss"], float) for r in losses)


def test_looper_terminates_when_dataset_exhausted(tmp_path):
    seen = []

    class Probe(rocket.Capsule):
        def launch(self, attrs=None):
            if attrs.batch is not None:
                seen.append(1)

    data = [(torch.randn(4), torch.tensor(0)) for _ in range(10)]
    rocket.Launcher([rocket.Looper([rocket.Dataset(data, batch_size=4), Probe()], repeats=100, progress=False)],
                    cpu=True, destroy_process_group_after_launch=False).launch()
    assert len(seen) == 3  # 10 samples / bs 4 -> 3 batches, then terminate
