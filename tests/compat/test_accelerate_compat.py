"""Checkpoint compatibility with HuggingFace ``accelerate`` (SURVEY §4 "Checkpoint compat",
Appendix C): accelerate is installed here as a test ORACLE only — rocket_amd never imports it.

* a checkpoint written by rocket_amd's Checkpointer loads with ``Accelerator.load_state`` and
  restores identical model / optimizer / scheduler state and RNG streams;
* a checkpoint written by ``Accelerator.save_state`` loads with rocket_amd's engine
  (``runtime.checkpoint_io.load_state``, weights_only loaders only).
"""

import os
import random

import numpy as np
import pytest
import torch

accelerate = pytest.importorskip("accelerate")

import rocket_amd as rocket  # noqa: E402
from rocket_amd.runtime import checkpoint_io  # noqa: E402
from rocket_amd.runtime.engine import Engine  # noqa: E402


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(4, 3)

    def forward(self, batch):
        return (batch[0], batch[1], self.lin(batch[0]))


class Objective(torch.nn.Module):
    def forward(self, batch):
        return torch.nn.functional.cross_entropy(batch[2], batch[1])


def _optim(net):
    opt = torch.optim.AdamW(net.parameters(), lr=0.05)
    return opt, torch.optim.lr_scheduler.StepLR(opt, 2, gamma=0.5)


def _rocket_run(tmp_path):
    torch.manual_seed(0)
    x, y = torch.randn(12, 4), torch.randint(0, 3, (12,))
    net = Net()
    opt, sched = _optim(net)
    rocket.Launcher([rocket.Looper([
        rocket.Dataset([(x[i], y[i]) for i in range(12)], batch_size=2),
        rocket.Module(net, [rocket.Loss(Objective()), rocket.Optimizer(opt), rocket.Scheduler(sched)]),
        rocket.Checkpointer(save_every=5),
    ], progress=False)], tag="c", logging_dir=str(tmp_path), cpu=True,
        destroy_process_group_after_launch=False).launch()
    return net, opt, sched, tmp_path / "c" / "v0" / "weights" / "004"


def _state_equal(a, b):
    if isinstance(a, torch.Tensor):
        return torch.equal(a.cpu(), b.cpu())
    if isinstance(a, dict):
        return a.keys() == b.keys() and all(_state_equal(a[k], b[k]) for k in a)
    if isinstance(a, (list, tuple)):
        return len(a) == len(b) and all(_state_equal(u, v) for u, v in zip(a, b))
    return a == b


@pytest.fixture
def fresh_accelerate_state():
    from accelerate.state import AcceleratorState, GradientState, PartialState

    yield
    AcceleratorState._reset_state(True)
    GradientState._reset_state()
    PartialState._reset_state()


def test_rocket_checkpoint_loads_in_accelerate(tmp_path, fresh_accelerate_state):
    net, opt, sched, ck = _rocket_run(tmp_path)
    assert (ck / "model.safetensors").exists()
    # RNG streams right after the checkpoint's RNG snapshot was restored by rocket_amd itself
    acc = accelerate.Accelerator(cpu=True)
    torch.manual_seed(123)
    net2 = Net()
    opt2, sched2 = _optim(net2)
    net2, opt2, sched2 = acc.prepare(net2, opt2, sched2)

    class Slot:  # stands in for a stateful capsule (Launcher, Looper, Dataset, Loss...)
        def __init__(self):
            self.sd = None

        def state_dict(self):
            return {}

        def load_state_dict(self, sd):
            self.sd = sd

    n_custom = len([f for f in os.listdir(ck) if f.startswith("custom_checkpoint_")])
    slots = [Slot() for _ in range(n_custom)]
    acc.register_for_checkpointing(*slots)
    acc.load_state(str(ck))
    assert all(isinstance(s.sd, dict) for s in slots)
    assert "iter_idx" in slots[0].sd  # registration order: Looper, Dataset, Loss (Launcher not statefull)
    for a, b in zip(net.parameters(), acc.unwrap_model(net2).parameters()):
        assert not torch.equal(a, torch.zeros_like(a))
    saved = checkpoint_io._load(ck / "optimizer.bin")
    assert _state_equal(opt2.optimizer.state_dict()["state"], saved["state"])
    assert sched2.scheduler.last_epoch == checkpoint_io._load(ck / "scheduler.bin")["last_epoch"]
    sd = acc.unwrap_model(net2).state_dict()
    from safetensors.torch import load_file

    ref = load_file(str(ck / "model.safetensors"))
    assert sd.keys() == ref.keys() and all(torch.equal(sd[k], ref[k]) for k in sd)
    # accelerate restored rocket_amd's RNG snapshot: same torch / numpy / python streams
    t_acc, n_acc, r_acc = torch.rand(3), np.random.rand(3), random.random()
    eng = Engine(cpu=True)
    eng.prepare(Net())
    checkpoint_io.load_state(eng, str(ck), load_custom=False)
    assert torch.equal(t_acc, torch.rand(3)) and np.array_equal(n_acc, np.random.rand(3)) and r_acc == random.random()


def test_accelerate_checkpoint_loads_in_rocket(tmp_path, fresh_accelerate_state):
    acc = accelerate.Accelerator(cpu=True)
    torch.manual_seed(7)
    net = Net()
    opt, sched = _optim(net)
    net, opt, sched = acc.prepare(net, opt, sched)
    x, y = torch.randn(8, 4), torch.randint(0, 3, (8,))
    for i in range(3):
        loss = Objective()(net((x, y)))
        acc.backward(loss)
        opt.step()
        sched.step()
        opt.zero_grad()
    out = tmp_path / "acc_ckpt"
    acc.save_state(str(out))
    t_ref, n_ref = torch.rand(4), np.random.rand(4)

    torch.manual_seed(99)
    eng = Engine(cpu=True)
    net2 = Net()
    opt2, sched2 = _optim(net2)
    net2, opt2, sched2 = eng.prepare(net2, opt2, sched2)
    checkpoint_io.load_state(eng, str(out), load_custom=False)
    for a, b in zip(acc.unwrap_model(net).parameters(), eng.unwrap_model(net2).parameters()):
        assert torch.equal(a, b)
    assert _state_equal(opt.optimizer.state_dict()["state"], opt2.state_dict()["state"])
    assert sched2.state_dict()["last_epoch"] == sched.scheduler.last_epoch
    assert torch.equal(t_ref, torch.rand(4)) and np.array_equal(n_ref, np.random.rand(4))
